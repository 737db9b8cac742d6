#!/bin/bash
# Round 5, final tree on one GPU box: the whole -m gpu suite, smoke(), the default bench line and
# the config-5 map line (each step under its own time limit; the first failure ends the call).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r05final}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { tail -20 $D/smoke.txt; exit 2; }
tail -2 $D/smoke.txt
timeout -k 10 500 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 3; }
head -c 400 $D/bench.json; echo
timeout -k 10 300 python -u bench.py --workload map > $D/bench_config5_map.json 2> $D/map.err || { tail -20 $D/map.err; exit 4; }
head -c 300 $D/bench_config5_map.json; echo
echo done > $D/DONE
