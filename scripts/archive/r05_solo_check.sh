#!/bin/bash
# Round 5: the whole -m gpu suite with the solo item build as the default, then the single-stream
# latency workload with and without it (alternating).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r05solochk}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
for v in DEF LISLAM_ENGINE_SOLO_ITEMS=0 DEF2 LISLAM_ENGINE_SOLO_ITEMS=0; do
  ( case $v in LISLAM*) export $v;; esac
    timeout -k 10 300 python -u bench.py --workload latency --cpu-budget 0 > $D/lat_$v.json 2> $D/lat_$v.err ) || exit 3
  python3 -c "import json; d=json.load(open('$D/lat_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
