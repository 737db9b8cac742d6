#!/bin/bash
# Round-6 GPU check: the GPU suite, then the profile of the stream workload (bench line + rocprof
# kernel trace + PMC passes, scripts/profile_round.sh), then an A/B bench of the ORB stream choice.
# Usage (on the GPU box): bash scripts/archive/r06_check.sh <tag> [skip-tests]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
bash scripts/profile_round.sh $TAG || exit $?
( while sleep 30; do date >> $OUT/heartbeat2; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
LISLAM_ORB_SIDE_STREAM=1 timeout -k 10 300 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans > $OUT/bench_orbside.json 2> $OUT/bench_orbside.err || exit 7
timeout -k 10 300 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans > $OUT/bench_ctx.json 2> $OUT/bench_ctx.err || exit 8
echo done > $OUT/ALL_DONE
