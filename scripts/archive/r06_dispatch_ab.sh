#!/bin/bash
# Round-6 A/B of the engine dispatcher (LISLAM_ENGINE_DISPATCH=1: a host thread launches each chain on
# the first free engine slot once its inputs exist; 0: launch n waits for launch n - depth on the
# device), after the chain / pipelined tests, at the driver's shape, alternating.
# Usage (GPU box): bash scripts/archive/r06_dispatch_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06q}
REPS=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run disp_$i LISLAM_ENGINE_DISPATCH=1
  run gate_$i LISLAM_ENGINE_DISPATCH=0
done
LISLAM_TIMELINE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/tl.json 2> $OUT/tl.err || exit 3
echo done > $OUT/ALL_DONE
