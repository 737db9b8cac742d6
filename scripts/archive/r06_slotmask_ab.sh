#!/bin/bash
# Round-6 A/B at the driver's shape: slots 4-5 leave SE 0 to the first four slots' items (default) at
# depth 5 and 4, vs every slot's items on SE 0 (LISLAM_ITEMS_SE0=2), alternating, after the chain tests.
# Usage (GPU box): bash scripts/archive/r06_slotmask_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06af}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 2; }
tail -1 $OUT/gpu_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'], d['config']['masked_queues']['timed'])"
}
for i in $(seq 1 $REPS); do
  run d5_$i
  run d4_$i LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=4
  run se0all_$i LISLAM_ITEMS_SE0=2
done
echo done > $OUT/ALL_DONE
