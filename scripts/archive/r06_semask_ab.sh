#!/bin/bash
# Round-6 A/B at the driver's shape: role CUs as two CUs of SE 0 per XCD (default) at engine depth 5
# and 4, vs one role CU per XCD (LISLAM_ROLE_CUS=1, the round-6 start) at depth 5, alternating, after
# the chain / pipelined tests.  Usage (GPU box): bash scripts/archive/r06_semask_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06ab}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -1 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'], d['config']['masked_queues'])"
}
for i in $(seq 1 $REPS); do
  run se_d5_$i
  run se_d4_$i LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=4
  run one_d5_$i LISLAM_ROLE_CUS=1
done
echo done > $OUT/ALL_DONE
