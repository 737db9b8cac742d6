#!/bin/bash
# Round-6 A/B at the driver's shape with the work streams on shader engines 1-3 (default): engine depth
# 5 vs 4, and the round-6-start layout (one role CU per XCD, work streams on SE 0 too), alternating,
# after the whole GPU suite.  Usage (GPU box): bash scripts/archive/r06_semask_ab2.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06ad}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 2; }
tail -1 $OUT/gpu_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'], d['config']['masked_queues']['timed'])"
}
for i in $(seq 1 $REPS); do
  run d5_$i
  run d4_$i LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=4
  run old_$i LISLAM_ROLE_CUS=1 LISLAM_WORK_SE0=1
done
echo done > $OUT/ALL_DONE
