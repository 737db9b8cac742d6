#!/bin/bash
# Round-6 A/B of the XCD-partitioned engine streams at the throughput shape (bench.py default
# schedule, 60 timed steps, no CPU leg), alternating variants on one box, after the pipelined
# and chain GPU tests.  Usage (GPU box): bash scripts/archive/r06_partition_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06p}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline_timed.py tests/test_gpu_chain.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --cpu-budget 0 --segmented 0 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['config']['masked_queues']['timed'], d['engine_aborts'], {k: round(v, 2) for k, v in r['kernel_ms_per_step'].items() if v > 0.5})"
}
for i in $(seq 1 $REPS); do
  run part24_$i LISLAM_ENGINE_PARTITION=1
  run full_$i LISLAM_ENGINE_PARTITION=0
  run part20_$i LISLAM_ENGINE_ITEM_CUS=20
  run part28_$i LISLAM_ENGINE_ITEM_CUS=28
  run part24pf_$i LISLAM_ENGINE_PREFETCH=1
done
echo done > $OUT/ALL_DONE
