#!/bin/bash
# Round-6 A/B: batches per pipelined context (bench.py --batches-per-context; 1 = round 5's one batch
# per context) x contexts, at the driver's shape, alternating.  Usage (GPU box): bash scripts/archive/r06_bpc_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06m}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['config']['masked_queues']['timed'], d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run c8b1_$i --contexts 8 --batches-per-context 1
  run c8b2_$i --contexts 8 --batches-per-context 2
  run c6b2_$i --contexts 6 --batches-per-context 2
  run c8b3_$i --contexts 8 --batches-per-context 3
  run c5b2_$i --contexts 5 --batches-per-context 2
done
echo done > $OUT/ALL_DONE
