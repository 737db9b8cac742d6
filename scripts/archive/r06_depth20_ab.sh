#!/bin/bash
# Round-6 A/B at the driver's own shape (--steps 20 --warmup 5): contexts x engine depth at qpw 3,
# alternating variants on one box.  Usage (GPU box): bash scripts/archive/r06_depth20_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06e}
REPS=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, contexts, env...
  local name=$1; local k=$2; shift; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 0 --contexts $k --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['config']['masked_queues']['timed'], d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run c6d4_$i 6
  run c8d6_$i 8 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=6
  run c8d5_$i 8 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
  run c7d5_$i 7 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
  run c10d6_$i 10 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=6
  run c5d5_$i 5 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
done
echo done > $OUT/ALL_DONE
