#!/bin/bash
# Round-6 A/B: pipelined contexts x engine depth at qpw 3 (bench.py's schedule, 60 timed steps,
# no CPU leg), alternating variants on one box; then the pipelined tests at depth 6.
# Usage (GPU box): bash scripts/archive/r06_depth_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06d}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, contexts, env...
  local name=$1; local k=$2; shift; shift
  env "$@" timeout -k 10 300 python bench.py --cpu-budget 0 --segmented 0 --contexts $k --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['config']['masked_queues'], d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run c6d4_$i 6
  run c7d5_$i 7 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
  run c8d6_$i 8 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=6
  run c7d4_$i 7
  run c8d5_$i 8 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
  run c6d5_$i 6 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5
done
echo done > $OUT/ALL_DONE
