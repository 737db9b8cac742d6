#!/bin/bash
# Round-6 A/B at the driver's shape: contexts x batches per context, with the ORB front end on the
# context stream (default) or a private side stream (LISLAM_ORB_SIDE_STREAM=1).
# Usage (GPU box): bash scripts/archive/r06_ctxmix_ab.sh <tag>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06ah}
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in "c8b1 --contexts 8" "c4b2s --contexts 4 --batches-per-context 2 LISLAM_ORB_SIDE_STREAM=1" "c6b2s --contexts 6 --batches-per-context 2 LISLAM_ORB_SIDE_STREAM=1" "c8b1s --contexts 8 LISLAM_ORB_SIDE_STREAM=1" "c4b2 --contexts 4 --batches-per-context 2"; do
  set -- $v; name=$1; shift
  args=""; envs=""
  for x in "$@"; do case $x in LISLAM_*) envs="$envs $x";; *) args="$args $x";; esac; done
  env $envs LISLAM_TIMELINE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans $args > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['sustained']['value'], d['config']['masked_queues']['timed'])"
  python scripts/timeline_summary.py $OUT/$name.err
done
