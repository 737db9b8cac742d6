#!/bin/bash
# Round-6 probe: the driver-shape bench with and without the ORB front end (timelines), to see
# whether ORB sets each context's period.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06aj}
mkdir -p $OUT
export TMPDIR=/tmp
for v in "orb" "noorb --no-orb"; do
  set -- $v; name=$1; shift
  LISLAM_TIMELINE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['sustained']['value'])"
  python scripts/timeline_summary.py $OUT/$name.err
done
