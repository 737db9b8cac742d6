#!/bin/bash
# Round-6: device timelines (LISLAM_TIMELINE=1) of the bench at the driver's shape for the role-CU /
# work-mask variants, summarised by scripts/timeline_summary.py.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06ac}
mkdir -p $OUT
export TMPDIR=/tmp
for v in "one_d5 LISLAM_ROLE_CUS=1" "se_d5" "se_d4 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=4" "se_d4_w LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=4 LISLAM_WORK_SE0=0" "se_d5_w LISLAM_WORK_SE0=0"; do
  set -- $v; name=$1; shift
  env LISLAM_TIMELINE=1 "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['single_sequence']['value'], d['roofline']['self_check'].get('pipelined_ms_per_launch'))"
  python scripts/timeline_summary.py $OUT/$name.err
done
