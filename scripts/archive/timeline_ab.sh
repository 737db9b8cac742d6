#!/bin/bash
# Device timelines of the pipelined bench (LISLAM_TIMELINE=1, LISLAM_BENCH_HOSTLOG=1) under several
# environment settings ("NAME=V,NAME2=V2" each): stderr kept for scripts/timeline.py.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-tl}
shift
mkdir -p $D
: > $D/steps.txt
for v in "$@"; do
  n=${v//,/_}; n=${n//\//_}
  BENCH_ARGS=""
  case "$v" in *CTX=*) c=${v##*CTX=}; c=${c%%,*}; BENCH_ARGS="--contexts $c";; esac
  ( for e in ${v//,/ }; do export "$e"; done
    LISLAM_TIMELINE=1 LISLAM_BENCH_HOSTLOG=1 timeout -k 10 300 python bench.py --steps ${TL_STEPS:-6} --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 --scan-cache /tmp/lislam_scans $BENCH_ARGS > $D/b_$n.json 2> $D/b_$n.err ) || { echo "$v failed" >> $D/steps.txt; cat $D/steps.txt; exit 3; }
  python3 -c "import json; d=json.load(open('$D/b_$n.json')); print('$v', d['value'], d['ms_per_step'], d['engine_aborts'])" >> $D/steps.txt
done
cat $D/steps.txt
