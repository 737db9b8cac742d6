#!/bin/bash
# Config-5 map bench under several environment settings ("NAME=V,NAME2=V2" each; "DEF" = none),
# alternating, after the map parity tests.  Usage (GPU box): bash scripts/archive/map_ab.sh <tag> [NOTEST] setting...
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-mapab}
shift
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$1" = NOTEST ]; then
  shift
else
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_map.py tests/test_gpu_cubemap.py > $D/tests.txt 2>&1 || { tail -30 $D/tests.txt; exit 2; }
  tail -2 $D/tests.txt
fi
: > $D/lines.txt
for v in "$@"; do
  n=${v//,/_}; n=${n//\//_}
  ( [ "$v" = DEF ] || for e in ${v//,/ }; do export "$e"; done
    timeout -k 10 300 python bench.py --workload map --cpu-budget 0 > $D/map_$n.json 2> $D/map_$n.err ) || exit 3
  python3 -c "import json; d=json.load(open('$D/map_$n.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel_ms_per_step'], d['pose_delta_vs_cpu'])" >> $D/lines.txt
done
cat $D/lines.txt
