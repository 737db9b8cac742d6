#!/bin/bash
# Round-6 closing measurements on the final tree: two more driver-shape lines (config 2), config 3
# (128x2048, 100-scan chain) and config 5 (map workload).  Usage (GPU box): bash scripts/r06_final_lines.sh <tag>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06final}
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/c2_$r.json 2> $OUT/c2_$r.err || { tail -20 $OUT/c2_$r.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --lines 128 --width 2048 --batch 100 --steps 20 --warmup 3 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 2; }
timeout -k 10 300 python3 bench.py --workload map --steps 60 --warmup 3 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 3; }
for f in c2_1 c2_2 c3 c5; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['unit'], d['ms_per_step'], d.get('sustained', {}).get('value'), (d.get('pose_delta_vs_cpu') or {}).get('max_abs_pose'))"; done
echo done > $OUT/ALL_DONE
