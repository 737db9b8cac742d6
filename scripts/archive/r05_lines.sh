#!/bin/bash
# Round 5: the other bench lines on the final tree (config 3, config 5 map, single-stream latency,
# PointCloud2 ingest inside the timed region).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r05lines}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python bench.py --lines 128 --width 2048 --batch 100 --cpu-budget 0 > $D/bench_config3.json 2> $D/config3.err || exit 1
timeout -k 10 300 python bench.py --workload map --cpu-budget 0 > $D/bench_config5_map.json 2> $D/map.err || exit 2
timeout -k 10 300 python bench.py --workload latency --cpu-budget 0 > $D/bench_latency.json 2> $D/latency.err || exit 3
timeout -k 10 300 python bench.py --workload ingest --cpu-budget 0 > $D/bench_ingest.json 2> $D/ingest.err || exit 4
for f in $D/bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['unit'], d.get('ms_per_step'), (d.get('pose_delta_vs_cpu') or {}).get('max_abs_pose') if isinstance(d.get('pose_delta_vs_cpu'), dict) else None, d.get('engine_aborts'))"; done
