#!/bin/bash
# Round-6 A/B at the driver's shape under the SE layout: throughput shape (3, 5) vs (4, 5) (four
# queries per wave on 16-lane rows, 4-wave items: 576 item waves per engine instead of 768).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06ai}
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for i in 1 2; do
for v in "q3_$i" "q4_$i LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_DEPTH=5" "q4d6_$i LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_DEPTH=6"; do
  set -- $v; name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'], d['config']['masked_queues']['timed'])"
done
done
