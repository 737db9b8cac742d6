#!/bin/bash
# Round-6: the driver's exact bench command (CPU baseline + segmented leg included) vs the A/B shape
# (--cpu-budget 0 --segmented 0), alternating on one box, after the ORB tests.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06am}
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv_$i.json 2> $OUT/drv_$i.err || { tail -5 $OUT/drv_$i.err; exit 2; }
  python -c "import json; d=json.load(open('$OUT/drv_$i.json')); print('drv_$i', d['value'], d['sustained']['value'], d['single_sequence']['value'])"
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { tail -5 $OUT/ab_$i.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/ab_$i.json')); print('ab_$i', d['value'], d['sustained']['value'], d['single_sequence']['value'])"
done
