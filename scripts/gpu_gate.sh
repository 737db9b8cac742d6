#!/bin/bash
# Round-6 checkpoint on the GPU box: the whole GPU suite, smoke, then the driver's bench command.
# Usage (GPU box): bash scripts/gpu_gate.sh <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-r06g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 2; }
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['self_check'], d['pose_delta_vs_cpu']['max_abs_pose'], d['pose_delta_vs_cpu']['pairs_compared'], d['engine_aborts'], d['config']['masked_queues'])"
echo done > $OUT/ALL_DONE
