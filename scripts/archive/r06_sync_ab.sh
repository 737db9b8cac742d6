#!/bin/bash
# Round-6 A/B of the per-XCD x copies (items poll and read their XCD's copy of the chain's x) with
# the register diet, against HEAD's library: chain / pipelined tests, the stand-in engine's kernel
# time and counters on 8 and 1 XCDs, bench lines alternating.  Usage (GPU box): bash scripts/archive/r06_sync_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06y}
REPS=${2:-3}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
HEADLIB=$ROOT/scripts/_ab/liblislam_head.so
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run new_$i
  run head_$i LISLAM_ALT_LIB=$HEADLIB
done
cd /tmp
for v in new head; do
  for n in 8 1; do
    if [ $v = head ]; then export LISLAM_ALT_LIB=$HEADLIB; else unset LISLAM_ALT_LIB; fi
    LISLAM_ENGINE_SINGLE=1 LISLAM_WORK_XCDS=$n timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_$n -o trace -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/trace_${v}_$n.json 2> $OUT/trace_${v}_$n.err || exit 3
    LISLAM_ENGINE_SINGLE=1 LISLAM_WORK_XCDS=$n timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_${v}_$n -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/fetch_${v}_$n.json 2> $OUT/fetch_${v}_$n.err || exit 4
  done
done
echo done > $OUT/ALL_DONE
