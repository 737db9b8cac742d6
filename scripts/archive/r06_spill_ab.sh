#!/bin/bash
# Round-6 A/B of the association items' register diet (x and the seeds read from LDS, the share
# emitted sum by sum into the row): the chain / pipelined tests, then bench lines alternating the
# new library with HEAD's (scripts/_ab/liblislam_head.so), then the single-launch engine's FETCH /
# WRITE counters for both.  Usage (GPU box): bash scripts/archive/r06_spill_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06s}
REPS=${2:-3}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 2; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run new_$i
  run head_$i LISLAM_ALT_LIB=$ROOT/scripts/_ab/liblislam_head.so
done
cd /tmp
export LISLAM_ENGINE_SINGLE=1
for v in new head; do
  if [ $v = head ]; then export LISLAM_ALT_LIB=$ROOT/scripts/_ab/liblislam_head.so; fi
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/$OUT/pmc_fetch_$v -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $ROOT/$OUT/fetch_$v.json 2> $ROOT/$OUT/fetch_$v.err || exit 3
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/$OUT/pmc_write_$v -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $ROOT/$OUT/write_$v.json 2> $ROOT/$OUT/write_$v.err || exit 4
done
echo done > $ROOT/$OUT/ALL_DONE
