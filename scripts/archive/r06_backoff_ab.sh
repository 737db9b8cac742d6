#!/bin/bash
# Round-6 A/B of eng_wait's poll backoff (LISLAM_ENGINE_BACKOFF = longest sleep between polls in
# units of 64 cycles; 1 = the fixed 64 of round 5): polls counted (developer build), bench lines at
# the driver's shape alternating, the single-launch engine's FETCH / WRITE.
# Usage (GPU box): bash scripts/archive/r06_backoff_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06b}
REPS=${2:-2}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for bo in 1 8 32; do
  LISLAM_ENGINE_BACKOFF=$bo LISLAM_ALT_LIB=$ROOT/scripts/_ab/liblislam_prof.so timeout -k 10 200 python scripts/engine_polls.py latency > $OUT/polls_lat_$bo.json 2>/dev/null || exit 2
  LISLAM_ENGINE_BACKOFF=$bo LISLAM_ALT_LIB=$ROOT/scripts/_ab/liblislam_prof.so timeout -k 10 200 python scripts/engine_polls.py throughput > $OUT/polls_thr_$bo.json 2>/dev/null || exit 2
  python -c "import json; [print('$bo', d['shape'], d['load_bytes_total'], {k: v['polls'] for k, v in d['waits'].items()}) for d in (json.load(open('$OUT/polls_lat_$bo.json')), json.load(open('$OUT/polls_thr_$bo.json')))]"
done
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  for bo in 1 8 32; do run bo${bo}_$i LISLAM_ENGINE_BACKOFF=$bo; done
done
cd /tmp
for bo in 1 8 32; do
  LISLAM_ENGINE_BACKOFF=$bo LISLAM_ENGINE_SINGLE=1 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$bo -o trace -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/trace_$bo.json 2> $OUT/trace_$bo.err || exit 4
  LISLAM_ENGINE_BACKOFF=$bo LISLAM_ENGINE_SINGLE=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$bo -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/fetch_$bo.json 2> $OUT/fetch_$bo.err || exit 5
  LISLAM_ENGINE_BACKOFF=$bo LISLAM_ENGINE_SINGLE=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$bo -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/write_$bo.json 2> $OUT/write_$bo.err || exit 6
done
echo done > $OUT/ALL_DONE
