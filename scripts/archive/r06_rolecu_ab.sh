#!/bin/bash
# Round-6 A/B of two role CUs per XCD with one solve role per XCD (default) vs one role CU per XCD
# (LISLAM_ROLE_CUS=1): engines alone (scripts/engines_concurrent.py), the chain tests, then the bench
# at the driver's shape, alternating.  Usage (GPU box): bash scripts/archive/r06_rolecu_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
TAG=${1:-r06s}
REPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
REPS=6 timeout -k 10 240 python -u scripts/engines_concurrent.py 1 3 5 > $OUT/conc_rc2.log 2>&1 || { tail -20 $OUT/conc_rc2.log; exit 1; }
cat $OUT/conc_rc2.log
LISLAM_ROLE_CUS=1 REPS=6 timeout -k 10 240 python -u scripts/engines_concurrent.py 1 3 5 > $OUT/conc_rc1.log 2>&1 || { tail -20 $OUT/conc_rc1.log; exit 1; }
grep K= $OUT/conc_rc1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -1 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['value'], d['sustained']['value'], d['single_sequence']['value'], r['avg_launch_ms'], r['self_check'].get('pipelined_ms_per_launch'), d['engine_aborts'])"
}
for i in $(seq 1 $REPS); do
  run rc2_$i
  run rc1_$i LISLAM_ROLE_CUS=1
done
echo done > $OUT/ALL_DONE
