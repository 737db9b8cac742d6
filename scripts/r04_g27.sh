# overflow queries claimed by the first waves done (work stealing): chain tests, phase profiles, A/B chain times, bench
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04af
mkdir -p $D
step() {  # step <log> <timeout s> <command...>
  local log=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $D/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $D/steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
export PYTHONUNBUFFERED=1
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
step chain_tests.log 300 python -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread
step engprof.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so python3 scripts/engine_prof.py 300
step chain_main1.txt 120 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
step chain_main2.txt 120 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
step bench.json 300 python bench.py --steps 12 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
