# pipelined bench: library work streams kept off the solve roles' CUs vs unmasked
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04k
mkdir -p $D
export PYTHONUNBUFFERED=1
step() {  # step <log> <timeout s> <command...>
  local log=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $D/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $D/steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step bench_workmask.json 300 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step bench_open.json 300 env LISLAM_ENGINE_STREAMS=open python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step chain_tests.log 600 python -m pytest tests/test_gpu_chain.py -x -v --timeout 300 --timeout-method thread
