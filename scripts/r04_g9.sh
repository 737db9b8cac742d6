# ORB descriptor bisect + the new ORB front end's timing + pipelined bench (priority vs CU-masked engine streams)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04i
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
step orb_tests_main.log 300 python -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread
step orb_tests_olddesc.log 300 env LISLAM_ALT_LIB=scripts/_ab/liblislam_olddesc.so python -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread
step orb_main.txt 120 python3 scripts/orb_quick.py 300
step orb_olddesc.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_olddesc.so python3 scripts/orb_quick.py 300
step bench_prio.json 300 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step bench_mask.json 300 env LISLAM_ENGINE_STREAMS=mask python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step chain_prio.txt 120 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
