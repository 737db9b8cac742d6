# pipelined bench with more hardware queues per process (streams sharing a queue run in order)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04n
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
step bench_q16.json 300 env GPU_MAX_HW_QUEUES=16 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step bench_q8.json 300 env GPU_MAX_HW_QUEUES=8 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step bench_q16_c3.json 300 env GPU_MAX_HW_QUEUES=16 python bench.py --steps 10 --warmup 3 --cpu-budget 0 --sustain-s 0 --segmented 0 --contexts 3
