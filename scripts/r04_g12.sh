# pipelined bench with the step's chain queued before the next batch's extraction; 2 and 3 contexts
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04l
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
step bench_c2.json 300 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
step bench_c3.json 300 python bench.py --steps 10 --warmup 3 --cpu-budget 0 --sustain-s 0 --segmented 0 --contexts 3
step bench_c2_open.json 300 env LISLAM_ENGINE_STREAMS=open python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0
