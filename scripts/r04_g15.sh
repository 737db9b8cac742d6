# pipelined bench: hardware queue mapping A/B (GPU_MAX_HW_QUEUES, masked vs open work streams)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04p
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
B="python bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0"
step default.json 300 $B
step q16.json 300 env GPU_MAX_HW_QUEUES=16 $B
step open.json 300 env LISLAM_ENGINE_STREAMS=open $B
step q16_open.json 300 env GPU_MAX_HW_QUEUES=16 LISLAM_ENGINE_STREAMS=open $B
step q8_open.json 300 env GPU_MAX_HW_QUEUES=8 LISLAM_ENGINE_STREAMS=open $B
