# association overflow: engine phase profile and chain time at the default grid (CUs - 8 item
# workgroups) and with more item workgroups than CUs (2 on some CUs)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04z
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
step engprof_def.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so python3 scripts/engine_prof.py 300
step engprof_288.txt 120 env LISLAM_ENGINE_WGS=288 LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so python3 scripts/engine_prof.py 300
step chain_def.txt 120 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
step chain_288.txt 120 env LISLAM_ENGINE_WGS=288 CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
step chain_320.txt 120 env LISLAM_ENGINE_WGS=320 CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5
