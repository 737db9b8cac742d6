# ORB: parity of the current tree, then per-kernel SQ counters of the ORB batch (orb_quick) — which
# counters exist, then two passes of 8 SQ counters each
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04j
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {  # step <log> <timeout s> <command...>
  local log=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $D/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $D/steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step orb_tests.log 300 python -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread
step orb_main.txt 120 python3 scripts/orb_quick.py 300
step counters.txt 60 rocprofv3 -L
step pmc1.txt 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $D/pmc1 -o pmc -- python3 scripts/orb_quick.py 300
step pmc2.txt 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d $D/pmc2 -o pmc -- python3 scripts/orb_quick.py 300
