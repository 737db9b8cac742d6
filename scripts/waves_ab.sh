#!/bin/bash
# A/B of the split engine's item workgroup size (LISLAM_ENGINE_ITEM_WAVES = queries per item):
# chain tests at each size, the chain's time per size, the phase profile per size.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r05g}
shift
SIZES=${*:-8 9 10}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for q in $SIZES; do
  LISLAM_ENGINE_ITEM_WAVES=$q timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_q$q.log 2>&1
  rc=$?; echo "Q=$q tests rc=$rc $(tail -1 $D/tests_q$q.log)" >> $D/steps.txt
  [ $rc -ne 0 ] && { cat $D/steps.txt; exit $rc; }
  LISLAM_ENGINE_ITEM_WAVES=$q CHAIN_ENGINE_ONLY=1 timeout -k 10 120 python scripts/chain_quick.py 300 10 2>&1 | grep -v amdgpu.ids > $D/chain_q$q.txt || exit 3
  echo "Q=$q: $(head -1 $D/chain_q$q.txt)" >> $D/steps.txt
  LISLAM_ENGINE_ITEM_WAVES=$q LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 120 python scripts/engine_prof.py 300 2>&1 | grep -v amdgpu.ids > $D/prof_q$q.txt || exit 4
done
cat $D/steps.txt
for q in $SIZES; do echo "== Q=$q"; grep -E "chain of|association span \(|slowest item|hand-off assoc|record load|gather tail|solve total|steal: claim|steal: stolen q" $D/prof_q$q.txt; done
