#!/bin/bash
# A/B of the chain engine's overflow stealing (round 5): chain tests on the main build, the chain's
# time with the main build and the no-steal variant, the engine phase profile with stealing.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r05d}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $D/steps.txt; tail -3 $D/tests.log
[ $rc -ne 0 ] && exit $rc
for v in main nosteal main; do
  if [ $v = main ]; then L=""; else L=scripts/_ab/liblislam_$v.so; fi
  CHAIN_ENGINE_ONLY=1 LISLAM_ALT_LIB=$L timeout -k 10 120 python scripts/chain_quick.py 300 10 > $D/chain_$v.txt 2>&1 || exit 3
  echo "$v: $(head -1 $D/chain_$v.txt)" >> $D/steps.txt
done
LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 120 python scripts/engine_prof.py 300 > $D/prof.txt 2>&1 || exit 4
cat $D/steps.txt; cat $D/prof.txt
