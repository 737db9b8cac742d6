#!/bin/bash
# Round 5: sequential multi-query waves (qpw 2, 3): chain tests at each, chain times, then bench lines.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-seq}
mkdir -p $D
for q in 2 3; do
  LISLAM_ENGINE_QPW=$q timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_qpw$q.log 2>&1
  rc=$?; echo "qpw$q tests rc=$rc $(tail -1 $D/tests_qpw$q.log)" >> $D/steps.txt
  [ $rc -ne 0 ] && { cat $D/steps.txt; tail -30 $D/tests_qpw$q.log; exit $rc; }
done
bash scripts/chain_ab.sh ${1:-seq}/chain LISLAM_ENGINE_QPW=1 LISLAM_ENGINE_QPW=2 LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_QPW=4 || exit 3
NOTEST=1 bash scripts/bench_ab.sh ${1:-seq}/bench LISLAM_ENGINE_QPW=2,LISLAM_ENGINE_DEPTH=3,CTX=3 LISLAM_ENGINE_QPW=2,LISLAM_ENGINE_DEPTH=3,CTX=4 LISLAM_ENGINE_QPW=3,LISLAM_ENGINE_DEPTH=4,CTX=4 LISLAM_ENGINE_QPW=2,LISLAM_ENGINE_DEPTH=4,CTX=4 DEF=1 || exit 4
cat $D/steps.txt
