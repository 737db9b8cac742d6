#!/bin/bash
# Round 5: the super-chunk-first 16-lane line search: parity + chain tests at qpw 4 and 1, the chain
# time and phase profile at qpw 4 (K = 8 / 4), then the pipelined bench at qpw 4 / depth 4 / 4 contexts.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-ab3}
mkdir -p $D
LISLAM_ENGINE_QPW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_qpw4.log 2>&1
rc=$?; echo "qpw4 tests rc=$rc $(tail -1 $D/tests_qpw4.log)" > $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -40 $D/tests_qpw4.log; exit $rc; }
LISLAM_ENGINE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_round.log 2>&1
rc=$?; echo "per-round parity rc=$rc $(tail -1 $D/tests_round.log)" >> $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -40 $D/tests_round.log; exit $rc; }
bash scripts/env_ab.sh ${1:-ab3}/env LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_QPW=4,LISLAM_ALT_LIB=scripts/_ab/liblislam_k4.so || exit 3
TL_STEPS=12 bash scripts/timeline_ab.sh ${1:-ab3}/tl LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=4,CTX=4,LISLAM_ENGINE_WGS=144 LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=3,CTX=3,LISLAM_ENGINE_WGS=144 || exit 4
cat $D/steps.txt
