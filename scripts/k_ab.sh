#!/bin/bash
# The 16-lane searches' chunks per round trip (LISLAM_NN16_K / LISLAM_LS16_K variants): engine
# tests at qpw 4 and 1 (the per-round schedule's tests use the same searches), then chain times.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-kab}
mkdir -p $D
LISLAM_ENGINE_QPW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_qpw4.log 2>&1
rc=$?; echo "qpw4 tests rc=$rc $(tail -1 $D/tests_qpw4.log)" > $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -40 $D/tests_qpw4.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_qpw1.log 2>&1
rc=$?; echo "qpw1 tests rc=$rc $(tail -1 $D/tests_qpw1.log)" >> $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -40 $D/tests_qpw1.log; exit $rc; }
bash scripts/env_ab.sh ${1:-kab}/env LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_QPW=4,LISLAM_ALT_LIB=scripts/_ab/liblislam_k4.so LISLAM_ENGINE_QPW=4,LISLAM_ALT_LIB=scripts/_ab/liblislam_k16.so || exit 3
cat $D/steps.txt
