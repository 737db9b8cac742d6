#!/bin/bash
# The split engine's items at one query per wave (64-lane searches) vs four (16-lane rows,
# LISLAM_ENGINE_QPW=4): chain + pipelined tests at qpw 4, chain times and phase profiles of both,
# then the pipelined bench's timelines.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-qpw}
mkdir -p $D
LISLAM_ENGINE_QPW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_qpw4.log 2>&1
rc=$?; echo "qpw4 tests rc=$rc $(tail -1 $D/tests_qpw4.log)" > $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -40 $D/tests_qpw4.log; exit $rc; }
bash scripts/env_ab.sh ${1:-qpw}/env LISLAM_ENGINE_QPW=1 LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_ITEM_WAVES=3 || exit 3
TL_STEPS=12 bash scripts/timeline_ab.sh ${1:-qpw}/tl LISLAM_ENGINE_QPW=1 LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=3 || exit 4
cat $D/steps.txt
