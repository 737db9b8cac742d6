#!/bin/bash
# The pipelined two-context test at several item workgroup sizes (LISLAM_ENGINE_ITEM_WAVES).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-pipeq}
shift
mkdir -p $D
: > $D/steps.txt
for q in "$@"; do
  LISLAM_ENGINE_ITEM_WAVES=$q timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_q$q.log 2>&1
  echo "Q=$q rc=$? $(grep -E 'AssertionError: |passed|failed' $D/tests_q$q.log | head -3 | tr '\n' ' ')" >> $D/steps.txt
done
cat $D/steps.txt
