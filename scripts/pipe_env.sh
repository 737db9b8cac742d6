#!/bin/bash
# The pipelined two-context test under several environment settings ("NAME=V,NAME2=V2" each).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-pipeenv}
shift
mkdir -p $D
: > $D/steps.txt
for v in "$@"; do
  n=${v//,/_}
  ( for e in ${v//,/ }; do export "$e"; done
    timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/t_$n.log 2>&1 )
  echo "$v rc=$? $(grep -E 'AssertionError: |passed|failed' $D/t_$n.log | head -3 | tr '\n' ' ')" >> $D/steps.txt
done
cat $D/steps.txt
