#!/bin/bash
# tests/test_gpu_parity.py's odometry tests under each odometry schedule (default = split engine,
# LISLAM_ENGINE=0 = per-round, LISLAM_ENGINE_SINGLE=1 = single-launch engine, LISLAM_ENGINE_QPW=4).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-pm}
mkdir -p $D
: > $D/steps.txt
for v in DEFAULT=1 LISLAM_ENGINE=0 LISLAM_ENGINE_SINGLE=1 LISLAM_ENGINE_QPW=4; do
  ( export $v; timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k odometry --timeout 200 --timeout-method thread > $D/t_$v.log 2>&1 )
  rc=$?
  echo "$v rc=$rc $(tail -1 $D/t_$v.log)" >> $D/steps.txt
  [ $rc -gt 1 ] && break
done
cat $D/steps.txt
grep -h "^FAILED" $D/t_*.log
