#!/bin/bash
# bench sweep over the pipelined context count (--contexts) and the odometry chain groups
# (LISLAM_ODOM_GROUPS); two runs of each, no CPU leg
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for C in 2 3 4; do
    for G in 2 3; do
      LISLAM_ODOM_GROUPS=$G timeout -k 10 150 python bench.py --cpu-budget 0 --contexts $C --scan-cache /tmp/lislam_scans \
        > gpurun_out/sw_c${C}g${G}_$i.json 2>> gpurun_out/sw.err || exit 1
    done
  done
done
