#!/bin/bash
# bench sweep over the odometry chain-group count (LISLAM_ODOM_GROUPS), with and without ORB
set -o pipefail
mkdir -p gpurun_out
for G in 1 2 3 4; do
  LISLAM_ODOM_GROUPS=$G timeout -k 10 120 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans > gpurun_out/g$G.json 2>> gpurun_out/sweep.err || exit 1
  LISLAM_ODOM_GROUPS=$G timeout -k 10 120 python bench.py --cpu-budget 0 --no-orb --scan-cache /tmp/lislam_scans > gpurun_out/g${G}n.json 2>> gpurun_out/sweep.err || exit 1
done
