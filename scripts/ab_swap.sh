#!/bin/bash
# bench A/B of whole-library variants (developer tool, GPU box): each scripts/_ab/liblislam_<v>.so
# is copied over the in-tree library for one bench run; the original is restored at the end.
set -o pipefail
mkdir -p gpurun_out
LIB=intensity_based_lidar_slam_for_me-_amd/liblislam.so
cp $LIB /tmp/liblislam_orig.so
rc=0
for i in 1 2; do
  for v in "$@"; do
    cp scripts/_ab/liblislam_$v.so $LIB
    timeout -k 10 150 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans > gpurun_out/ab_${v}_$i.json 2>> gpurun_out/ab.err || { rc=1; break 2; }
  done
done
cp /tmp/liblislam_orig.so $LIB
exit $rc
