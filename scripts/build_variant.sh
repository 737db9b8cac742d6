#!/bin/bash
# A/B variant of the library: lislam_odometry.hip recompiled with extra -D flags, linked with the
# other objects of the current build (python -c "import __graft_entry__ as g; g.build()" first).
#   scripts/build_variant.sh prog -DLISLAM_ENG_PROG=1   ->  scripts/_ab/liblislam_prog.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=intensity_based_lidar_slam_for_me-_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -mcode-object-version=5 -Wno-unused-value -Wno-unused-result"
mkdir -p scripts/_ab/$name
/opt/rocm/bin/hipcc $F "$@" -c -o scripts/_ab/$name/lislam_odometry.o $C/lislam_odometry.hip
objs=""
for o in build/obj/*.o; do
  [ "$(basename $o)" = lislam_odometry.o ] && o=scripts/_ab/$name/lislam_odometry.o
  objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/_ab/liblislam_$name.so $objs
echo scripts/_ab/liblislam_$name.so
