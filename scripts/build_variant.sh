#!/bin/bash
# Developer A/B builds: recompile one translation unit with extra -D flags and link it with the
# other objects of the last build() into scripts/_ab/liblislam_<name>.so (load it with
# LISLAM_ALT_LIB=<path> in scripts/gpu_quick.py).  Usage: scripts/build_variant.sh <name> <source> [-DFOO=1 ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; shift 2
CSRC=$ROOT/intensity_based_lidar_slam_for_me-_amd/csrc
OBJ=$ROOT/build/obj
OUT=$ROOT/scripts/_ab
mkdir -p $OUT/$NAME
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -mcode-object-version=5 -Wno-unused-value -Wno-unused-result"
BASE=${REPLACES:-${SRC%.*}}  # REPLACES=<object base name> when SRC is a renamed copy
(cd $CSRC && /opt/rocm/bin/hipcc $FLAGS "$@" -c -o $OUT/$NAME/$BASE.o $SRC)
OBJS=""
for o in $OBJ/*.o; do [ "$(basename $o)" = "$BASE.o" ] && OBJS="$OBJS $OUT/$NAME/$BASE.o" || OBJS="$OBJS $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liblislam_$NAME.so $OBJS
echo $OUT/liblislam_$NAME.so
