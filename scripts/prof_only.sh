#!/bin/bash
# The chain engine's phase profile alone (a -DLISLAM_ENG_PROF=1 variant, scripts/build_variant.sh prof).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-prof}
mkdir -p $D
LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 120 python scripts/engine_prof.py 300 > $D/prof.txt 2>&1
rc=$?
grep -v amdgpu.ids $D/prof.txt
exit $rc
