#!/bin/bash
# Round 5: the 16-lane searches' chunks per round trip (chain time, phase profile), then the
# pipelined bench at qpw 4 / depth 3 / 3 contexts against the qpw 1 / depth 2 / 2 contexts default.
cd $GRAFT_REPO_ROOT
bash scripts/env_ab.sh ${1:-ab2}/env LISLAM_ENGINE_QPW=4 LISLAM_ENGINE_QPW=4,LISLAM_ALT_LIB=scripts/_ab/liblislam_k4.so LISLAM_ENGINE_QPW=4,LISLAM_ALT_LIB=scripts/_ab/liblislam_k16.so LISLAM_ENGINE_QPW=1 || exit 3
TL_STEPS=12 bash scripts/timeline_ab.sh ${1:-ab2}/tl LISLAM_ENGINE_QPW=1 LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=3,CTX=3 LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=3,CTX=3,LISLAM_ALT_LIB=scripts/_ab/liblislam_k16.so LISLAM_ENGINE_QPW=4,LISLAM_ENGINE_DEPTH=4,CTX=4 || exit 4
