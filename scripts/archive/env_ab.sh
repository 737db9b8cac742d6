#!/bin/bash
# Chain time + engine phase profile under several environment settings ("NAME=V,NAME2=V2" each).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-envab}
shift
mkdir -p $D
: > $D/steps.txt
for v in "$@"; do
  n=${v//,/_}; n=${n//\//_}
  ( for e in ${v//,/ }; do export "$e"; done
    CHAIN_ENGINE_ONLY=1 timeout -k 10 120 python scripts/chain_quick.py 300 10 2>&1 | grep -v amdgpu.ids > $D/chain_$n.txt
    LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 120 python scripts/engine_prof.py 300 2>&1 | grep -v amdgpu.ids > $D/prof_$n.txt ) || exit 3
  echo "$v: $(head -1 $D/chain_$n.txt)" >> $D/steps.txt
done
cat $D/steps.txt
for v in "$@"; do echo "== $v"; n=${v//,/_}; grep -E "chain of|association span \(|slowest item|hand-off assoc|record load|gather tail|solve total|item median \(|wave 0: 1-NN \(|wave 0: line" $D/prof_${n//\//_}.txt; done
