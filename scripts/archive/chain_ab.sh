#!/bin/bash
# Chain time alone (scripts/chain_quick.py, 300 scans, 10 repetitions) under several environment
# settings ("NAME=V,NAME2=V2" each), twice each in alternating order.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-chainab}
shift
mkdir -p $D
: > $D/steps.txt
for rep in 1 2; do
  for v in "$@"; do
    n=${v//,/_}; n=${n//\//_}
    ( for e in ${v//,/ }; do export "$e"; done
      CHAIN_ENGINE_ONLY=1 timeout -k 10 120 python scripts/chain_quick.py 300 10 2>&1 | grep -v amdgpu.ids > $D/chain_${n}_$rep.txt ) || exit 3
    echo "$v: $(head -1 $D/chain_${n}_$rep.txt)" >> $D/steps.txt
  done
done
cat $D/steps.txt
