#!/bin/bash
# Round-6 A/B: the split engine's items confined to the first n XCDs (LISLAM_ENGINE_XCDS, developer),
# one chain alone (scripts/chain_quick.py, engine only), latency and throughput shapes.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06n}
mkdir -p $OUT
export CHAIN_ENGINE_ONLY=1
for n in 8 4 2 1; do
  if [ $n = 8 ]; then W=""; else W=$((31 * n)); fi
  env LISLAM_ENGINE_XCDS=$n ${W:+LISLAM_ENGINE_WGS=$W} timeout -k 10 120 python scripts/chain_quick.py 300 5 2>/dev/null | sed "s/^/lat xcds=$n wgs=$W: /" || exit 1
done
for n in 8 4 2 1; do
  if [ $n = 8 ]; then W=""; else W=$((62 * n)); fi
  env LISLAM_ENGINE_QPW=3 LISLAM_ENGINE_DEPTH=5 LISLAM_ENGINE_XCDS=$n ${W:+LISLAM_ENGINE_WGS=$W} timeout -k 10 120 python scripts/chain_quick.py 300 5 2>/dev/null | sed "s/^/thr xcds=$n wgs=$W: /" || exit 2
done
