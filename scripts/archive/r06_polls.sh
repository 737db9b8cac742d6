#!/bin/bash
# Round-6: the chain engine's device waits counted (developer build, scripts/engine_polls.py).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06w}
mkdir -p $OUT
export LISLAM_ALT_LIB=$(pwd)/scripts/_ab/liblislam_prof.so
timeout -k 10 200 python scripts/engine_polls.py latency > $OUT/split_latency.json 2> $OUT/split_latency.err || exit 1
timeout -k 10 200 python scripts/engine_polls.py throughput > $OUT/split_throughput.json 2> $OUT/split_throughput.err || exit 2
LISLAM_ENGINE_SINGLE=1 timeout -k 10 200 python scripts/engine_polls.py latency > $OUT/single.json 2> $OUT/single.err || exit 3
cat $OUT/*.json
