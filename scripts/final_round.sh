#!/bin/bash
# Round-end evidence on one GPU box (from the repo root): the GPU suite, the profile round
# (bench + rocprof kernel trace + FETCH_SIZE / WRITE_SIZE passes) and the streaming variants.
# Usage: bash scripts/final_round.sh <tag>
set -o pipefail
TAG=${1:-r02v}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/gpu_tests.log 2>&1 || exit 1
bash scripts/profile_round.sh $TAG || exit 2
for v in "chain299:--chain 299" "latency:--workload latency" "ingest:--workload ingest"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans $args \
    > gpurun_out/$TAG/bench_$name.json 2>> gpurun_out/$TAG/variants.err || exit 3
done
echo done > gpurun_out/$TAG/FINAL_DONE
