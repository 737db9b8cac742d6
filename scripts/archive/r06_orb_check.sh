#!/bin/bash
# Round-6 ORB check on the GPU box: the ORB and pipelined parity tests, then one driver-shape bench
# with the per-kernel pipelined / isolated ms per step.  Usage: bash scripts/archive/r06_orb_check.sh <tag>
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06ag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
env $EXTRA_ENV timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --segmented 0 --sustain-s 2.5 --scan-cache /tmp/lislam_scans > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 2; }
python - $OUT/b.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print(d["value"], d["sustained"]["value"], d["single_sequence"]["value"])
iso = r["kernel_ms_isolated_per_step"]
print({k: (round(v, 2), round(iso.get(k, 0), 3)) for k, v in r["kernel_ms_per_step"].items() if v})
PY
