#!/bin/bash
# The map path's GPU tests and the config-5 bench line.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-mapchk}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_cubemap.py tests/test_gpu_pipeline.py tests/test_gpu_factors_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1
rc=$?; echo "map tests rc=$rc $(tail -1 $D/tests.log)" > $D/steps.txt
[ $rc -ne 0 ] && { cat $D/steps.txt; tail -30 $D/tests.log; exit $rc; }
timeout -k 10 300 python bench.py --workload map --steps 20 --cpu-budget 0 > $D/bench_map.json 2> $D/bench_map.err
echo "map bench rc=$?" >> $D/steps.txt
python3 -c "import json; d=json.load(open('$D/bench_map.json')); print(d['value'], d['ms_per_step'], d['pose_delta_vs_cpu'], d['roofline']['kernel_ms_per_step'])" >> $D/steps.txt
cat $D/steps.txt
