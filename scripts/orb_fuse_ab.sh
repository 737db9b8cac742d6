#!/bin/bash
# Round 6: the ORB launch folds (k_orb_pairs, the solve's tail, k_target_index_all) against the split
# launches (LISLAM_ORB_PAIR_SPLIT=1 LISLAM_TI_SPLIT=1), after the GPU tests.
# Alternating driver-shape bench lines on one box.  Usage (GPU box): bash scripts/orb_fuse_ab.sh <tag> [reps]
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-orbfuse}
R=${2:-2}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_pipeline_timed.py tests/test_gpu_chain.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
: > $D/ab.txt
for r in $(seq 1 $R); do
  for v in fused split; do
    if [ $v = split ]; then E="LISLAM_ORB_PAIR_SPLIT=1 LISLAM_TI_SPLIT=1"; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 2 > $D/${v}_$r.json 2> $D/${v}_$r.err || { tail -20 $D/${v}_$r.err; exit 3; }
    python3 -c "
import json; d=json.load(open('$D/${v}_$r.json')); k=d['roofline']['kernel_ms_isolated_per_step']; p=d['roofline']['kernel_ms_per_step']
orb=sum(v for n,v in k.items() if n.startswith('k_orb')); orbp=sum(v for n,v in p.items() if n.startswith('k_orb'))
print('$v', $r, d['value'], d['sustained']['value'], d['single_sequence']['value'], 'orb iso %.3f pipe %.2f' % (orb, orbp), 'sel %.3f match %.3f ti %.3f' % (k['k_orb_select'], k['k_orb_match'], k['k_target_index']), d['pose_delta_vs_cpu']['orb_stats_mismatches'], d['pose_delta_vs_cpu']['orb_max_abs_T'])" | tee -a $D/ab.txt
  done
done
echo done > $D/ALL_DONE
