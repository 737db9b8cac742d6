#!/bin/bash
# Bench lines (no CPU baseline) under several environment settings ("NAME=V,NAME2=V2" each), after
# the chain tests under the first setting (NOTEST=1: none).  CTX=<n> in a setting: --contexts n.
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-benchab}
shift
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
: > $D/steps.txt
first=1
for v in "$@"; do
  n=${v//,/_}; n=${n//\//_}
  BENCH_ARGS=""
  case "$v" in *CTX=*) c=${v##*CTX=}; c=${c%%,*}; BENCH_ARGS="--contexts $c";; esac
  ( for e in ${v//,/ }; do export "$e"; done
    if [ $first = 1 ] && [ -z "$NOTEST" ]; then
      timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_pipeline_timed.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests_$n.log 2>&1 || exit 2
    fi
    timeout -k 10 300 python bench.py --cpu-budget 0 --scan-cache /tmp/lislam_scans $BENCH_ARGS > $D/bench_$n.json 2> $D/bench_$n.err ) || { echo "$v failed" >> $D/steps.txt; cat $D/steps.txt; exit 3; }
  first=0
  python3 -c "import json; d=json.load(open('$D/bench_$n.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'single', d['single_sequence']['value'], 'chain iso', r['kernel_ms_isolated_per_step'].get('k_odom_chain'), 'chain pipelined', r['kernel_ms_per_step'].get('k_odom_chain'), 'aborts', d['engine_aborts'])" >> $D/steps.txt
done
cat $D/steps.txt
