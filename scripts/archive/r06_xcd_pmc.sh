#!/bin/bash
# Round-6 traffic attribution of the chain engine (the single-launch engine, LISLAM_ENGINE_SINGLE=1,
# which runs under dispatch-serialized counter collection): FETCH_SIZE / WRITE_SIZE / kernel time
# with the engine's stream kept on 1, 2, 4 or all 8 XCDs (LISLAM_WORK_XCDS): what each extra XCD's
# L2 re-fetches of the pairs' target structures costs.  Usage (GPU box): bash scripts/archive/r06_xcd_pmc.sh <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-r06x}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export LISLAM_ENGINE_SINGLE=1
( while sleep 30; do date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 200 python3 scripts/engine_pmc.py --launches 1 > $OUT/warm.json 2> $OUT/warm.err || exit 1
cd /tmp
for n in 8 4 2 1; do
  export LISLAM_WORK_XCDS=$n
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$n -o trace -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/trace_$n.json 2> $OUT/trace_$n.err || exit 2
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$n -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/fetch_$n.json 2> $OUT/fetch_$n.err || exit 3
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$n -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches 3 > $OUT/write_$n.json 2> $OUT/write_$n.err || exit 4
done
echo done > $OUT/ALL_DONE
