#!/bin/bash
# The chain engine's counters (scripts/engine_pmc.py says why the single-launch engine): a kernel
# trace pass and FETCH_SIZE / WRITE_SIZE / SQ passes, each its own rocprofv3 run, the program right
# after --.  Then scripts/summarize_engine_pmc.py <tag> (on the CPU side) writes profiles/<tag>_*.
cd $GRAFT_REPO_ROOT
ROOT=$(pwd)
D=$ROOT/gpurun_out/${1:-r05c}
N=${2:-6}
mkdir -p $D
export TMPDIR=/tmp
export LISLAM_ENGINE_SINGLE=1
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 200 python3 scripts/engine_pmc.py --launches 2 > $D/plain.json 2> $D/plain.err || exit 1
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o trace -- python3 $ROOT/scripts/engine_pmc.py --launches $N > $D/trace.json 2> $D/trace.err || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches $N > $D/fetch.json 2> $D/fetch.err || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches $N > $D/write.json 2> $D/write.err || exit 4
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $D/pmc_sq -o pmc -- python3 $ROOT/scripts/engine_pmc.py --launches $N > $D/sq.json 2> $D/sq.err || exit 5
cat $D/plain.json $D/trace.json $D/fetch.json $D/write.json $D/sq.json
