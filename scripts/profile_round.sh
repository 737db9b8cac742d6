#!/bin/bash
# Bench + rocprofv3 kernel-trace/stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE).
# Usage (on the GPU box, from the repo root): bash scripts/profile_round.sh <tag> [extra bench.py args]
set -o pipefail
TAG=${1:-r01}
shift
EXTRA="$*"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat; done ) &  # progress for the box's silence watchdog
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python bench.py --scan-cache /tmp/lislam_scans $EXTRA > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $ROOT/bench.py --steps 3 --warmup 1 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans $EXTRA > $OUT/trace_bench.json 2> $OUT/trace.err || exit 2
# (the PMC passes run the per-round odometry schedule, LISLAM_ENGINE=0: counter collection
# serializes dispatches, and the chain engine's persistent workgroups must run together — both the
# split and the single-launch engine give up on their bounded waits under it)
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans $EXTRA > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 3
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans $EXTRA > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 4
# the dominant kernel's stall picture: wave cycles, cycles waiting on anything / on instruction
# issue, cycles with an instruction active (SQ block, 4 of its 8 counters; a pass of its own)
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans $EXTRA > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit 5
echo done > $OUT/DONE
