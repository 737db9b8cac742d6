#!/bin/bash
# Can the chain engine's counters be collected?  rocprofv3 --pmc FETCH_SIZE over one bench step
# (config 2) with the split engine, the single-launch engine, and the single-launch engine capped
# at a few workgroups; each line's engine_aborts says whether a bounded wait expired under the
# profiler (an abort is re-run on the per-round schedule, so every pass completes).
cd $GRAFT_REPO_ROOT
ROOT=$(pwd)
D=$ROOT/gpurun_out/${1:-r05b}
mkdir -p $D
export TMPDIR=/tmp
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="--steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --segmented 0 --scan-cache /tmp/lislam_scans"
timeout -k 10 200 python bench.py $B > $D/plain.json 2> $D/plain.err || exit 1
cd /tmp
for v in "split:" "single:LISLAM_ENGINE_SINGLE=1" "single_wgs8:LISLAM_ENGINE_SINGLE=1 LISLAM_ENGINE_WGS=8"; do
  name=${v%%:*}; envs=${v#*:}
  ( for e in $envs; do export "$e"; done
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_$name -o pmc -- python3 $ROOT/bench.py $B > $D/$name.json 2> $D/$name.err )
  echo "$name rc=$?" >> $D/steps.txt
  python3 -c "import json,sys; d=json.load(open('$D/$name.json')); print('$name', d['engine_aborts'], d['config']['odometry_schedule'], d['ms_per_step'])" >> $D/steps.txt 2>&1
done
cat $D/steps.txt
