# the PMC passes of profile_round.sh r04e (its bench and kernel trace already ran), single-launch engine
cd $GRAFT_REPO_ROOT
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
( while sleep 30; do date >> $OUT/heartbeat2; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/cache_bench.json 2> $OUT/cache_bench.err || exit 2  # the scan cache (no spawn pool under the profiler)
cd /tmp
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 3
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 4
LISLAM_ENGINE=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 0 --cpu-budget 0 --sustain-s 0 --scan-cache /tmp/lislam_scans > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit 5
echo done > $OUT/DONE
