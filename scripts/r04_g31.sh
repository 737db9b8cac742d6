# round-4 lines for config 3 (128x2048, one continuous 99-pair chain per 100-scan step) and
# config 5 (map-scale kNN: 20k queries vs a 5 M-point map)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04ai
mkdir -p $D
export PYTHONUNBUFFERED=1
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python bench.py --lines 128 --width 2048 --batch 100 --steps 5 --warmup 2 --cpu-budget 12 --sustain-s 0 --segmented 0 > $D/bench_c3.json 2> $D/bench_c3.err
rc=$?; echo "c3 rc=$rc" >> $D/steps.txt; [ $rc -lt 124 ] || exit $rc
timeout -k 10 400 python bench.py --workload map --steps 5 --warmup 2 > $D/bench_map.json 2> $D/bench_map.err
rc=$?; echo "map rc=$rc" >> $D/steps.txt; exit $rc
