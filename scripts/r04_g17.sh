cd $GRAFT_REPO_ROOT
D=gpurun_out/r04t
mkdir -p $D
timeout -k 10 300 env LISLAM_BENCH_HOSTLOG=1 python bench.py --steps 6 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_reorder.json 2> $D/bench_reorder.err && \
timeout -k 10 300 env LISLAM_BENCH_HOSTLOG=1 python bench.py --steps 20 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_reorder20.json 2> $D/bench_reorder20.err
echo "rc=$?" > $D/steps.txt
