cd $GRAFT_REPO_ROOT
D=gpurun_out/r04u
mkdir -p $D
timeout -k 10 300 env LISLAM_BENCH_HOSTLOG=1 python bench.py --steps 12 --warmup 3 --cpu-budget 0 --sustain-s 0 --segmented 0 --contexts 3 > $D/bench_c3.json 2> $D/bench_c3.err && \
timeout -k 10 300 env LISLAM_BENCH_HOSTLOG=1 python bench.py --steps 12 --warmup 4 --cpu-budget 0 --sustain-s 0 --segmented 0 --contexts 4 > $D/bench_c4.json 2> $D/bench_c4.err
echo "rc=$?" > $D/steps.txt
