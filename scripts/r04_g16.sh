# host-side call spans of the pipelined bench
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04r
mkdir -p $D
timeout -k 10 300 env LISLAM_BENCH_HOSTLOG=1 python bench.py --steps 6 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench.json 2> $D/bench.err
echo "rc=$?" > $D/steps.txt
