# A/B: engine wave priority 3 (main) vs 0 (variant), pipelined bench, alternating
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04x
mkdir -p $D
B="python bench.py --steps 12 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0"
timeout -k 10 300 $B > $D/p3_1.json 2> $D/p3_1.err && \
timeout -k 10 300 env LISLAM_ALT_LIB=scripts/_ab/liblislam_prio0.so $B > $D/p0_1.json 2> $D/p0_1.err && \
timeout -k 10 300 $B > $D/p3_2.json 2> $D/p3_2.err && \
timeout -k 10 300 env LISLAM_ALT_LIB=scripts/_ab/liblislam_prio0.so $B > $D/p0_2.json 2> $D/p0_2.err
echo "rc=$?" > $D/steps.txt
