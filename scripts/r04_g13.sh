# kernel trace of the pipelined bench (timeline of chains vs extraction / ORB); a heartbeat file
# shows progress while the profiled bench runs
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04v
mkdir -p $D
export TMPDIR=/tmp PYTHONUNBUFFERED=1
( while sleep 20; do date >> $D/heartbeat; done ) &
HB=$!
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench.json 2> $D/bench.err
echo "rc=$?" > $D/steps.txt
kill $HB
