# the default bench line (20 timed steps)
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04aj
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
echo "bench rc=$?" >> $D/steps.txt
