# the round-end checks on the current tree: the whole -m gpu suite, smoke(), the default bench line
cd $GRAFT_REPO_ROOT
D=gpurun_out/${R04FULL_TAG:-r04full}
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $D/steps.txt
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> $D/steps.txt
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
echo "bench rc=$?" >> $D/steps.txt
