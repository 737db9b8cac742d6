# the chain tests incl. the single-launch engine test
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04ak
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > $D/chain_tests.log 2>&1
echo "rc=$?" >> $D/steps.txt
