# the steal build with a divergence-free claim loop (variant library): a short chain, the chain
# tests, chain timing, stopping at the first failure
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04am
mkdir -p $D
export PYTHONUNBUFFERED=1
export LISLAM_ALT_LIB=scripts/_ab/liblislam_steal2.so
timeout -k 5 40 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 61 2 > $D/quick61.txt 2>&1
rc=$?; echo "quick61 rc=$rc" >> $D/steps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > $D/chain_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $D/steps.txt; [ $rc -lt 124 ] || exit $rc
timeout -k 10 120 env CHAIN_ENGINE_ONLY=1 python3 scripts/chain_quick.py 300 5 > $D/chain300.txt 2>&1
rc=$?; echo "chain300 rc=$rc" >> $D/steps.txt; exit $rc
