set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/chain_tests.log 2>&1 && \
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/r04a/smoke.log 2>&1
