set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
bash scripts/ab_chain.sh gpurun_out/r04c noprof main > gpurun_out/r04c/ab.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c/chain_tests.log 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 300 python -u scripts/engine_prof.py 300 > gpurun_out/r04c/engine_prof.txt 2>&1
