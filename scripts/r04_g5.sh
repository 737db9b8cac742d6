set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04e
bash scripts/ab_chain.sh gpurun_out/r04e noprof main > gpurun_out/r04e/ab.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_prims.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04e/tests.log 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 300 python -u scripts/engine_prof.py 300 > gpurun_out/r04e/engine_prof.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_cubemap.py tests/test_gpu_loop.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04e/map_tests.log 2>&1
