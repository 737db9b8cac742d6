set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04f
mkdir -p $D
REF=/tmp/ab_ref.npz
rm -f $REF
# A/B: the round-3 engine (noprof build) as the reference, then single-launch and split engines
LISLAM_ALT_LIB=scripts/_ab/liblislam_noprof.so CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_old.txt 2>&1 && \
LISLAM_ENGINE_SINGLE=1 CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_single.txt 2>&1 && \
CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_split.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_prims.py -x -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_split.json 2> $D/bench_split.err && \
LISLAM_ENGINE_SINGLE=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_single.json 2> $D/bench_single.err && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_cubemap.py tests/test_gpu_loop.py -x -v --timeout 300 --timeout-method thread > $D/map_tests.log 2>&1
