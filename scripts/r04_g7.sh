set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04g
mkdir -p $D
REF=/tmp/ab_ref.npz
rm -f $REF
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py -x -v --timeout 300 --timeout-method thread > $D/orb_tests.log 2>&1 && \
timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_fb4.txt 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_fb8.so timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_fb8.txt 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_fb16.so timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_fb16.txt 2>&1 && \
LISLAM_ENGINE_SINGLE=1 CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_single.txt 2>&1 && \
CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_split.txt 2>&1 && \
LISLAM_ENGINE_WGS=600 CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_split600.txt 2>&1 && \
LISLAM_ENGINE_WGS=124 CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 > $D/chain_split124.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_split.json 2> $D/bench_split.err && \
LISLAM_ENGINE_WGS=124 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-budget 0 --sustain-s 0 --segmented 0 > $D/bench_split124.json 2> $D/bench_split124.err
