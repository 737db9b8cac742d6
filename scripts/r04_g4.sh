set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04d
LISLAM_ALT_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 300 python -u scripts/engine_prof.py 300 > gpurun_out/r04d/engine_prof.txt 2>&1
