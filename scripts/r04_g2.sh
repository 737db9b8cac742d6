set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
timeout -k 10 60 ./scripts/micro/cumask 0 > gpurun_out/r04b/cumask0.txt 2>&1 && \
timeout -k 10 60 ./scripts/micro/cumask 37 > gpurun_out/r04b/cumask37.txt 2>&1 && \
bash scripts/ab_chain.sh gpurun_out/r04b main noprof > gpurun_out/r04b/ab.txt 2>&1
