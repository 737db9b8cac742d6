# traced steal build on a 5-scan chain (0.3 s wait bounds): per-workgroup ticket / steal claims / role stage
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04al
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 5 40 env LISLAM_ALT_LIB=scripts/_ab/liblislam_stealtrace.so LISLAM_ENGINE_WAIT_US=300000 python3 scripts/engine_trace.py 5 > $D/trace5.txt 2>&1
echo "rc=$?" >> $D/steps.txt
