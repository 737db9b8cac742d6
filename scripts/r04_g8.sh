set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04h
mkdir -p $D
LISLAM_ALT_LIB=scripts/_ab/liblislam_pyr2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread > $D/orb_tests_pyr2.log 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_orbbase.so timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_base.txt 2>&1 && \
timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_main.txt 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_orbprof.so timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_prof.txt 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_pyr2prof.so timeout -k 10 120 python3 -u scripts/orb_quick.py 300 > $D/orb_pyr2prof.txt 2>&1 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so timeout -k 10 180 python3 -u scripts/engine_prof.py 300 > $D/engprof_split.txt 2>&1 && \
LISLAM_ENGINE_WGS=248 LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so timeout -k 10 180 python3 -u scripts/engine_prof.py 300 > $D/engprof_split248.txt 2>&1 && \
LISLAM_ENGINE_SINGLE=1 LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so timeout -k 10 180 python3 -u scripts/engine_prof.py 300 > $D/engprof_single.txt 2>&1
test $? -eq 0 && \
LISLAM_ALT_LIB=scripts/_ab/liblislam_lines2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $D/parity_lines2.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/ab_lines.py scripts/_ab/liblislam_linesbase.so main > $D/ab_lines2.txt 2>&1 && \
LISLAM_PROF_LIB=scripts/_ab/liblislam_linesbaseprof.so timeout -k 10 120 python3 -u scripts/phase_prof.py lines 300 > $D/lines_phase_base.txt 2>&1 && \
LISLAM_PROF_LIB=scripts/_ab/liblislam_lines2prof.so timeout -k 10 120 python3 -u scripts/phase_prof.py lines 300 > $D/lines_phase_new.txt 2>&1
