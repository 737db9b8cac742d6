# round-4 A/B + profiles: each step logs to $D; a test failure does not stop the later steps, a
# fault / abort / time limit (exit >= 124) ends the script
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04h
mkdir -p $D
step() {  # step <log> <timeout s> <command...>
  local log=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $D/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $D/steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
export PYTHONUNBUFFERED=1
step orb_tests_pyr3.log 300 env LISLAM_ALT_LIB=scripts/_ab/liblislam_pyr3.so python -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread
step orb_tests_main.log 300 python -m pytest tests/test_gpu_orb.py -x -v --timeout 200 --timeout-method thread
step orb_pyr3.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_pyr3.so python3 scripts/orb_quick.py 300
step orb_main.txt 120 python3 scripts/orb_quick.py 300
step orb_base.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_orbbase.so python3 scripts/orb_quick.py 300
step orb_fb8.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_fb8.so python3 scripts/orb_quick.py 300
step orb_fb16.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_fb16.so python3 scripts/orb_quick.py 300
step orb_desc4.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_desc4.so python3 scripts/orb_quick.py 300
step orb_prof.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_orbprof.so python3 scripts/orb_quick.py 300
step orb_prof4.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_orbprof4.so python3 scripts/orb_quick.py 300
step orb_pyr3prof.txt 120 env LISLAM_ALT_LIB=scripts/_ab/liblislam_pyr3prof.so python3 scripts/orb_quick.py 300
step parity_main.log 400 python -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread
step ab_lines.txt 300 python3 scripts/ab_lines.py scripts/_ab/liblislam_linesbase.so main
step lines_phase_base.txt 120 env LISLAM_PROF_LIB=scripts/_ab/liblislam_linesbaseprof.so python3 scripts/phase_prof.py lines 300
step lines_phase_new.txt 120 env LISLAM_PROF_LIB=scripts/_ab/liblislam_lines2prof.so python3 scripts/phase_prof.py lines 300
step engprof_split.txt 180 env LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so python3 scripts/engine_prof.py 300
step engprof_split248.txt 180 env LISLAM_ENGINE_WGS=248 LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so python3 scripts/engine_prof.py 300
step engprof_single.txt 180 env LISLAM_ENGINE_SINGLE=1 LISLAM_ALT_LIB=scripts/_ab/liblislam_engprof.so python3 scripts/engine_prof.py 300
