mkdir -p gpurun_out/r06aa
export LISLAM_ALT_LIB=scripts/_ab/liblislam_stamps.so REPS=10
for v in "rc2" "rc2_nose0 LISLAM_ITEMS_SE0=0" "rc1 LISLAM_ROLE_CUS=1"; do
  set -- $v; name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/engines_concurrent.py 3 4 5 > gpurun_out/r06aa/$name.log 2>&1 || exit 1
  echo "== $name"; grep -E "K=" gpurun_out/r06aa/$name.log
done
