set -o pipefail
mkdir -p gpurun_out/r03a
for v in 1 0; do
  LISLAM_ASSOC16=$v LISLAM_ASSOC_WAVES=4 timeout -k 10 200 python -u scripts/chain_quick.py 300 3 > gpurun_out/r03a/assoc_ab_$v.log 2>&1 || exit 1
done
