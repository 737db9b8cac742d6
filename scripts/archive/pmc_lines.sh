#!/bin/bash
# SQ counter passes over the extraction of the A/B batch (developer tool, GPU box):
#   bash scripts/archive/pmc_lines.sh <lib|main> <outdir>
set -o pipefail
LIB=${1:-main}; OUT=${2:-gpurun_out/pmc_lines}
ROOT=$(pwd); mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/archive/ab_lines.py main --reps 1 > $OUT/gen.log 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $ROOT/$OUT/p$i -o pmc -- python3 $ROOT/scripts/archive/ab_lines.py --child $LIB --out /tmp/pmc_x.npz --reps 1) > $OUT/p$i.log 2>&1 || exit $((i+1))
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_scan_lines" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()): print(f"  {c:24s} {v:16.0f}")
PY
