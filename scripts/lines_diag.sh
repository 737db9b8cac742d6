#!/bin/bash
# k_scan_lines diagnosis on the GPU box: the per-phase cycle split (developer build, atomics out of
# the phases), the counters the box offers, and an instruction-mix pass over the extraction alone.
# Usage (GPU box): bash scripts/lines_diag.sh <tag>
cd $GRAFT_REPO_ROOT
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-linesdiag}
mkdir -p $OUT
export TMPDIR=/tmp
LISLAM_PROF_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 180 python scripts/phase_prof.py lines 300 > $OUT/phase.txt 2>&1 || { tail -20 $OUT/phase.txt; exit 1; }
cat $OUT/phase.txt | grep -v amdgpu.ids
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $OUT/mix -o pmc -- python3 $ROOT/scripts/extract_prof.py 300 2 > $OUT/mix.log 2>&1 || { tail -5 $OUT/mix.log; exit 2; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/cyc -o pmc -- python3 $ROOT/scripts/extract_prof.py 300 2 > $OUT/cyc.log 2>&1 || { tail -5 $OUT/cyc.log; exit 3; }
python3 - <<EOF
import csv, glob, collections
for p in ("mix", "cyc"):
    f = glob.glob("$OUT/%s/**/*counter_collection.csv" % p, recursive=True)
    if not f:
        print(p, "no csv"); continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "k_scan_lines" not in k: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    print(p, "sums over 2 launches:", {c: round(v) for c, v in acc.items()}, "rows", dict(n))
EOF
echo done > $OUT/ALL_DONE
