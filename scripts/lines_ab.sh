#!/bin/bash
# k_scan_lines A/B on the GPU box: the scan-line parity tests on the in-tree library, the phase split
# of the developer build, then rocprofv3 kernel traces of the extraction alone, alternating the
# in-tree library and the scripts/_ab/liblislam_<variant>.so builds named after the reps (default: base).
# Usage (GPU box): bash scripts/lines_ab.sh <tag> [reps] [variant ...]
cd $GRAFT_REPO_ROOT
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-linesab}
R=${2:-3}
shift 2
VARS=${*:-base}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LISLAM_PROF_LIB=scripts/_ab/liblislam_prof.so timeout -k 10 180 python scripts/phase_prof.py lines 300 > $OUT/phase.txt 2>&1 || { tail -20 $OUT/phase.txt; exit 2; }
grep -v amdgpu.ids $OUT/phase.txt | tail -14
cd /tmp
: > $OUT/ab.txt
for r in $(seq 1 $R); do
  for v in new $VARS; do
    if [ $v != new ]; then export LISLAM_ALT_LIB=$ROOT/scripts/_ab/liblislam_$v.so; else unset LISLAM_ALT_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${v}_$r -o t -- python3 $ROOT/scripts/extract_prof.py 300 6 > $OUT/${v}_$r.log 2>&1 || { tail -5 $OUT/${v}_$r.log; exit 3; }
    python3 -c "
import csv, glob
f = glob.glob('$OUT/${v}_$r/**/t_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_scan_lines' in r['Name']: print('$v', $r, r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg', round(float(r['MinNs']) / 1e3, 1), 'min')" | tee -a $OUT/ab.txt
  done
done
echo done > $OUT/ALL_DONE
