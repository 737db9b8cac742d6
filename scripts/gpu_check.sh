#!/bin/bash
# One GPU box call: the named -m gpu test files (or the whole suite), then optionally the default
# bench line.  Usage: bash scripts/gpu_check.sh <tag> [bench|nobench] [test files...]
set -o pipefail
TAG=${1:-chk}; shift
BENCH=${1:-bench}; shift
D=gpurun_out/$TAG
mkdir -p $D
( while sleep 30; do date >> $D/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
FILES="$*"
[ -z "$FILES" ] && FILES=tests
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $D/steps.txt
tail -3 $D/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
if [ "$BENCH" = bench ]; then
  timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
  rc=$?
  echo "bench rc=$rc" >> $D/steps.txt
  cat $D/bench.json | head -c 600
  exit $rc
fi
