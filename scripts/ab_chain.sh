#!/bin/bash
# Chain-engine A/B (developer tool, GPU box): the continuous 299-pair chain through each library
# variant scripts/_ab/liblislam_<v>.so ("main" = the in-tree build), outputs checked against the
# first variant's.  Usage: bash scripts/ab_chain.sh <out> <v1> <v2> ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
REF=/tmp/ab_chain_ref.npz
rm -f $REF
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then LIB=""; else LIB=scripts/_ab/liblislam_$v.so; fi
    LISLAM_ALT_LIB=$LIB CHAIN_ENGINE_ONLY=1 CHAIN_REF=$REF timeout -k 10 120 python3 -u scripts/chain_quick.py 300 5 \
      > $OUT/chain_${v}_$rep.txt 2>&1 || exit 1
    grep -h "engine" $OUT/chain_${v}_$rep.txt | sed "s/^/$v: /"
  done
done
