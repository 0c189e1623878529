#!/bin/bash
# Parameters as scalar loads (JIT=1, default) vs compiled in as literals (JIT=2, baked):
# how much of the walk's time is scalar-load latency.  C3 full grid and 1/8 share, C5.
set -o pipefail
OUT=gpurun_out/r03baked
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for j in 1 2; do
  JIT=$j CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
for j in 1 2; do
  JIT=$j CONFIG=C5 SHARES=1 ENGINES=4 VB=8 FB=4 K=100 timeout -k 10 300 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
cat $OUT/ab.txt
