#!/bin/bash
# One engine (a blocking caller) on the baked tier: k_finish vertices per wave (FQ 0: 64,
# 3: 32, 1: 16) x k_vertex layout (VW 1: one lane per vertex, 0: a quad per vertex), C3 full
# grid, single-engine grids (16 / 8 blocks per CU), two rounds; then 4 engines for the
# layouts that win.
set -o pipefail
OUT=gpurun_out/r03lat
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for fq in 0 3 1; do
for vw in 1 0; do
  JIT=2 FQ=$fq VW=$vw CONFIG=C3 SHARES=1 ENGINES=1 VB=16 FB=8 K=300 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
done
for fq in 0 3 1; do
  JIT=2 FQ=$fq VW=1 CONFIG=C3 SHARES=1 ENGINES=4 VB=8 FB=4 K=500 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
grep "ms/step" $OUT/ab.txt | sed 's/BD=- DBG=- GR=- //'
