#!/bin/bash
# Tree split crossover: TS=0 vs TS=1 over every rank's C3 1/2 and 1/4 shares and C5's 1/8
# shares (the share sizes between the 1/8 C3 gain and the full-grid loss).
set -o pipefail
OUT=gpurun_out/r03split2
mkdir -p $OUT
export TMPDIR=/tmp
for ts in 0 1; do
  TS=$ts CONFIG=C3 SHARES=2,4 ALLR=1 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
  TS=$ts CONFIG=C5 SHARES=8 ALLR=1 ENGINES=4 VB=8 FB=4 K=150 timeout -k 10 300 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
grep "slowest" $OUT/ab.txt
