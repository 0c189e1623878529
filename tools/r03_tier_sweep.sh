#!/bin/bash
# The baked tier (JIT=2): engines per device and the persistent k_vertex / k_finish grids
# (blocks per CU), C3 full grid, two rounds.
set -o pipefail
OUT=gpurun_out/r03tiersweep
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  JIT=2 CONFIG=C3 SHARES=1 ENGINES=3,4,5,6 VB=8 FB=4 K=600 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/sweep.txt 2>&1 || { tail -5 $OUT/sweep.txt; exit 1; }
  for vf in "6 3" "8 6" "12 4" "8 8" "4 4"; do
    set -- $vf
    JIT=2 CONFIG=C3 SHARES=1 ENGINES=4 VB=$1 FB=$2 K=600 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/sweep.txt 2>&1 || { tail -5 $OUT/sweep.txt; exit 1; }
  done
done
cat $OUT/sweep.txt
