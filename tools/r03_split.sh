#!/bin/bash
# Tree split at the root in k_precheck / k_mpu (TS=1) vs one wave per item (TS=0): GPU parity,
# then A/B at the C3 full grid (1 and 4 engines) and every rank's 1/8 share, and C5.
set -o pipefail
OUT=gpurun_out/r03split
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split or random_trees or golden" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for r in 1 2; do
for ts in 0 1; do
  TS=$ts CONFIG=C3 SHARES=1 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
for ts in 0 1; do
  TS=$ts CONFIG=C3 SHARES=8 ALLR=1 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
  TS=$ts CONFIG=C5 SHARES=1 ENGINES=4 VB=8 FB=4 K=100 timeout -k 10 300 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
cat $OUT/ab.txt
