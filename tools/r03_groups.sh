#!/bin/bash
# Parameter groups (mode 1 loads a subtree's parameters together) vs one load per primitive
# (PSGPU_NO_GROUPS=1) vs parameters compiled in (JIT=2): GPU parity, then A/B.
set -o pipefail
OUT=gpurun_out/r03grp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for r in 1 2; do
  CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
  PSGPU_NO_GROUPS=1 CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py | sed 's/$/ nogroups/' >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
  JIT=2 CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
CONFIG=C5 SHARES=1 ENGINES=4 VB=8 FB=4 K=100 timeout -k 10 300 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
PSGPU_NO_GROUPS=1 CONFIG=C5 SHARES=1 ENGINES=4 VB=8 FB=4 K=100 timeout -k 10 300 python3 -u tools/range_test.py | sed 's/$/ nogroups/' >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
