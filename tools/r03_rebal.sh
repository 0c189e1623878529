#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03reb
mkdir -p $OUT
export TMPDIR=/tmp
CONFIG=C5 SHARES=2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $OUT/c5.txt 2>&1 || { tail -5 $OUT/c5.txt; exit 1; }
grep "slowest" $OUT/c5.txt
CONFIG=C3 SHARES=4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3.txt 2>&1 || { tail -5 $OUT/c3.txt; exit 1; }
grep "slowest" $OUT/c3.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
