#!/bin/bash
# Strong-scaling rehearsal with 8 hardware queues (as bench.py runs): every rank's share of
# C3 and C5, 4 engines, then two rounds of measured-time rebalancing.
set -o pipefail
OUT=gpurun_out/r03s8
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
CONFIG=C3 SHARES=1,2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3.txt 2>&1 || { tail -5 $OUT/c3.txt; exit 1; }
grep "slowest\|1/1" $OUT/c3.txt
CONFIG=C5 SHARES=1,2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $OUT/c5.txt 2>&1 || { tail -5 $OUT/c5.txt; exit 1; }
grep "slowest\|1/1" $OUT/c5.txt
RT_QUEUES=4 CONFIG=C3 SHARES=8 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 200 python3 -u tools/range_test.py > $OUT/c3_q4.txt 2>&1 || { tail -5 $OUT/c3_q4.txt; exit 1; }
grep "rank 0\|rank 4" $OUT/c3_q4.txt
# the empty step (every MPU fails S1: launch + kernel-boundary floor) at 8 queues, 1 and 4 engines
CONFIG=C3 SHARES=8 ENGINES=1,4 VB=8 FB=4 DBG=8 K=400 timeout -k 10 120 python3 -u tools/range_test.py > $OUT/c3_empty.txt 2>&1 || { tail -5 $OUT/c3_empty.txt; exit 1; }
cat $OUT/c3_empty.txt
# one host thread per engine (C-ABI, no Python) at the 1/8 share, 8 queues
timeout -k 10 200 tools/_bin/engine_threads tools/_bin/c3.bin 4 8 800 > $OUT/c3_threads.txt 2>&1 || { tail -5 $OUT/c3_threads.txt; exit 1; }
cat $OUT/c3_threads.txt
