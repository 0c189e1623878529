#!/bin/bash
# r03 first GPU session: launch-cost probe, C5 / C3 strong-scaling rehearsal over every rank's
# share (4 engines, persistent grids 8 / 4 per CU as bench.py), instruction-cache counters.
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 tools/_bin/launch_cost > $OUT/launch_cost.txt 2>&1 || { tail -5 $OUT/launch_cost.txt; exit 1; }
cat $OUT/launch_cost.txt
CONFIG=C5 SHARES=1,2,4,8 ALLR=1 ENGINES=4 VB=8 FB=4 K=200 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c5_shares.txt 2>&1 || { tail -5 $OUT/c5_shares.txt; exit 1; }
cat $OUT/c5_shares.txt
CONFIG=C3 SHARES=1,2,4,8 ALLR=1 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3_shares.txt 2>&1 || { tail -5 $OUT/c3_shares.txt; exit 1; }
cat $OUT/c3_shares.txt
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -E "SQC_ICACHE|SQ_IFETCH|SQ_WAIT_INST|SQ_INSTS_SMEM|SQC_" $OUT/avail.txt | head -40
