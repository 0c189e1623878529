#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03p2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 tools/_bin/launch_cost > $OUT/launch_cost.txt 2>&1 || { tail -5 $OUT/launch_cost.txt; exit 1; }
grep -E "module|threads|round trip" $OUT/launch_cost.txt
for E in 4 6 8; do
  GPU_MAX_HW_QUEUES=$((E*2)) timeout -k 10 200 tools/_bin/engine_threads tools/_bin/c3.bin $E 1,8 800 > $OUT/c3_E$E.txt 2>&1 || { tail -5 $OUT/c3_E$E.txt; exit 1; }
  cat $OUT/c3_E$E.txt
done
