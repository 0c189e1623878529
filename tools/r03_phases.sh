#!/bin/bash
# Where the isolated spans go on the baked tier: per-wave timeline of one engine's
# polygonization, k_mpu phases (debug bit 4096) and k_precheck phases (8192).
set -o pipefail
OUT=gpurun_out/r03phases
mkdir -p $OUT
export TMPDIR=/tmp
export PSGPU_JIT=2
timeout -k 10 120 python3 -u tools/timeline.py --jit 2 > $OUT/timeline.txt 2>&1 || { tail -5 $OUT/timeline.txt; exit 1; }
timeout -k 10 120 python3 -u tools/timeline.py --phases > $OUT/mpu_phases.txt 2>&1 || { tail -5 $OUT/mpu_phases.txt; exit 1; }
timeout -k 10 120 python3 -u tools/timeline.py --precheck > $OUT/precheck_phases.txt 2>&1 || { tail -5 $OUT/precheck_phases.txt; exit 1; }
cat $OUT/timeline.txt $OUT/mpu_phases.txt $OUT/precheck_phases.txt
