#!/bin/bash
# The blocking contract's per-call phases (tools/blocking_seq.py, PSGPU_EXPORT_TRACE) with the
# scatter threads woken ahead of the export (default) and without (PSGPU_PREWAKE=0), REPS rounds
# each, interleaved; one box.  Usage (on the box): bash tools/blocking_ab.sh TAG [REPS]
set -o pipefail
TAG=$1; R=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq $R); do
  for w in 1 0; do
    PSGPU_PREWAKE=$w timeout -k 10 240 python3 -u tools/blocking_seq.py > $OUT/w${w}_$r.txt 2> $OUT/w${w}_$r.trace || { tail -5 $OUT/w${w}_$r.trace; exit 1; }
    echo "prewake $w round $r"; cut -c1-60 $OUT/w${w}_$r.txt
  done
done
