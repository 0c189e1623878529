#!/bin/bash
# k_vertex layouts: GPU parity, then A/B of the quad layout (VW=0) against the per-run choice
# (VW=2: one lane per vertex on large runs) on C3 / C5 full grids and the C3 1/8 share.
set -o pipefail
OUT=gpurun_out/r03vw
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "vertex_layouts or random_trees or c3_full or finish_layouts or golden_digests" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for r in 1 2; do
for vw in 0 2; do
  VW=$vw CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 120 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
  VW=$vw CONFIG=C5 SHARES=1 ENGINES=4 VB=8 FB=4 K=100 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
cat $OUT/ab.txt
