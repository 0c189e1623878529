#!/bin/bash
# Full GPU test suite, then the tree-split A/B over every rank's C3 1/8 share (warm-up fixed)
# and a default bench line.
set -o pipefail
OUT=gpurun_out/r03chk
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for ts in 0 1; do
  TS=$ts CONFIG=C3 SHARES=8 ALLR=1 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 150 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
cat $OUT/ab.txt
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d.get('latency_ms_single'))"
