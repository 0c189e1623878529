#!/bin/bash
# Strong-scaling rehearsal on the baked tier (JIT=2: the kernels tier 2 of the bench's
# default --jit 3 serves a static grid), with the automatic tree split (TS=2, as bench.py
# --gpus N > 1 sets) and 2 rebalancing rounds: every rank's C3/C4 share; then the same on the
# structure kernels for the A/B on this box; then bench --gpus 2 on one device.
set -o pipefail
OUT=gpurun_out/r03tiershares
mkdir -p $OUT
export TMPDIR=/tmp
JIT=2 TS=2 CONFIG=C3 SHARES=1,2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3_baked.txt 2>&1 || { tail -5 $OUT/c3_baked.txt; exit 1; }
grep "slowest\|1/1" $OUT/c3_baked.txt
JIT=1 TS=2 CONFIG=C3 SHARES=1,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3_structure.txt 2>&1 || { tail -5 $OUT/c3_structure.txt; exit 1; }
grep "slowest\|1/1" $OUT/c3_structure.txt
PSGPU_BENCH_DEVICE=0 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 200 > $OUT/bench2.json 2> $OUT/bench2.err || { tail -5 $OUT/bench2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench2.json')); print(d['value'], d['ms_per_step'], d['config'].get('tree_split'), d['config'].get('tiered'))"
