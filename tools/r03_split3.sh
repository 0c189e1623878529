#!/bin/bash
# Strong-scaling rehearsal with the automatic tree split (TS=2, as bench.py --gpus N > 1 sets):
# every rank's C3 and C5 share with 2 rebalancing rounds; bench --gpus 2 on one device.
set -o pipefail
OUT=gpurun_out/r03split3
mkdir -p $OUT
export TMPDIR=/tmp
TS=2 CONFIG=C3 SHARES=1,2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/c3.txt 2>&1 || { tail -5 $OUT/c3.txt; exit 1; }
grep "slowest\|1/1" $OUT/c3.txt
TS=2 CONFIG=C5 SHARES=1,2,4,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $OUT/c5.txt 2>&1 || { tail -5 $OUT/c5.txt; exit 1; }
grep "slowest\|1/1" $OUT/c5.txt
PSGPU_BENCH_DEVICE=0 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 200 > $OUT/bench2.json 2> $OUT/bench2.err || { tail -5 $OUT/bench2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench2.json')); print(d['value'], d['ms_per_step'], d['config'].get('tree_split'))"
