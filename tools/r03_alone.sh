#!/bin/bash
# Layout defaults that know whether a run is alone on its device: parity subset, then C3
# on the baked tier with the default layouts at 1 and 4 engines (twice), then the bench line.
set -o pipefail
OUT=gpurun_out/r03alone
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  JIT=2 CONFIG=C3 SHARES=1,8 ENGINES=1,4 K=400 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
grep "ms/step" $OUT/ab.txt | sed 's/FQ=- BD=- DBG=- GR=- VW=- //'
timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['latency_ms_single'], d['kernel_ms_per_launch_isolated'])"
