#!/bin/bash
# Tiered kernels: the GPU test, then the default bench line (structure pass + baked headline)
# and the C5 line (structure kernels: its parameters change every frame).
set -o pipefail
OUT=gpurun_out/r03tier
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "tiered or c3_interpreter" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -5 $OUT/tests.log
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['config']['kernels'], d['config'].get('tiered'), d.get('latency_ms_single'))"
