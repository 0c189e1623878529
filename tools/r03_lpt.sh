#!/bin/bash
# Heaviest-first S1-survivor queue (k_precheck weight classes) vs brick order (debug bit 21):
# parity subset, then C3 full grid (1 and 4 engines) and the 1/8 share, on the baked tier;
# per-kernel isolated spans from the bench line.
set -o pipefail
OUT=gpurun_out/r03lpt
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
for d in 0 2097152; do
  JIT=2 DBG=$d CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
grep "ms/step" $OUT/ab.txt | sed 's/FQ=- BD=- //; s/GR=- VW=- //'
timeout -k 10 300 python3 -u bench.py --no-cpu --no-extras > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu --no-extras --debug 2097152 > $OUT/bench_brick.json 2> $OUT/bench_brick.err || { tail -5 $OUT/bench_brick.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench", "bench_brick"):
    d = json.load(open(f"gpurun_out/r03lpt/{f}.json"))
    print(f, d["ms_per_step"], d["kernel_ms_per_launch_isolated"], d["kernel_ms_per_launch_hipevent"])
PY
