#!/bin/bash
# A/B: compat-mode generated kernels with / without packed fp32 (PSGUI_JIT_PACKED=1 keeps it),
# train scene at three cell sizes, twice; then the compat GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-guipk}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in 1 0; do
    PSGUI_JIT=2 PSGUI_JIT_PACKED=$v timeout -k 10 300 python3 tools/gui_bench.py 0.13 0.05 0.03 --no-cpu > $OUT/g_pk$v_$i.jsonl 2> $OUT/g_pk${v}_$i.err || { tail -20 $OUT/g_pk${v}_$i.err; exit 1; }
    python3 -c "import json; print('packed=$v', [json.loads(l)['gpu_ms'] for l in open('$OUT/g_pk$v_$i.jsonl')])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gui.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gui_tests.log 2>&1 || { tail -30 $OUT/gui_tests.log; exit 1; }
tail -2 $OUT/gui_tests.log
