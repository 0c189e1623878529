#!/bin/bash
# Compat-mode GPU tests (PCM / Instance extended walk included).
set -o pipefail
OUT=gpurun_out/r03s2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gui.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gui_tests.log 2>&1 || { tail -40 $OUT/gui_tests.log; exit 1; }
tail -25 $OUT/gui_tests.log
