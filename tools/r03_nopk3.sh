#!/bin/bash
# Packed-fp32 policy of the baked tier (PSGPU_JIT_NOPK="structure baked" hex masks, bit k:
# precheck, mpu, vertex, finish): C3 4 engines and 1 engine, 3 rounds, one box; then the GPU
# parity tests on the default policy.  Usage: bash tools/r03_nopk3.sh TAG [notests]
set -o pipefail
OUT=gpurun_out/${1:-nopk3}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in "f 0" "f f" "f 2" "f e"; do
    t=$(echo $v | tr -d ' ')
    for e in 4 1; do
      PSGPU_JIT_NOPK="$v" timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $e > $OUT/c3_${t}_e$e_$i.json 2> $OUT/c3_${t}_e${e}_$i.err || { tail -20 $OUT/c3_${t}_e${e}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c3_${t}_e$e_$i.json')); print('C3 nopk=$t engines $e baked', d['ms_per_step'], 'structure', d['config']['tiered']['structure_kernels']['ms_per_step'])"
    done
  done
done
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
