#!/bin/bash
# The baked tier's scheduler (default: iterative max-occupancy; PSGPU_JIT_BAKED_FLAGS=" "
# restores LLVM's default): C3 4 and 1 engines, 3 rounds; the 1/8 shares; then the GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-sched2}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in new old; do
    for e in 4 1; do
      if [ $v = old ]; then export PSGPU_JIT_BAKED_FLAGS=" "; else unset PSGPU_JIT_BAKED_FLAGS; fi
      timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $e > $OUT/c3_${v}_e${e}_$i.json 2> $OUT/c3_${v}_e${e}_$i.err || { tail -5 $OUT/c3_${v}_e${e}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c3_${v}_e${e}_$i.json')); print('C3 $v engines $e baked', d['ms_per_step'], 'structure', d['config']['tiered']['structure_kernels']['ms_per_step'])"
    done
  done
done
unset PSGPU_JIT_BAKED_FLAGS
for v in new old; do
  if [ $v = old ]; then export PSGPU_JIT_BAKED_FLAGS=" "; else unset PSGPU_JIT_BAKED_FLAGS; fi
  CONFIG=C3 JIT=2 TS=2 SHARES=8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/share8_$v.txt 2>&1 || { tail -5 $OUT/share8_$v.txt; exit 1; }
  echo "== $v"; grep "slowest" $OUT/share8_$v.txt
done
unset PSGPU_JIT_BAKED_FLAGS
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
