#!/bin/bash
# Baked-tier variants around the default (iterative max-occupancy scheduler, packed fp32 in the
# throughput kernels): + no packed fp32 anywhere, iterative min-reg, max-occupancy bias.
# C3 4 and 1 engines, 3 rounds.  Stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-sched4}
mkdir -p $OUT
export TMPDIR=/tmp
IT="-mllvm -amdgpu-sched-strategy=iterative-maxocc"
for i in 1 2 3; do
  for v in default nopk minreg bias100; do
    unset PSGPU_JIT_BAKED_FLAGS PSGPU_JIT_NOPK
    case $v in
      nopk) export PSGPU_JIT_NOPK="ff ff" ;;
      minreg) export PSGPU_JIT_BAKED_FLAGS="-mllvm -amdgpu-sched-strategy=iterative-minreg" ;;
      bias100) export PSGPU_JIT_BAKED_FLAGS="$IT -mllvm -amdgpu-schedule-metric-bias=100" ;;
    esac
    for e in 4 1; do
      timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $e > $OUT/c3_${v}_e${e}_$i.json 2> $OUT/c3_${v}_e${e}_$i.err || { tail -5 $OUT/c3_${v}_e${e}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c3_${v}_e${e}_$i.json')); print('C3 $v engines $e baked', d['ms_per_step'])"
    done
  done
done
