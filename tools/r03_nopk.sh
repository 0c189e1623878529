#!/bin/bash
# A/B: the generated kernels with and without packed fp32 instructions (v_pk_add/mul_f32 and
# their hazard s_nops) -- PSGPU_JIT_FLAGS="-Xclang -target-feature -Xclang -packed-fp32-ops".
# C3 (baked tier) and C5 (structure kernels), alternating, twice each, on one box.
set -o pipefail
OUT=gpurun_out/${1:-nopk}
mkdir -p $OUT
export TMPDIR=/tmp
NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops"
for i in 1 2; do
  for v in pk nopk; do
    F=""; [ $v = nopk ] && F="$NOPK"
    PSGPU_JIT_FLAGS="$F" timeout -k 10 300 python3 bench.py --no-cpu --no-extras > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err || { tail -20 $OUT/c3_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_$v$i.json')); print('C3 $v', d['ms_per_step'], d['config']['tiered']['structure_kernels']['ms_per_step'], d['kernel_ms_per_launch_isolated'])"
  done
done
for i in 1 2; do
  for v in pk nopk; do
    F=""; [ $v = nopk ] && F="$NOPK"
    PSGPU_JIT_FLAGS="$F" timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 100 > $OUT/c5_$v$i.json 2> $OUT/c5_$v$i.err || { tail -20 $OUT/c5_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c5_$v$i.json')); print('C5 $v', d['ms_per_step'], d['kernel_ms_per_launch_isolated'])"
  done
done
