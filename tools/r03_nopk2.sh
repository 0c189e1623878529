#!/bin/bash
# A/B of packed fp32 per generated kernel: the kernels' attribute hooks
# (PSGPU_{PRE,MPU,VTX,FIN}_ATTR) take __attribute__((target("no-packed-fp32-ops"))).
# C3 (structure pass and baked tier in one line) and C5 (structure kernels), one box.
set -o pipefail
OUT=gpurun_out/${1:-nopk2}
mkdir -p $OUT
export TMPDIR=/tmp
A='__attribute__((target("no-packed-fp32-ops")))'
declare -A V
V[pk]=""
V[all]="-DPSGPU_PRE_ATTR=$A -DPSGPU_MPU_ATTR=$A -DPSGPU_VTX_ATTR=$A -DPSGPU_FIN_ATTR=$A"
V[nopre]="-DPSGPU_MPU_ATTR=$A -DPSGPU_VTX_ATTR=$A -DPSGPU_FIN_ATTR=$A"
V[mpu]="-DPSGPU_MPU_ATTR=$A"
V[mpufin]="-DPSGPU_MPU_ATTR=$A -DPSGPU_FIN_ATTR=$A"
for i in 1 2; do
  for v in pk all nopre mpu mpufin; do
    PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --no-cpu --no-extras > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err || { tail -20 $OUT/c3_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_$v$i.json')); print('C3 $v baked', d['ms_per_step'], 'structure', d['config']['tiered']['structure_kernels']['ms_per_step'], d['kernel_ms_per_launch_isolated'])"
  done
done
for v in pk all nopre; do
  PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 100 > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -20 $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('C5 $v', d['ms_per_step'], d['kernel_ms_per_launch_isolated'])"
done
