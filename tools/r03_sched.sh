#!/bin/bash
# A/B of the generated kernels' machine scheduler (PSGPU_JIT_FLAGS -mllvm options):
# C3 4 engines and 1 engine (baked and structure passes in each line), 2 rounds; C5 once.
set -o pipefail
OUT=gpurun_out/${1:-sched}
mkdir -p $OUT
export TMPDIR=/tmp
declare -A V
V[default]=""
V[maxilp]="-mllvm -amdgpu-sched-strategy=max-ilp"
V[itmaxocc]="-mllvm -amdgpu-sched-strategy=iterative-maxocc"
V[itilp]="-mllvm -amdgpu-sched-strategy=iterative-ilp"
V[bias0]="-mllvm -amdgpu-schedule-metric-bias=0"
for i in 1 2; do
  for v in default maxilp itmaxocc itilp bias0; do
    for e in 4 1; do
      PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $e > $OUT/c3_${v}_e${e}_$i.json 2> $OUT/c3_${v}_e${e}_$i.err || { tail -5 $OUT/c3_${v}_e${e}_$i.err; echo "C3 $v engines $e FAILED"; continue; }
      python3 -c "import json; d=json.load(open('$OUT/c3_${v}_e${e}_$i.json')); print('C3 $v engines $e baked', d['ms_per_step'], 'structure', d['config']['tiered']['structure_kernels']['ms_per_step'])"
    done
  done
done
for v in default maxilp itmaxocc itilp bias0; do
  PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 100 > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail -5 $OUT/c5_$v.err; echo "C5 $v FAILED"; continue; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('C5 $v', d['ms_per_step'])"
done
