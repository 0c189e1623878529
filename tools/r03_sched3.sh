#!/bin/bash
# Structure-tier scheduler / optimisation flags (PSGPU_JIT_FLAGS; --jit 1 so only the
# structure kernels run): C5 (the animation's kernels) and C3 4 engines, 2 rounds.  Stops at
# the first failure.
set -o pipefail
OUT=gpurun_out/${1:-sched3}
mkdir -p $OUT
export TMPDIR=/tmp
declare -A V
V[default]=""
V[bias0]="-mllvm -amdgpu-schedule-metric-bias=0"
V[itmaxocc]="-mllvm -amdgpu-sched-strategy=iterative-maxocc"
V[itminreg]="-mllvm -amdgpu-sched-strategy=iterative-minreg"
V[relaxocc]="-mllvm -amdgpu-schedule-relaxed-occupancy"
V[O3]="-O3"
for i in 1 2; do
  for v in default bias0 itmaxocc itminreg relaxocc O3; do
    PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --config C5 --jit 1 --no-cpu --no-extras --steps 100 > $OUT/c5_${v}_$i.json 2> $OUT/c5_${v}_$i.err || { tail -5 $OUT/c5_${v}_$i.err; exit 1; }
    PSGPU_JIT_FLAGS="${V[$v]}" timeout -k 10 300 python3 bench.py --jit 1 --no-cpu --no-extras > $OUT/c3_${v}_$i.json 2> $OUT/c3_${v}_$i.err || { tail -5 $OUT/c3_${v}_$i.err; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/c5_${v}_$i.json')); b=json.load(open('$OUT/c3_${v}_$i.json')); print('$v C5', a['ms_per_step'], 'C3 structure', b['ms_per_step'])"
  done
done
