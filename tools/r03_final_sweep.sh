#!/bin/bash
# Engines x hardware queues on the final kernels (C3, tiered: the baked pass is the value),
# twice.  Stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-fsweep}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for eq in "4 8" "5 12" "6 12" "3 8" "8 16"; do
    set -- $eq
    timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $1 --hw-queues $2 > $OUT/e$1q$2_$i.json 2> $OUT/e$1q$2_$i.err || { tail -5 $OUT/e$1q$2_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/e$1q$2_$i.json')); print('engines $1 queues $2', d['ms_per_step'], d['config']['tiered']['structure_kernels']['ms_per_step'])"
  done
done
