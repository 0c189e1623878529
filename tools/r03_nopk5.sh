#!/bin/bash
# Baked tier: the default mask ('ff f0') vs also dropping packed fp32 in the throughput k_vertex
# ('ff f4') or k_finish ('ff f8'); C3 4 engines, 3 rounds.  Stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-nopk5}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in "ff f0" "ff f4" "ff f8"; do
    t=$(echo $v | tr -d ' ')
    PSGPU_JIT_NOPK="$v" timeout -k 10 300 python3 bench.py --no-cpu --no-extras > $OUT/c3_${t}_$i.json 2> $OUT/c3_${t}_$i.err || { tail -5 $OUT/c3_${t}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_${t}_$i.json')); print('C3 nopk=$t baked', d['ms_per_step'])"
  done
done
