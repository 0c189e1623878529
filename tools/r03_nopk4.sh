#!/bin/bash
# Baked tier: lone / small-launch variants without packed fp32 (the default 'ff f0') vs
# packed everywhere ('ff 00') vs none ('ff ff'): C3 4 engines and 1 engine, 3 rounds; the
# 1/8 shares (tree split, 2 rebalancing rounds) for the first two.  One box.
set -o pipefail
OUT=gpurun_out/${1:-nopk4}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in "ff f0" "ff 00" "ff ff"; do
    t=$(echo $v | tr -d ' ')
    for e in 4 1; do
      PSGPU_JIT_NOPK="$v" timeout -k 10 300 python3 bench.py --no-cpu --no-extras --engines $e > $OUT/c3_${t}_e${e}_$i.json 2> $OUT/c3_${t}_e${e}_$i.err || { tail -20 $OUT/c3_${t}_e${e}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/c3_${t}_e${e}_$i.json')); print('C3 nopk=$t engines $e baked', d['ms_per_step'], 'structure', d['config']['tiered']['structure_kernels']['ms_per_step'])"
    done
  done
done
for v in "ff f0" "ff 00"; do
  t=$(echo $v | tr -d ' ')
  PSGPU_JIT_NOPK="$v" CONFIG=C3 JIT=2 TS=2 SHARES=8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/share8_$t.txt 2>&1 || { tail -5 $OUT/share8_$t.txt; exit 1; }
  echo "== $t"; grep "slowest" $OUT/share8_$t.txt
done
