#!/bin/bash
# Strong-scaling rehearsal after the packed-fp32 policy: C3/C4 1/1 and 1/8 shares (4 engines,
# tree split TS=2, 2 rebalancing rounds) on the baked tier (packed), the baked tier without
# packed fp32, and the structure tier (without packed fp32); C5 1/1 and 1/8 on the structure
# tier (an animation's kernels).
set -o pipefail
OUT=gpurun_out/${1:-nopkshares}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" TS=2 SHARES=1,8 REBAL=2 ENGINES=4 VB=8 FB=4 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $OUT/$tag.txt 2>&1 || { tail -5 $OUT/$tag.txt; exit 1; }
  echo "== $tag"; grep "slowest\|1/1" $OUT/$tag.txt
}
run c3_baked_pk CONFIG=C3 JIT=2 || exit 1
run c3_baked_nopk CONFIG=C3 JIT=2 PSGPU_JIT_NOPK="f f" || exit 1
run c3_structure CONFIG=C3 JIT=1 || exit 1
run c5_structure CONFIG=C5 JIT=1 || exit 1
