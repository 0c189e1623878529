#!/bin/bash
# The default bench line with a cold JIT code-object cache (as on a fresh box): the
# structure kernels and then the baked ones compile inside the run.
set -o pipefail
OUT=gpurun_out/r03cold
mkdir -p $OUT
export TMPDIR=/tmp
export PSGPU_JIT_CACHE=$(mktemp -d)
s=$(date +%s)
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
e=$(date +%s)
echo "wall $((e - s)) s"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['config']['jit_ready_s'], d['config']['tiered']['baked_ready_s'], d['config']['tiered']['structure_kernels'])"
