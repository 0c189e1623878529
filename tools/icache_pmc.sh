#!/bin/bash
# Instruction-fetch / scalar-cache counters per kernel under the bench command (verdict r02
# item 2): one rocprofv3 --pmc pass per counter set, --kernel-trace only, each under its own
# time limit; ENG=1 for the isolated regime (one engine), default the headline (4 engines).
# Usage on the box: bash tools/icache_pmc.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-ic}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 $*"
i=0
for SET in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAVES SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc.py $OUT > $OUT/pmc.json && python3 -c "
import json;d=json.load(open('$OUT/pmc.json'))
for k,v in d['kernels'].items(): print(k, {a:round(b,3) for a,b in v.items()})
"
