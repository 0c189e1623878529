#!/bin/bash
# PMC passes over the bench command (one rocprofv3 run per counter set, --kernel-trace only),
# summarised per kernel by tools/pmc.py.  Usage on the box: bash tools/pmc.sh TAG JIT [bench args]
# (JIT: the bench's --jit, recorded in the summary)
set -o pipefail
TAG=${1:-pmc}; shift
JIT=${1:-2}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --jit $JIT $*"
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc.py $OUT $JIT > $OUT/pmc.json && cat $OUT/pmc.json
