#!/bin/bash
# Instruction-mix / stall PMC passes of the bench workload (one --pmc set per pass,
# --kernel-trace only beside it).  Usage: bash tools/pmc_round.sh TAG
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_LEVEL_WAVES"
P3="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_IFETCH SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"
P4="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VSKIPPED"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 $BENCH_ARGS > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/p*/run_counter_collection.csv
