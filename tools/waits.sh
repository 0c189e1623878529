#!/bin/bash
# Where the parked half of the waves' lives goes (verdict r05 item 4): PMC passes of the bench
# command per kernel variant, the kernels launched separately (PSGPU_FRONT=0, no tree split),
# rocprofv3 serialising the dispatches (every kernel isolated):
#   s   the structure kernels (--jit 1): per-primitive parameters through scalar loads
#   b   the baked kernels (--jit 2): the same walks with the parameters as literals
#   s1  --jit 1, debug bit 0: k_mpu stops after S2 (no record passes / LDS tables)
#   s32 --jit 1, debug bit 5: k_vertex / k_finish without their walks (loads, records, stores)
# Counters per pass (8 SQ at most): waves, wave cycles, WAIT_ANY (parked on s_waitcnt or a
# barrier), WAIT_INST_ANY, and the in-flight levels of vector / scalar / LDS memory
# instructions with their counts (LEVEL / INSTS = mean cycles an instruction of that class is
# outstanding), where the hardware has them (rocprofv3 -L).  Summary: tools/waits_summary.py.
# Usage (on the box): bash tools/waits.sh TAG
set -o pipefail
TAG=${1:-waits}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
have() { grep -qw "$1" $OUT/counters.txt; }
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS")
P2=""
for c in SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM; do
  if have $c && [ $(echo $P2 | wc -w) -lt 8 ]; then P2="$P2 $c"; fi
done
[ -n "$P2" ] && SETS+=("$P2")
echo "pass 2 counters:$P2"
for V in "s|--jit 1|0" "b|--jit 2|0" "s1|--jit 1|1" "s32|--jit 1|32"; do
  IFS='|' read -r name args dbg <<< "$V"
  mkdir -p $OUT/$name
  i=0
  for SET in "${SETS[@]}"; do
    i=$((i+1))
    PSGPU_FRONT=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/$name/p$i -o run -- \
      python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --tree-split 0 --debug $dbg $args > $OUT/$name/p$i.log 2>&1 \
      || { echo "$name pass $i failed"; tail -5 $OUT/$name/p$i.log; exit 1; }
  done
  python3 tools/pmc.py $OUT/$name > $OUT/$name.json || exit 1
done
python3 tools/waits_summary.py $OUT
