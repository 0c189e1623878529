#!/bin/bash
# Occupancy hints per generated kernel (amdgpu_waves_per_eu through PSGPU_JIT_FLAGS: the
# compiler caps VGPRs at 512 / N) against the baseline and the baked-parameter kernels:
# C3 full grid with 1 and 4 engines, and the first 1/8 share with 4 engines; two rounds.
set -o pipefail
OUT=gpurun_out/r03occ
mkdir -p $OUT
export TMPDIR=/tmp
A='__attribute__((amdgpu_waves_per_eu'
for r in 1 2; do
for v in base mpu6 mpu8 fin8 pre8 baked; do
  F=""; J=1
  case $v in
    mpu6) F="-DPSGPU_MPU_ATTR=${A}(6)))";;
    mpu8) F="-DPSGPU_MPU_ATTR=${A}(8)))";;
    fin8) F="-DPSGPU_FIN_ATTR=${A}(8)))";;
    pre8) F="-DPSGPU_PRE_ATTR=${A}(8)))";;
    baked) J=2;;
  esac
  echo "== $v round $r" >> $OUT/ab.txt
  PSGPU_JIT_FLAGS="$F" JIT=$J CONFIG=C3 SHARES=1,8 ENGINES=1,4 VB=8 FB=4 K=400 timeout -k 10 200 python3 -u tools/range_test.py >> $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
done
done
cat $OUT/ab.txt
