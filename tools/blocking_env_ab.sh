#!/bin/bash
# Interleaved A/B of the blocking contract (tools/blocking_seq.py, one-context C3 calls with the
# per-call phase trace) under environment variants.
# Usage (on the box): bash tools/blocking_env_ab.sh TAG REPS "label|ENV=a;ENV2=b" ...
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq $R); do
  for v in "$@"; do
    IFS='|' read -r label envs <<< "$v"
    IFS=';' read -ra E <<< "$envs"
    env CONFIGS=C3 GROUP=${GROUP:-0} REPS=24 "${E[@]}" timeout -k 10 200 python3 -u tools/blocking_seq.py > $OUT/${label}_$r.txt 2> $OUT/${label}_$r.trace || { tail -3 $OUT/${label}_$r.trace; exit 1; }
    echo "$label $r $(cut -c1-60 $OUT/${label}_$r.txt | tr '\n' ' ')"
  done
done
