#!/bin/bash
# Interleaved A/B of the strong-scaling rehearsal (tools/range_test.py: one rank's share of a
# config, 4 engines, rebalanced) on one box: REPS rounds, every variant once per round, a fresh
# process each; prints each run's "rebalance" line and the median of the slowest rank per variant.
# Usage (on the box): bash tools/shares_ab.sh TAG REPS "BASE_ENV" "label|ENV=a;ENV2=b" ...
#   BASE_ENV: the rehearsal's settings, e.g. "SHARES=8;ENGINES=4;REBAL=2;JIT=1;TS=2;K=400"
# e.g. bash tools/shares_ab.sh r06front 3 "SHARES=8;ENGINES=4;REBAL=2;JIT=1;TS=2;K=400" "f0|PSGPU_FRONT=0" "f2|PSGPU_FRONT=2"
set -o pipefail
TAG=$1; REPS=$2; BASE=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
: > $OUT/ab.txt
IFS=';' read -ra B <<< "$BASE"
REB=$(printf '%s\n' "${B[@]}" | sed -n 's/^REBAL=//p'); REB=${REB:-0}
for r in $(seq $REPS); do
  for v in "$@"; do
    IFS='|' read -r label envs <<< "$v"
    IFS=';' read -ra E <<< "$envs"
    f=$OUT/${label}_$r.txt
    env "${B[@]}" "${E[@]}" timeout -k 10 300 python3 -u tools/range_test.py > $f 2>&1 || { echo "FAILED $label $r"; tail -5 $f; exit 1; }
    line=$(grep "rebalance $REB:" $f | tail -1)
    [ -z "$line" ] && line=$(grep "slowest rank" $f | tail -1)
    echo "$label $r $line" | tee -a $OUT/ab.txt
  done
done
python3 - "$OUT/ab.txt" <<'EOF'
import collections, re, statistics, sys
v = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.search(r"slowest rank ([0-9.]+)", line)
    if m:
        v[line.split()[0]].append(float(m.group(1)))
for k, x in v.items():
    print(f"{k:12s} slowest-rank median {statistics.median(x):.4f} ms/step  min {min(x):.4f}  max {max(x):.4f}  n={len(x)}")
EOF
