#!/bin/bash
# Interleaved A/B of bench.py command lines on one box: REPS rounds, every variant once per
# round, a fresh process each (ms_per_step per run, then the median per variant).
# Usage (on the box): bash tools/bench_ab.sh TAG REPS "label|bench args[|ENV=val;ENV2=val two]" ...
# e.g. bash tools/bench_ab.sh ab 3 "s|--jit 1 --steps 200" "b|--jit 2 --steps 200"
set -o pipefail
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
: > $OUT/ab.txt
for r in $(seq $REPS); do
  for v in "$@"; do
    IFS='|' read -r label args envs <<< "$v"
    IFS=';' read -ra E <<< "$envs"
    f=$OUT/${label}_$r.json
    env "${E[@]}" timeout -k 10 240 python3 bench.py --no-cpu --no-extras $args > $f 2> $OUT/${label}_$r.err || { echo "FAILED $label $r"; tail -5 $OUT/${label}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$f'));t=d['config'].get('tiered',{}).get('structure_kernels',{}).get('ms_per_step');k=d.get('kernel_ms_per_launch_isolated',{});print('$label', $r, d['ms_per_step'], 'structure_pass', t, 'isolated', ' '.join('%s=%.1f'%(a[2:],b*1e3) for a,b in k.items()))" | tee -a $OUT/ab.txt
  done
done
python3 - "$OUT/ab.txt" <<'EOF'
import collections, statistics, sys
v = collections.defaultdict(list)
for line in open(sys.argv[1]):
    p = line.split()
    v[p[0]].append(float(p[2]))
for k, x in v.items():
    print(f"{k:20s} median {statistics.median(x):.4f} ms/step  min {min(x):.4f}  max {max(x):.4f}  n={len(x)}")
EOF
