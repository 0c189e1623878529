#!/bin/bash
# Interleaved A/B of the lone-caller latency (bench.py's latency_ms_single / _parts: one
# polygonization waited for) under environment / argument variants, REPS rounds, one box.
# Usage (on the box): bash tools/latency_ab.sh TAG REPS "label|bench args|ENV=a;ENV2=b" ...
set -o pipefail
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq $REPS); do
  for v in "$@"; do
    IFS='|' read -r label args envs <<< "$v"
    IFS=';' read -ra E <<< "$envs"
    f=$OUT/${label}_$r.json
    env "${E[@]}" timeout -k 10 300 python3 bench.py --no-cpu --steps 20 --warmup 5 $args > $f 2> $OUT/${label}_$r.err || { echo "FAILED $label"; tail -5 $OUT/${label}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));a=d['latency_ms_single'];b=d['latency_ms_single_parts'];print('$label', $r, 'single', a['median'], a['best'], 'parts', b['median'], b['best'], 'step', d['ms_per_step'])"
  done
done
