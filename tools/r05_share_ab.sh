# PSGPU_SHARE A/B (one box): parity with shared model / tables first, then interleaved fresh
# processes, 200-step and the driver's 20-step window, base vs model (1), tables (2), both (3)
set -o pipefail
O=gpurun_out/r5share
mkdir -p $O
PSGPU_SHARE=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or engines or random_trees" > $O/parity_share.log 2>&1 || { echo parity failed; exit 1; }
for i in 1 2 3; do
  for s in 0 1 2 3; do
    PSGPU_SHARE=$s timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu --no-extras > $O/s${s}_200_$i.json 2> $O/s${s}_200_$i.err || exit 1
    PSGPU_SHARE=$s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/s${s}_20_$i.json 2> $O/s${s}_20_$i.err || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for s in range(4):
        v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5share/s{s}_{K}_*.json"))]
        print(f"K {K:3d} PSGPU_SHARE={s}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
