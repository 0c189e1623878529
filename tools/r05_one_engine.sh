# one engine (a single device context, or one 2-part group on 2 streams), steps queued back to
# back, 200 steps, interleaved fresh processes on one box
set -o pipefail
O=gpurun_out/r5one
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --engines 1 --steps 200 --warmup 20 --no-cpu --no-extras > $O/e1p1_$i.json 2> $O/e1p1_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --engines 1 --parts 2 --steps 200 --warmup 20 --no-cpu --no-extras > $O/e1p2_$i.json 2> $O/e1p2_$i.err || exit 1
done
python - <<'PY'
import json, glob, statistics
for n in ("e1p1", "e1p2"):
    v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5one/{n}_*.json"))]
    print(f"{n}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
