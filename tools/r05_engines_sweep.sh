# engines per device (4 default) x hardware queues, 200 steps and the driver's 20, interleaved
# fresh processes on one box
set -o pipefail
O=gpurun_out/r5eng
mkdir -p $O
run() {  # name, K, W, args
  timeout -k 10 200 python -u bench.py --steps $2 --warmup $3 --no-cpu --no-extras $4 > $O/$1_$2_$i.json 2> $O/$1_$2_$i.err
}
for i in 1 2 3; do
  for K in 200 20; do
    W=5; [ $K = 200 ] && W=20
    run e4q8 $K $W "--engines 4" || exit 1
    run e5q8 $K $W "--engines 5" || exit 1
    run e6q8 $K $W "--engines 6" || exit 1
    run e6q12 $K $W "--engines 6 --hw-queues 12" || exit 1
    run e8q16 $K $W "--engines 8 --hw-queues 16" || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for n in ("e4q8", "e5q8", "e6q8", "e6q12", "e8q16"):
        v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5eng/{n}_{K}_*.json"))]
        print(f"{n:6s} K {K:3d}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
