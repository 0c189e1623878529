# k_finish / k_vertex persistent grids (blocks per CU) with 4 engines, on the driver's 20-step
# window and at 200 steps, interleaved fresh processes on one box
set -o pipefail
O=gpurun_out/r5grids
mkdir -p $O
run() {  # name, K, W, args
  timeout -k 10 200 python -u bench.py --steps $2 --warmup $3 --no-cpu --no-extras $4 > $O/$1_$2_$i.json 2> $O/$1_$2_$i.err
}
for i in 1 2 3 4; do
  for K in 20 200; do
    W=5; [ $K = 200 ] && W=20
    run f4v8 $K $W "" || exit 1
    run f8v8 $K $W "--finish-blocks 8" || exit 1
    run f6v8 $K $W "--finish-blocks 6" || exit 1
    run f8v16 $K $W "--finish-blocks 8 --vertex-blocks 16" || exit 1
    run f8v4 $K $W "--finish-blocks 8 --vertex-blocks 4" || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in (20, 200):
    for n in ("f4v8", "f8v8", "f6v8", "f8v16", "f8v4"):
        v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5grids/{n}_{K}_*.json"))]
        print(f"{n:6s} K {K:3d}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
