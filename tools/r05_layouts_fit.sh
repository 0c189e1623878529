# k_finish / k_vertex layouts with the fitted grids (the default since late r05), 4 engines,
# 200 steps and the driver's 20, interleaved fresh processes on one box
set -o pipefail
O=gpurun_out/r5lay
mkdir -p $O
run() {  # name, K, W, env
  env $4 timeout -k 10 200 python -u bench.py --steps $2 --warmup $3 --no-cpu --no-extras > $O/$1_$2_$i.json 2> $O/$1_$2_$i.err
}
for i in 1 2 3; do
  for K in 200 20; do
    W=5; [ $K = 200 ] && W=20
    run auto $K $W "PSGPU_X=0" || exit 1
    run fpair $K $W "PSGPU_FINISH_QUAD=3" || exit 1
    run fquad $K $W "PSGPU_FINISH_QUAD=1" || exit 1
    run vquad $K $W "PSGPU_VERTEX_WIDE=0" || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for n in ("auto", "fpair", "fquad", "vquad"):
        v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5lay/{n}_{K}_*.json"))]
        print(f"{n:6s} K {K:3d}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
