# k_mpu cell maps (PSGPU_MPU_MAPS) A/B on one box: GPU parity with the maps first, then
# interleaved fresh processes, the maps off (-DPSGPU_MPU_MAPS=0) vs on: 200 steps, the
# driver's 20, and the bench's isolated / single-polygonization figures
set -o pipefail
O=gpurun_out/r5maps
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > $O/parity.log 2>&1 || { echo parity failed; tail -30 $O/parity.log; exit 1; }
for i in 1 2 3; do
  for m in 0 1; do
    PSGPU_JIT_FLAGS="-DPSGPU_MPU_MAPS=$m" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu > $O/m${m}_200_$i.json 2> $O/m${m}_200_$i.err || exit 1
    PSGPU_JIT_FLAGS="-DPSGPU_MPU_MAPS=$m" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/m${m}_20_$i.json 2> $O/m${m}_20_$i.err || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for m in (0, 1):
        d = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/r5maps/m{m}_{K}_*.json"))]
        v = [x["ms_per_step"] for x in d]
        line = f"K {K:3d} MAPS={m}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}"
        if K == 200:
            iso = [x["kernel_ms_per_launch_isolated"]["k_mpu"] for x in d]
            lat = [x["latency_ms_single"]["median"] for x in d]
            line += f" | k_mpu isolated {' '.join(f'{x:.4f}' for x in iso)} | single {' '.join(f'{x:.4f}' for x in lat)}"
        print(line)
PY
