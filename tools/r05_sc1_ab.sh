# k_mpu's records stored with sc1 (PSGPU_REC_SC1) A/B on one box: parity with it first, then the
# lone per-wave timeline (kernel gaps), and interleaved fresh bench processes
set -o pipefail
O=gpurun_out/r5sc1
mkdir -p $O
PSGPU_JIT_FLAGS="-DPSGPU_REC_SC1=1" timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or engines or random_trees" > $O/parity.log 2>&1 || { echo parity failed; tail -30 $O/parity.log; exit 1; }
for m in 0 1; do
  PSGPU_JIT_FLAGS="-DPSGPU_REC_SC1=$m" timeout -k 10 200 python -u tools/timeline.py > $O/tl_$m.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for m in 0 1; do
    PSGPU_JIT_FLAGS="-DPSGPU_REC_SC1=$m" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu > $O/s${m}_200_$i.json 2> $O/s${m}_200_$i.err || exit 1
    PSGPU_JIT_FLAGS="-DPSGPU_REC_SC1=$m" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/s${m}_20_$i.json 2> $O/s${m}_20_$i.err || exit 1
  done
done
for m in 0 1; do echo "## timeline SC1=$m"; grep -E "^k_" $O/tl_$m.txt; done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for m in (0, 1):
        d = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/r5sc1/s{m}_{K}_*.json"))]
        v = [x["ms_per_step"] for x in d]
        line = f"K {K:3d} SC1={m}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}"
        if K == 200:
            iso = [x["kernel_ms_per_launch_isolated"]["k_mpu"] for x in d]
            lat = [x["latency_ms_single"]["median"] for x in d]
            line += f" | k_mpu isolated {' '.join(f'{x:.4f}' for x in iso)} | single {' '.join(f'{x:.4f}' for x in lat)}"
        print(line)
PY
