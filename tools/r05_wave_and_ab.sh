# The 64-vertex layouts' culling mask as one wave AND (PSGPU_CULL_WAVE_AND) vs one scalar load
# per distinct MPU: parity first, then k_finish's phases (the mask phase), and interleaved bench
# processes on one box
set -o pipefail
O=gpurun_out/r5wand
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "golden or layouts or random_trees or fuzz or engines" > $O/parity.log 2>&1 || { echo parity failed; tail -30 $O/parity.log; exit 1; }
for m in 0 1; do
  PSGPU_JIT_FLAGS="-DPSGPU_CULL_WAVE_AND=$m -DPSGPU_FIN_PHASES=1" timeout -k 10 200 python -u tools/timeline.py --finish > $O/fin_$m.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for m in 0 1; do
    PSGPU_JIT_FLAGS="-DPSGPU_CULL_WAVE_AND=$m" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu > $O/w${m}_200_$i.json 2> $O/w${m}_200_$i.err || exit 1
    PSGPU_JIT_FLAGS="-DPSGPU_CULL_WAVE_AND=$m" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/w${m}_20_$i.json 2> $O/w${m}_20_$i.err || exit 1
  done
done
for m in 0 1; do echo "## k_finish phases WAVE_AND=$m"; head -12 $O/fin_$m.txt; done
python - <<'PY'
import json, glob, statistics
for K in (200, 20):
    for m in (0, 1):
        d = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/r5wand/w{m}_{K}_*.json"))]
        v = [x["ms_per_step"] for x in d]
        line = f"K {K:3d} WAVE_AND={m}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}"
        if K == 200:
            iso = [x["kernel_ms_per_launch_isolated"] for x in d]
            line += " | isolated vertex " + " ".join(f"{x['k_vertex']:.4f}" for x in iso)
            line += " finish " + " ".join(f"{x['k_finish']:.4f}" for x in iso)
            line += " | single " + " ".join(f"{x['latency_ms_single']['median']:.4f}" for x in d)
        print(line)
PY
