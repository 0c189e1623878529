# Fitted k_vertex / k_finish grids (PSGPU_GRID_FIT) across the workloads, interleaved fresh
# processes on one box: 4 engines 200 steps, the driver's 20, one engine, C5, the C4 1/8 shares
set -o pipefail
O=gpurun_out/r5fit2
mkdir -p $O
for i in 1 2 3; do
  for f in 0 1; do
    PSGPU_GRID_FIT=$f timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu > $O/f${f}_200_$i.json 2> $O/f${f}_200_$i.err || exit 1
    PSGPU_GRID_FIT=$f timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras > $O/f${f}_20_$i.json 2> $O/f${f}_20_$i.err || exit 1
    PSGPU_GRID_FIT=$f timeout -k 10 200 python -u bench.py --engines 1 --steps 200 --warmup 20 --no-cpu --no-extras > $O/f${f}_e1_$i.json 2> $O/f${f}_e1_$i.err || exit 1
    PSGPU_GRID_FIT=$f timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 8 --no-cpu --no-extras > $O/f${f}_c5_$i.json 2> $O/f${f}_c5_$i.err || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for K in ("200", "20", "e1", "c5"):
    for f in (0, 1):
        d = [json.load(open(x)) for x in sorted(glob.glob(f"gpurun_out/r5fit2/f{f}_{K}_*.json"))]
        v = [x["ms_per_step"] for x in d]
        line = f"{K:4s} GRID_FIT={f}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}"
        if K == "200":
            line += " | single " + " ".join(f"{x['latency_ms_single']['median']:.4f}" for x in d)
            line += " | parts " + " ".join(f"{x['latency_ms_single_parts']['median']:.4f}" for x in d)
        print(line)
PY
for i in 1 2; do
  for f in 0 1; do
    PSGPU_GRID_FIT=$f SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f${f}_$i.txt 2>&1 || exit 1
    echo "C4 GRID_FIT=$f run $i: $(grep 'rebalance 2:' $O/c4_f${f}_$i.txt)"
  done
done
