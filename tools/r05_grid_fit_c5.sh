# Fitted grids on C5 (512^3, 64 primitives): the animated bench frames (200 steps) and the
# static frame's full grid and 1/8 shares (tools/range_test.py), interleaved, one box
set -o pipefail
O=gpurun_out/r5fit3
mkdir -p $O
for i in 1 2 3; do
  for f in 0 1; do
    PSGPU_GRID_FIT=$f timeout -k 10 300 python -u bench.py --config C5 --steps 200 --warmup 20 --no-cpu --no-extras > $O/f${f}_c5_$i.json 2> $O/f${f}_c5_$i.err || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for f in (0, 1):
    v = [json.load(open(x))["ms_per_step"] for x in sorted(glob.glob(f"gpurun_out/r5fit3/f{f}_c5_*.json"))]
    print(f"C5 bench 200 frames GRID_FIT={f}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
for i in 1 2; do
  for f in 0 1; do
    PSGPU_GRID_FIT=$f CONFIG=C5 SHARES=1,8 ENGINES=4 REBAL=1 JIT=1 TS=2 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $O/c5r_f${f}_$i.txt 2>&1 || exit 1
    echo "C5 static GRID_FIT=$f run $i: $(grep 'share 1/1' $O/c5r_f${f}_$i.txt | head -1 | sed 's/.*q=8//') | $(grep 'rebalance 1:' $O/c5r_f${f}_$i.txt)"
  done
done
