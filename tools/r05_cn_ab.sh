# pass 1's crossNtri from LDS (PSGPU_MPU_CN_LDS) A/B on one box, and the C4 1/8-share
# rehearsal with the tree-split k_mpu launched with 2 MPUs' LDS per block (7 waves per SIMD)
set -o pipefail
O=gpurun_out/r5cn
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or engines or random_trees or split" > $O/parity.log 2>&1 || { echo parity failed; tail -30 $O/parity.log; exit 1; }
for i in 1 2 3; do
  for m in 0 1; do
    PSGPU_JIT_FLAGS="-DPSGPU_MPU_CN_LDS=$m" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu > $O/c${m}_200_$i.json 2> $O/c${m}_200_$i.err || exit 1
  done
done
python - <<'PY'
import json, glob, statistics
for m in (0, 1):
    d = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/r5cn/c{m}_200_*.json"))]
    v = [x["ms_per_step"] for x in d]
    iso = [x["kernel_ms_per_launch_isolated"]["k_mpu"] for x in d]
    lat = [x["latency_ms_single"]["median"] for x in d]
    print(f"K 200 CN_LDS={m}: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f} | "
          f"k_mpu isolated {' '.join(f'{x:.4f}' for x in iso)} | single {' '.join(f'{x:.4f}' for x in lat)}")
PY
SHARES=1,8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 500 python3 -u tools/range_test.py > $O/c4_shares.txt 2>&1 || exit 1
grep "slowest" $O/c4_shares.txt
