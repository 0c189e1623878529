set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
PSGPU_GRID_FIT=1 PSGPU_MPU_MARGIN=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or engines or random_trees or capacity" > $O/parity_fit.log 2>&1 || { echo parity failed; exit 1; }
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/base_$i.json 2> $O/base_$i.err &&
  PSGPU_GRID_FIT=1 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/fit_$i.json 2> $O/fit_$i.err &&
  PSGPU_GRID_FIT=1 PSGPU_MPU_MARGIN=32 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/fitm_$i.json 2> $O/fitm_$i.err || exit 1
done
