set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or random_trees or capacity or c3" > $O/parity.log 2>&1 || { echo parity failed; exit 1; }
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/new_$i.json 2> $O/new_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_FIN_TRI_PREFETCH=0 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --engines 1 --steps 200 --warmup 20 > $O/new1e_$i.json 2> $O/new1e_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_FIN_TRI_PREFETCH=0 timeout -k 10 200 python -u bench.py --engines 1 --steps 200 --warmup 20 > $O/old1e_$i.json 2> $O/old1e_$i.err || exit 1
done
