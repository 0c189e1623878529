set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k"
PSGPU_JIT_FLAGS=-DPSGPU_S2_OCT=2 timeout -k 10 400 $T "golden or random_trees or c5 or scene or max_size or disc_ring" > $O/parity_oct2.log 2>&1 || { echo parity oct2 failed; tail -30 $O/parity_oct2.log; exit 1; }
PSGPU_JIT_FLAGS=-DPSGPU_S2_OCT=1 timeout -k 10 400 $T "golden or random_trees" > $O/parity_oct1.log 2>&1 || { echo parity oct1 failed; tail -30 $O/parity_oct1.log; exit 1; }
B="python -u bench.py --steps 200 --warmup 20 --no-cpu"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/base_$i.json 2> $O/base_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_S2_OCT=2 timeout -k 10 200 $B > $O/oct2_$i.json 2> $O/oct2_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_S2_OCT=1 timeout -k 10 200 $B > $O/oct1_$i.json 2> $O/oct1_$i.err || exit 1
done
