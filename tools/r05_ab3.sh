set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
B="python -u bench.py --engines 1 --steps 200 --warmup 20 --no-cpu --no-extras"
for i in 1 2; do
  timeout -k 10 120 $B > $O/base_$i.json 2> $O/base_$i.err &&
  PSGPU_FINISH_QUAD=1 timeout -k 10 120 $B --finish-blocks 32 > $O/q32_$i.json 2> $O/q32_$i.err &&
  PSGPU_FINISH_QUAD=1 timeout -k 10 120 $B --finish-blocks 32 --vertex-blocks 32 > $O/qv32_$i.json 2> $O/qv32_$i.err &&
  PSGPU_FINISH_QUAD=3 timeout -k 10 120 $B --finish-blocks 32 > $O/p32_$i.json 2> $O/p32_$i.err &&
  PSGPU_FINISH_QUAD=1 PSGPU_GRID_FIT=1 timeout -k 10 120 $B --finish-blocks 32 --vertex-blocks 32 > $O/qvfit_$i.json 2> $O/qvfit_$i.err || exit 1
done
