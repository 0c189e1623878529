#!/bin/bash
# Compact work records (8-B vertex roots and triangle records): GPU parity tests, the
# step's HBM traffic (FETCH_SIZE / WRITE_SIZE passes of the bench command, baked kernels)
# and the bench line.  Usage on the box: bash tools/r03_records.sh TAG [notests]
set -o pipefail
TAG=${1:-r03rec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --jit 2 > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --jit 2 > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
python3 tools/traffic.py $OUT > $OUT/traffic.json || exit 1
cat $OUT/traffic.json
# A/B on this box: the new records vs the previous build (tools/_bin/old, PSGPU_AB_LIB)
for i in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L=tools/_bin/old/libparsip_gpu.so
    PSGPU_AB_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-extras > $OUT/bench_${v}$i.json 2> $OUT/bench_${v}$i.err || { tail -20 $OUT/bench_${v}$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_${v}$i.json')); print('C3 $v', d['ms_per_step'], d['config']['tiered']['structure_kernels']['ms_per_step'], d['kernel_ms_per_launch_isolated'])"
  done
done
timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 200 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c5.json')); print('C5', d['ms_per_step'])"
