#!/bin/bash
# One GPU-box session: parity tests, smoke, a kernel-trace profile of the bench command (its
# kernels pinned to the baked ones, --jit 2: the tier the default --jit 3 times), PMC
# passes (FETCH_SIZE, WRITE_SIZE; instruction mix, stalls, occupancy), then the bench lines
# (C3 headline, C5 frame).  Every GPU step has its own time limit; the first failure ends the
# script.  Usage (from the repo root, on the box): bash tools/gpu_round.sh TAG [notests]
# Only gpurun_out/ comes back from the box: afterwards, here, run
#   bash tools/gpu_round.sh TAG --collect
# to copy the summaries into profiles/.
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
if [ "$2" = "--collect" ]; then
  for f in kernel_stats.csv traffic.json pmc.json bench.json bench_c5.json gui_bench.jsonl gui_kernel_stats.csv; do
    src=$OUT/$f; [ $f = kernel_stats.csv ] && src=$OUT/kt/run_kernel_stats.csv
    [ $f = pmc.json ] && src=$OUT/pmc/pmc.json
    [ $f = gui_kernel_stats.csv ] && src=$OUT/guikt/run_kernel_stats.csv
    [ -f $src ] && cp $src profiles/${TAG}_$f
  done
  exit 0
fi
mkdir -p $OUT profiles
export TMPDIR=/tmp
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu --no-extras --jit 2 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --jit 2 > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 1 --jit 2 > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
python3 tools/traffic.py $OUT > $OUT/traffic.json && cp $OUT/traffic.json profiles/${TAG}_traffic.json || exit 1
bash tools/pmc.sh $TAG/pmc --jit 2 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc.json profiles/${TAG}_pmc.json || exit 1
cp $OUT/kt/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
cat $OUT/traffic.json
# the bench lines, measured after the profiles so they report their traffic / VALU figures
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cp $OUT/bench.json profiles/${TAG}_bench.json
cat $OUT/bench.json
timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 200 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
# compat mode (the GUI path): the train scene at three cell sizes, generated kernels, and its
# kernel trace at cellsize 0.03
PSGUI_JIT=2 timeout -k 10 300 python3 tools/gui_bench.py 0.13 0.05 0.03 > $OUT/gui_bench.jsonl 2> $OUT/gui_bench.err || { tail -20 $OUT/gui_bench.err; exit 1; }
cat $OUT/gui_bench.jsonl
PSGUI_JIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/guikt -o run -- python3 tools/gui_bench.py 0.03 --no-cpu > $OUT/guikt.log 2>&1 || { tail -20 $OUT/guikt.log; exit 1; }
