#!/bin/bash
# One GPU-box session: parity tests, smoke, then per kernel tier (--jit 2 baked, --jit 1
# structure) a kernel-trace profile of the driver's bench command, the FETCH_SIZE / WRITE_SIZE
# passes and the PMC sets (instruction mix, stalls, occupancy); then the driver's exact bench
# command, the long C3 line and the C5 frame.  Every GPU step has its own time limit; the first
# failure ends the script.
# Usage (from the repo root, on the box): bash tools/gpu_round.sh TAG [notests] [nogui] [JITS]
# (JITS: the tiers to profile, default "2 1"; e.g. "1" for the structure tier alone)
# Only gpurun_out/ comes back from the box: afterwards, here, run
#   bash tools/gpu_round.sh TAG --collect
# to copy the summaries into profiles/ (baked tier: TAG_{kernel_stats.csv,traffic,pmc}.json;
# structure tier: the same names with _structure).
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
if [ "$2" = "--collect" ]; then
  for J in 2 1; do
    SUF=""; [ $J = 1 ] && SUF="_structure"
    [ -f $OUT/j$J/kt/run_kernel_stats.csv ] && cp $OUT/j$J/kt/run_kernel_stats.csv profiles/${TAG}_kernel_stats$SUF.csv
    [ -f $OUT/j$J/traffic.json ] && cp $OUT/j$J/traffic.json profiles/${TAG}_traffic$SUF.json
    [ -f $OUT/j$J/pmc/pmc.json ] && cp $OUT/j$J/pmc/pmc.json profiles/${TAG}_pmc$SUF.json
  done
  for f in bench_driver.json bench.json bench_c5.json gui_bench.jsonl; do
    [ -f $OUT/$f ] && cp $OUT/$f profiles/${TAG}_$f
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
# the driver's command with the kernels of one tier pinned (--jit J), no CPU leg / extras
DRV="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extras"
for J in ${4:-2 1}; do
  D=$OUT/j$J
  mkdir -p $D
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- $DRV --jit $J > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $DRV --jit $J > $D/fetch.log 2>&1 || { tail -20 $D/fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $DRV --jit $J > $D/write.log 2>&1 || { tail -20 $D/write.log; exit 1; }
  python3 tools/traffic.py $D $J > $D/traffic.json || exit 1
  bash tools/pmc.sh $TAG/j$J/pmc $J > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
  SUF=""; [ $J = 1 ] && SUF="_structure"
  cp $D/traffic.json profiles/${TAG}_traffic$SUF.json && cp $D/pmc/pmc.json profiles/${TAG}_pmc$SUF.json || exit 1
done
# the bench lines, measured after the profiles so they report their traffic / VALU figures:
# the driver's exact command first
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
cat $OUT/bench_driver.json
timeout -k 10 400 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python3 bench.py --config C5 --no-cpu --no-extras --steps 200 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
[ "$3" = "nogui" ] && exit 0
# compat mode (the GUI path): the train scene at three cell sizes, generated kernels
PSGUI_JIT=2 timeout -k 10 300 python3 tools/gui_bench.py 0.13 0.05 0.03 > $OUT/gui_bench.jsonl 2> $OUT/gui_bench.err || { tail -20 $OUT/gui_bench.err; exit 1; }
cat $OUT/gui_bench.jsonl
