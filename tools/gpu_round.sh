#!/bin/bash
# One GPU-box session: parity tests, the bench line, a kernel-trace profile of the same
# bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic.
# Usage (from the repo root, on the box): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/valu -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > $OUT/valu.log 2>&1 || { tail -20 $OUT/valu.log; exit 1; }
python3 tools/valu.py $OUT/valu > $OUT/valu.json && cp $OUT/valu.json profiles/${TAG}_valu.json
python3 tools/traffic.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json && cp $OUT/traffic.json profiles/${TAG}_traffic.json && timeout -k 10 400 python3 bench.py > $OUT/bench2.json 2> $OUT/bench2.err; cat $OUT/bench2.json
