# k_front with the per-shard done counts (one frontDone add per shard, not per block): parity
# of the split-path suites with it on, then C4 1/8 shares: off, on, on with write-through queue
# entries and a wait instead of the L2 write-back (debug bit 25)
set -o pipefail
O=gpurun_out/r5frontd2
mkdir -p $O
PSGPU_FUSED_FRONT=1 timeout -k 10 700 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py \
  -x -q --timeout 300 --timeout-method thread > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
for i in 1 2 3; do
  for v in "0 0" "1 0" "1 33554432"; do
    set -- $v
    PSGPU_FUSED_FRONT=$1 DBG=$2 SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f$1_d$2_$i.txt 2>&1 || exit 1
    echo "C4 front $1 dbg $2 run $i: $(grep 'rebalance 2:' $O/c4_f$1_d$2_$i.txt)"
  done
done
