# k_front timing diagnosis on the C4 1/8-share rehearsal: off, on, on without the queue release
# (debug bit 25: write-through entries and a wait, no L2 write-back), on with slow polling (bit 26), both
set -o pipefail
O=gpurun_out/r5frontd
mkdir -p $O
for i in 1 2; do
  for v in "0 0" "1 0" "1 33554432" "1 67108864" "1 100663296"; do
    set -- $v
    PSGPU_FUSED_FRONT=$1 DBG=$2 SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f$1_d$2_$i.txt 2>&1 || exit 1
    echo "C4 front $1 dbg $2 run $i: $(grep 'rebalance 2:' $O/c4_f$1_d$2_$i.txt)"
  done
done
