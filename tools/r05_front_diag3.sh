# k_front cost split on C4 1/8 shares: off; on with write-through entries (bit 25); + slow
# polling (bit 26); + no barrier at all (bit 27: wrong output, timing of the fused kernel alone)
set -o pipefail
O=gpurun_out/r5frontd3
mkdir -p $O
for i in 1 2; do
  for v in "0 0" "1 33554432" "1 100663296" "1 167772160"; do
    set -- $v
    PSGPU_FUSED_FRONT=$1 DBG=$2 SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f$1_d$2_$i.txt 2>&1 || exit 1
    echo "C4 front $1 dbg $2 run $i: $(grep 'rebalance 2:' $O/c4_f$1_d$2_$i.txt)"
  done
done
grep -i "brick\|block\|queued" $O/c4_f0_d0_1.txt | head -5
