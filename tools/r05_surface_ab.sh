# k_vertex + k_finish as one launch for small launches (PSGPU_FUSED_SURFACE: 0 off, 2 auto, the
# default) on the C4 1/8-share rehearsal, interleaved, one box; then the C5 shares
set -o pipefail
O=gpurun_out/r5surf
mkdir -p $O
for i in 1 2 3; do
  for f in 0 2; do
    PSGPU_FUSED_SURFACE=$f SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f${f}_$i.txt 2>&1 || exit 1
    echo "C4 fused $f run $i: $(grep 'rebalance 2:' $O/c4_f${f}_$i.txt)"
  done
done
for f in 0 2; do
  PSGPU_FUSED_SURFACE=$f CONFIG=C5 SHARES=8 ENGINES=4 REBAL=1 JIT=1 TS=2 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $O/c5_f${f}.txt 2>&1 || exit 1
  echo "C5 fused $f: $(grep 'rebalance 1:' $O/c5_f${f}.txt)"
done
