# k_precheck + k_mpu as one launch (PSGPU_FUSED_FRONT: 0 off, 1 on for split runs): parity of
# the split-path suites with it on, then the C4 1/8-share rehearsal interleaved, one box; C5 shares
set -o pipefail
O=gpurun_out/r5front
mkdir -p $O
PSGPU_FUSED_FRONT=1 timeout -k 10 700 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_multi.py \
  -x -q --timeout 300 --timeout-method thread > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -3 $O/parity.txt
for i in 1 2 3; do
  for f in 0 1; do
    PSGPU_FUSED_FRONT=$f SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_f${f}_$i.txt 2>&1 || exit 1
    echo "C4 front $f run $i: $(grep 'rebalance 2:' $O/c4_f${f}_$i.txt)"
  done
done
for f in 0 1; do
  PSGPU_FUSED_FRONT=$f CONFIG=C5 SHARES=8 ENGINES=4 REBAL=1 JIT=1 TS=2 K=200 timeout -k 10 400 python3 -u tools/range_test.py > $O/c5_f${f}.txt 2>&1 || exit 1
  echo "C5 front $f: $(grep 'rebalance 1:' $O/c5_f${f}.txt)"
done
