# k_mpu waves per MPU at strong-scaling rank shares: tools/range_test.py with each library
# variant (built beforehand as in tools/mpu_waves.sh and copied to exp/lib_w<w>.so).
mkdir -p gpurun_out; o=gpurun_out/mws.txt; : > $o
cp parsip_amd/libparsip_gpu.so exp/lib_default.so
for w in ${WAVES:-1 2 4}; do
  cp exp/lib_w$w.so parsip_amd/libparsip_gpu.so
  echo "W=$w" >> $o
  GPU_MAX_HW_QUEUES=8 ENGINES=${ENGINES:-4} SHARES=${SHARES:-8,4,1} timeout -k 10 120 python -u tools/range_test.py >> $o 2>&1 || exit 1
done
cp exp/lib_default.so parsip_amd/libparsip_gpu.so
