# k_finish vertices per wave (PSGPU_FIN_VPW 64 / 16): GPU parity suite on the 16 variant, then
# the bench and the strong-scaling rank shares with each library (built here beforehand and
# copied to exp/lib_f<vpw>.so).  Results in gpurun_out/fin.txt.
mkdir -p gpurun_out; o=gpurun_out/fin.txt; : > $o
cp parsip_amd/libparsip_gpu.so exp/lib_default.so
if [ -z "$NOTEST" ]; then
  cp exp/lib_f16.so parsip_amd/libparsip_gpu.so
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin_tests.log 2>&1 || { tail -30 gpurun_out/fin_tests.log; exit 1; }
  tail -2 gpurun_out/fin_tests.log >> $o
fi
for v in ${VARIANTS:-16 64 16 64}; do
  cp exp/lib_f$v.so parsip_amd/libparsip_gpu.so
  echo "VPW=$v" >> $o
  timeout -k 10 200 python3 -u bench.py --no-cpu > gpurun_out/fin1.json 2>>$o || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/fin1.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r['kernels_ms']['k_finish'])" >> $o
  GPU_MAX_HW_QUEUES=8 ENGINES=4 SHARES=8,4 timeout -k 10 120 python3 -u tools/range_test.py >> $o 2>&1 || exit 1
done
cp exp/lib_default.so parsip_amd/libparsip_gpu.so
