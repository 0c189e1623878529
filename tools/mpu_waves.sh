# k_mpu waves per MPU: the bench with each library variant (built here beforehand with
#   PSGPU_MPU_WAVES=<w> python -c "from parsip_amd import build; build.build(force=True)"
# and copied to exp/lib_w<w>.so).  WAVES="1 2 4" picks the order, BENCH_ARGS adds bench flags.
mkdir -p gpurun_out; o=gpurun_out/mw.txt; : > $o
cp parsip_amd/libparsip_gpu.so exp/lib_default.so
for w in ${WAVES:-1 2 4}; do
  cp exp/lib_w$w.so parsip_amd/libparsip_gpu.so
  echo "W=$w $BENCH_ARGS" >> $o
  timeout -k 10 200 python -u bench.py --no-cpu $BENCH_ARGS > gpurun_out/mw1.json 2>>$o || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/mw1.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r['kernels_ms']['k_mpu'])" >> $o
done
cp exp/lib_default.so parsip_amd/libparsip_gpu.so
