# k_mpu shape experiments on the default bench (ms/step): S2 walk width via PSGPU_S2N (JIT flag)
mkdir -p gpurun_out; o=gpurun_out/mv.txt; : > $o
for s2 in ${S2N_LIST:-"4 2"}; do
  echo "S2N=$s2" >> $o
  PSGPU_S2N=$s2 timeout -k 10 150 python -u bench.py --no-cpu > gpurun_out/mv1.json 2>>$o || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/mv1.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], r['kernels_ms'])" >> $o
done
