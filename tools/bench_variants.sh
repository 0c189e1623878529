# bench.py under several engine / hardware-queue settings (ms_per_step, queues)
mkdir -p gpurun_out; o=gpurun_out/bv.txt; : > $o
IFS=';' read -ra VS <<< "${VARIANTS:---engines 4;--engines 2 --hw-queues 4}"
for a in "${VS[@]}"; do
  echo "$a" >> $o
  timeout -k 10 150 python -u bench.py --no-cpu $a > gpurun_out/bv1.json 2>>$o || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bv1.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['ms_per_step'], d['config']['hw_queues'], r['kernel'], r['frac'], r.get('isolated',{}).get('frac'), r['kernels_ms'])" >> $o
done
