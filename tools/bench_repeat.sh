# the headline bench N times on one box (ms_per_step each): run-to-run spread
mkdir -p gpurun_out; o=gpurun_out/rep.txt; : > $o
for i in $(seq ${N:-5}); do
  timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/rep1.json 2>>$o || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/rep1.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])" >> $o
done
