set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d gpurun_out/ic/p1 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/ic/p1.log 2>&1 || { tail -5 gpurun_out/ic/p1.log; exit 1; }
python3 tools/pmc.py gpurun_out/ic > gpurun_out/ic/pmc.json
python3 -c "
import json;d=json.load(open('gpurun_out/ic/pmc.json'))
for k,v in d['kernels'].items(): print(k, {a:round(b,1) for a,b in v.items() if a.startswith('SQ')})
"
