set -o pipefail
mkdir -p gpurun_out/r5a
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a
timeout -k 10 120 tools/_bin/fused_step_probe 2000 > $O/fused_probe.txt 2>&1 &&
timeout -k 10 240 python -u tools/engines_timeline.py --engines 4 --json $O/etl_base.json > $O/etl_base.txt 2>&1 &&
PSGPU_JIT_FLAGS=-DPSGPU_S2_GROUP=5 timeout -k 10 240 python -u tools/engines_timeline.py --engines 4 --json $O/etl_s2g5.json > $O/etl_s2g5.txt 2>&1 &&
timeout -k 10 240 python -u tools/engines_timeline.py --engines 1 --json $O/etl_one.json > $O/etl_one.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 > $O/bench_base_$i.json 2> $O/bench_base_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_S2_GROUP=5 timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 > $O/bench_s2g5_$i.json 2> $O/bench_s2g5_$i.err || exit 1
done
