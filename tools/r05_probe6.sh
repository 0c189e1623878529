set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 200 python -u tools/window_timeline.py > $O/window.txt 2>&1 &&
timeout -k 10 240 python -u tools/engines_timeline.py --engines 4 --json $O/etl_base.json > $O/etl_base.txt 2>&1 &&
PSGPU_JIT_FLAGS=-DPSGPU_S2_GROUP=5 timeout -k 10 240 python -u tools/engines_timeline.py --engines 4 --json $O/etl_s2g5.json > $O/etl_s2g5.txt 2>&1 &&
timeout -k 10 200 python -u tools/timeline.py --phases > $O/mpu_phases.txt 2>&1
