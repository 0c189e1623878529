set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
PSGPU_JIT_FLAGS=-DPSGPU_FIN_PHASES=1 timeout -k 10 200 python -u tools/timeline.py --finish > $O/finish_phases.txt 2>&1 &&
timeout -k 10 200 python -u tools/timeline.py --config C3 > $O/timeline_c3.txt 2>&1
