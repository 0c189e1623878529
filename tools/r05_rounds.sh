set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
(rocm-smi --showclocks > $O/clocks_before.txt 2>&1 || true)
timeout -k 10 200 python -u tools/window_timeline.py --steps 20 --reps 2 > $O/w20.txt 2>&1 &&
timeout -k 10 200 python -u tools/window_timeline.py --steps 400 --reps 2 > $O/w400.txt 2>&1 &&
timeout -k 10 200 python -u tools/window_timeline.py --steps 400 --reps 1 --engines 1 > $O/w400_e1.txt 2>&1
(rocm-smi --showclocks > $O/clocks_after.txt 2>&1 || true)
