set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 200 python -u tools/window_timeline.py > $O/window.txt 2>&1 &&
timeout -k 10 200 python -u tools/window_timeline.py --stagger-us 15 > $O/window_stagger15.txt 2>&1 &&
for i in 1 2 3; do
  for S in 0 10 20; do
    timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extras --stagger-us $S > $O/drv_s${S}_$i.json 2> $O/drv_s${S}_$i.err || exit 1
  done
done
timeout -k 10 200 python -u tools/timeline.py --phases > $O/mpu_phases.txt 2>&1
