set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
for S in 30 55 80; do
  timeout -k 10 200 python -u tools/window_timeline.py --stagger-us $S --reps 2 > $O/window_s$S.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for S in 0 30 55 80; do
    timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extras --stagger-us $S > $O/drv_s${S}_$i.json 2> $O/drv_s${S}_$i.err || exit 1
  done
done
