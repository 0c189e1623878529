set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "golden or random_trees or c5 or scene or split" > $O/parity.log 2>&1 || { echo parity failed; tail -30 $O/parity.log; exit 1; }
B="python -u bench.py --steps 200 --warmup 20 --no-cpu"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/new_$i.json 2> $O/new_$i.err &&
  PSGPU_JIT_FLAGS=-DPSGPU_MPU_LDS_TABLES=0 timeout -k 10 200 $B > $O/hoist_$i.json 2> $O/hoist_$i.err &&
  PSGPU_JIT_FLAGS="-DPSGPU_MPU_LDS_TABLES=0 -DPSGPU_PASS1_HOIST=0" timeout -k 10 200 $B > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
timeout -k 10 200 python -u tools/window_timeline.py > $O/window.txt 2>&1 &&
timeout -k 10 200 python -u tools/window_timeline.py --stagger-us 15 > $O/window_stagger15.txt 2>&1 &&
for i in 1 2 3; do
  for S in 0 15; do
    timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extras --stagger-us $S > $O/drv_s${S}_$i.json 2> $O/drv_s${S}_$i.err || exit 1
  done
done
timeout -k 10 200 python -u tools/timeline.py --phases > $O/mpu_phases.txt 2>&1
