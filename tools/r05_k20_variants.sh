# The driver's 20-step window (bench.py --steps 20 --warmup 5) with kernel variants whose
# occupancy differs, interleaved fresh processes on one box: in the window the four engines
# run in lockstep (the same kernel at the same time), unlike the 200-step steady state
set -o pipefail
O=gpurun_out/r5k20v
mkdir -p $O
run() {  # name, env, args
  env $2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras $3 > $O/$1_$i.json 2> $O/$1_$i.err
}
for i in 1 2 3 4 5; do
  run base "PSGPU_X=0" "" || exit 1
  run s2g5 "PSGPU_JIT_FLAGS=-DPSGPU_S2_GROUP=5" "" || exit 1
  run baked "PSGPU_X=0" "--jit 2" || exit 1
  run fin8 "PSGPU_X=0" "--finish-blocks 8" || exit 1
done
python - <<'PY'
import json, glob, statistics
for n in ("base", "s2g5", "baked", "fin8"):
    v = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/r5k20v/{n}_*.json"))]
    print(f"{n:6s} K 20: ms/step {' '.join(f'{x:.4f}' for x in v)}  median {statistics.median(v):.4f}")
PY
