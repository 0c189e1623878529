# The 4-way tree split (PSGPU_OPT_SPLIT_WAYS 4: k_precheck / k_mpu walk the root's grandchild
# subtrees in four waves per item) vs the root split (2): parity first, then the C4 1/8-share
# rehearsal and a lone 1/8-share timeline, interleaved, one box
set -o pipefail
O=gpurun_out/r5s4
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "split or random_trees or fuzz or golden" > $O/parity.log 2>&1 || { echo parity failed; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2; do
  for w in 2 4; do
    PSGPU_SPLIT_WAYS=$w SHARES=8 ENGINES=4 REBAL=2 JIT=1 TS=2 K=400 timeout -k 10 300 python3 -u tools/range_test.py > $O/c4_w${w}_$i.txt 2>&1 || exit 1
    echo "C4 ways $w run $i: $(grep 'rebalance 2:' $O/c4_w${w}_$i.txt)"
  done
done
for w in 2 4; do
  PSGPU_SPLIT_WAYS=$w timeout -k 10 300 python3 -u tools/engines_timeline.py --engines 1 --share 8 --rank 4 --tree-split 1 --json $O/tl1_w$w.json > /dev/null 2>&1 || exit 1
  PSGPU_SPLIT_WAYS=$w timeout -k 10 300 python3 -u tools/engines_timeline.py --engines 4 --share 8 --rank 4 --tree-split 1 --json $O/tl4_w$w.json > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import json
for e in (1, 4):
    for w in (2, 4):
        d = json.load(open(f"gpurun_out/r5s4/tl{e}_w{w}.json"))
        ks = d["kernels"]
        print(f"timeline {e} engine(s), ways {w}: window {d['window_us']} us; " + "; ".join(
            f"{k} span {max(v['span_us'])} max life {max(v['life_us_max'])} sum {round(v['wave_us_sum'])}" for k, v in ks.items()))
PY
