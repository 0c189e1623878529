"""Strong-scaling rehearsal on one device: the ms/step of ONE rank's share of a config (C3 by
default, CONFIG=C5 for the 512^3 frame; 1/N of the cost-balanced split, the FIRST range, or
every range with ALLR=1) as E engines take the steps in turn (queued, no host sync).
REBAL=n: after measuring every rank's share, rebalance the split n times from the measured
times (gpu.rebalance, what bench.py --gpus N does before its timed steps) and measure again."""
import os
import sys
import time

# as bench.py: every engine on a hardware queue of its own (the box's default is 4, and a
# context sharing the null stream's queue slows every step); set before HIP starts
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_QUEUES", "8")  # RT_QUEUES=4: the box's default
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

CONFIG = os.environ.get("CONFIG", "C3")
model, cs, N = synth.make_config(CONFIG)
plan = gpu.Polygonizer(0)
plan.set_model(model)
plan.run(cs)
costs = plan.mpu_costs()
OPTS = ((gpu.OPT_VERTEX_BLOCKS_PER_CU, "VB"), (gpu.OPT_FINISH_BLOCKS_PER_CU, "FB"), (gpu.OPT_FINISH_QUAD, "FQ"),
        (gpu.OPT_BOUND, "BD"), (gpu.OPT_DEBUG, "DBG"), (gpu.OPT_GRAPH, "GR"), (gpu.OPT_VERTEX_WIDE, "VW"), (gpu.OPT_JIT, "JIT"), (gpu.OPT_TREE_SPLIT, "TS"), (gpu.OPT_SPLIT_MAX_QUEUED, "SMQ"))
TAG = " ".join(f"{e}={os.environ.get(e, '-')}" for _, e in OPTS) + f" q={os.environ['GPU_MAX_HW_QUEUES']}"


def measure(lo, hi, neng, K):
    ps = []
    for _ in range(neng):
        p = gpu.Polygonizer(0)
        for opt, env in OPTS:
            if os.environ.get(env):
                p.set_option(opt, int(os.environ[env]))
        p.set_model(model)
        p.run(cs, lo, hi)
        ps.append(p)
    for k in range(max(50, K // 4)):  # warm-up (the first range a process times runs slow otherwise)
        ps[k % neng].polygonize(cs, lo, hi)
    for p in ps:
        p.finish()
    t0 = time.perf_counter()
    for k in range(K):
        ps[k % neng].polygonize(cs, lo, hi)
    for p in ps:
        p.finish()
    dt = (time.perf_counter() - t0) / K * 1e3
    for p in ps:
        p.close()
    return dt


K = int(os.environ.get("K", "400"))
for ranks in [int(x) for x in os.environ.get("SHARES", "1,2,4,8").split(",")]:
    b = gpu.split_costs(costs, ranks)
    for it in range(int(os.environ.get("REBAL", "0")) + 1):
        for neng in [int(x) for x in os.environ.get("ENGINES", "1,2,4").split(",")]:
            times = []
            for r in (range(ranks) if os.environ.get("ALLR") or os.environ.get("REBAL") else [0]):
                lo, hi = int(b[r]), int(b[r + 1])
                dt = measure(lo, hi, neng, K)
                times.append(dt)
                print(f"{CONFIG} rank {r} share 1/{ranks} (MPUs {hi - lo}): {neng} engines {TAG} "
                      f"{'rebalance ' + str(it) + ' ' if it else ''}{dt:.4f} ms/step", flush=True)
        if len(times) == ranks and ranks > 1:
            print(f"{CONFIG} share 1/{ranks} {'rebalance ' + str(it) if it else 'cost split'}: slowest rank "
                  f"{max(times):.4f} ms/step, mean {sum(times) / ranks:.4f}", flush=True)
            b = gpu.rebalance(costs, b, times)
