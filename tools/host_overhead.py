"""Host cost of enqueueing a polygonization (4 launches, or one hipGraph replay) against the
device time per step, at a rank's share of C3 (strong scaling, 1/SHARE of the cost split) with
E engines: if the enqueue takes as long as a step, the step rate is host-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

E = int(os.environ.get("ENGINES", "4"))
model, cs, N = synth.make_config("C3")
plan = gpu.Polygonizer(0)
plan.set_model(model)
plan.run(cs)
costs = plan.mpu_costs()
for share in [int(x) for x in os.environ.get("SHARES", "1,8").split(",")]:
    b = gpu.split_costs(costs, share)
    lo, hi = int(b[0]), int(b[1])
    for graph in (0, 1):
        ps = []
        for _ in range(E):
            p = gpu.Polygonizer(0)
            p.set_option(gpu.OPT_GRAPH, graph)
            p.set_model(model)
            p.run(cs, lo, hi)
            ps.append(p)
        for k in range(40):
            ps[k % E].polygonize(cs, lo, hi)
        for p in ps:
            p.finish()
        K = 400
        t0 = time.perf_counter()
        enq = 0.0
        for k in range(K):
            a = time.perf_counter()
            ps[k % E].polygonize(cs, lo, hi)
            enq += time.perf_counter() - a
        for p in ps:
            p.finish()
        dt = (time.perf_counter() - t0) / K * 1e6
        print(f"share 1/{share} graph={graph}: {dt:.1f} us/step, enqueue {enq / K * 1e6:.1f} us/step", flush=True)
        # one host thread per engine (ctypes releases the GIL inside the library calls)
        import threading

        def worker(e):
            for k in range(e, K, E):
                ps[e].polygonize(cs, lo, hi)

        t0 = time.perf_counter()
        th = [threading.Thread(target=worker, args=(e,)) for e in range(E)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for p in ps:
            p.finish()
        dt = (time.perf_counter() - t0) / K * 1e6
        print(f"share 1/{share} graph={graph} threads: {dt:.1f} us/step", flush=True)
        for p in ps:
            p.close()
