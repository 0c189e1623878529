#!/usr/bin/env python3
"""Benchmark: Mcells/s polygonized, 256^3 grid, 32-primitive BlobTree (BASELINE.json).

One step = one full polygonization of the C3 workload (32 prims, 31 ops
with Union/Dif, 256^3 cells over [-4,4]^3 = 50,653 MPUs) on one GPU with the model
already resident in HBM: S1 precheck -> compaction -> per-MPU field cache, classification
and vertex ownership -> offsets -> vertices (root, colour, normal) -> triangles.  The
compact mesh stays in HBM.

N GPUs (torchrun, one process per GPU): weak scaling.  Rank r polygonizes its own
256^3 grid of frame r of the animated C3 tree (independent objects, no data-path
collective); value = N * 256^3 / max-over-ranks step time.  `--scaling strong` instead
splits one 256^3 grid into contiguous MPU ranges (config C4).

Output: one JSON line on rank 0 (the driver's contract) with `roofline` for the dominant
kernel (hipEvent-timed on the library's stream) and `cpu_baseline` (the oracle, rank 0,
N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from parsip_amd import costmodel, gpu, synth  # noqa: E402

VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md "Peak FP32 (vector)" (= FP32 MFMA rate)
HBM_PEAK_GBS = 8000.0


class Group:
    """Barrier / max-reduce across ranks.  torch.distributed (gloo, CPU tensors) is only
    imported for N > 1 and after the HIP library has initialised the device."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None

    def init(self):
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def allgather(self, vals):
        if not self.dist:
            return [list(vals)]
        import torch

        t = torch.tensor(list(vals), dtype=torch.int64)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]


def measured_traffic(kernel: str, jit: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/<round>_traffic.json, made by tools/gpu_round.sh + tools/traffic.py on the
    same workload): 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE.  None if absent."""
    import glob

    names = [f"jit_{kernel[2:]}" if jit else f"psgpu::{kernel}", kernel]
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for n in names:
            if n in ks and "traffic_bytes" in ks[n]:
                return ks[n]["traffic_bytes"], os.path.basename(path)
    return None, None


def workload_ops(config: str):
    path = os.path.join(ROOT, "tests", "golden", "workload_ops.json")
    try:
        with open(path) as f:
            return json.load(f).get(config)
    except (OSError, ValueError):
        return None


def valu_utilisation(kernel: str, jit: int, ms: float):
    """VALU issue utilisation of `kernel` from the committed PMC pass
    (profiles/*_valu.json: SQ_INSTS_VALU per launch): instructions x 4 cycles (wave64 on
    16-lane SIMDs) over the launch's SIMD-cycles (1024 SIMDs at 2.4 GHz)."""
    import glob

    names = [f"jit_{kernel[2:]}" if jit else f"psgpu::{kernel}", kernel]
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu.json")), reverse=True):
        try:
            with open(path) as f:
                ks = json.load(f)["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for n in names:
            if n in ks and "SQ_INSTS_VALU" in ks[n]:
                return round(ks[n]["SQ_INSTS_VALU"] * 4 / (ms * 1e-3 * 2.4e9 * 1024), 4), os.path.basename(path)
    return None, None


def cpu_baseline(model, cs, n_cells):
    """The oracle (CPU restatement, 'port') on the host's cores: bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import psoracle

    psoracle.build()
    threads = int(os.environ.get("PSGPU_CPU_THREADS", os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    threads = max(1, min(threads, os.cpu_count() or 1))
    times = []
    psoracle.polygonize(model, cs, threads=threads, keep=False)  # warm-up
    t_budget = float(os.environ.get("PSGPU_CPU_SECONDS", "12"))
    t_start = time.perf_counter()
    while len(times) < 10 and (time.perf_counter() - t_start) < t_budget:
        t0 = time.perf_counter()
        psoracle.polygonize(model, cs, threads=threads, keep=False)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": round(n_cells / med / 1e6, 3), "unit": "Mcells/s", "cores": threads, "kind": "port",
            "sample": f"full C3 256^3 polygonization x{len(times)} (median {med * 1e3:.1f} ms, "
                      f"best {min(times) * 1e3:.1f} ms), oracle/psoracle.c with {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-cull", action="store_true", help="disable exact primitive culling")
    ap.add_argument("--jit", type=int, default=1, choices=[0, 1, 2],
                    help="0 interpreter, 1 kernels specialised per tree structure, 2 + parameters baked in")
    ap.add_argument("--debug", type=int, default=0, help=argparse.SUPPRESS)  # profiling ablations only
    args = ap.parse_args()

    grp = Group()
    # one process per GPU (LOCAL_RANK); PSGPU_BENCH_DEVICE pins every rank to one device
    # (multi-rank rehearsal on a one-GPU box)
    poly = gpu.Polygonizer(int(os.environ.get("PSGPU_BENCH_DEVICE", grp.local)))  # HIP before torch
    grp.init()
    if args.no_cull:
        poly.set_option(gpu.OPT_CULLING, 0)
    poly.set_option(gpu.OPT_JIT, args.jit)
    if args.debug:
        poly.set_option(gpu.OPT_DEBUG, args.debug)

    frame = grp.rank if args.scaling == "weak" else 0
    model, cs, N = synth.make_config(args.config, frame=frame)
    t_model = time.perf_counter()
    poly.set_model(model)  # uploads the SoA and builds/compiles the tree kernels
    t_model = time.perf_counter() - t_model
    n_mpus = gpu.count_mpus(cs, *model.bbox)
    if args.scaling == "strong" and grp.world > 1:
        per = (n_mpus + grp.world - 1) // grp.world
        begin, end = grp.rank * per, min(n_mpus, (grp.rank + 1) * per)
    else:
        begin, end = 0, n_mpus

    for _ in range(args.warmup):
        poly.run(cs, begin, end)
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        poly.polygonize(cs, begin, end)
    info = poly.finish()
    grp.barrier()
    t1 = time.perf_counter()
    dt = grp.max(t1 - t0)
    ms_step = dt / args.steps * 1e3
    cells_per_step = N ** 3 * (grp.world if args.scaling == "weak" else 1)
    value = cells_per_step / (ms_step * 1e-3) / 1e6

    # roofline pass: per-kernel hipEvent timing on the library's stream
    poly.set_option(1, 1)
    kt = {}
    reps = max(3, min(args.steps, 10))
    for _ in range(reps):
        poly.run(cs, begin, end)
        for k, v in poly.kernel_times().items():
            kt[k] = kt.get(k, 0.0) + v / reps
    poly.set_option(1, 0)
    dom = max(kt, key=kt.get)
    per_eval = costmodel.ops_per_eval(model)
    kernel_evals = {"k_precheck": 8 * info.ctMPUs, "k_mpu": 512 * info.ctPassedPrecheck,
                    "k_vertex": 7 * info.ctVertices, "k_finish": info.ctVertices}
    # algorithmic work: the fp32 ops the reference executes on this input (after its own
    # op-box pruning), counted by the oracle and priced by costmodel
    # (tests/golden/workload_ops.json); else SURVEY §8(d)'s unpruned per-eval figure
    wops = workload_ops(args.config)
    if wops and wops.get("vertices") == info.ctVertices and dom in wops:
        dom_flops, flops_src = wops[dom], "tests/golden/workload_ops.json (reference-executed ops)"
    else:
        dom_flops, flops_src = kernel_evals.get(dom, 0) * per_eval, "lane-evals x costmodel.ops_per_eval"
    achieved = dom_flops / (kt[dom] * 1e-3) / 1e12
    counts = grp.allgather([info.ctVertices, info.ctTriangles])
    traffic, traffic_src = measured_traffic(dom, args.jit) if args.config == "C3" else (None, None)
    valu_util, valu_src = valu_utilisation(dom, args.jit, kt[dom]) if args.config == "C3" else (None, None)

    out = {
        "metric": "Mcells/sec polygonized, 256^3 grid 32-prim BlobTree, at 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "Mcells/s",
        "n_gpus": grp.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: C3 BlobTree from std::mt19937(42) as in the reference probe (SURVEY.md §6, §8(d))",
        "config": {"workload": f"{args.config}: {model.ct_prims}-prim/{model.ct_ops}-op BlobTree, {N}^3 cells, "
                               f"{n_mpus} MPUs" + (f", frame=rank" if args.scaling == "weak" and grp.world > 1 else ""),
                   "grid": N, "mpus": n_mpus, "prims": model.ct_prims, "ops": model.ct_ops,
                   "parallelism": f"{args.scaling}-{grp.world}gpu",
                   "mpu_range": [begin, end], "culling": not args.no_cull,
                   "kernels": ["interpreter", "jit-structure", "jit-baked"][args.jit] if poly.jit_active or args.jit == 0
                   else "interpreter (jit unavailable)", "set_model_s": round(t_model, 3)},
        "roofline": {"bound": "mfma", "pipe": "fp32 VALU (peak = FP32 vector = FP32 MFMA rate)",
                     "kernel": dom, "achieved": round(achieved, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / VALU_PEAK_TFLOPS, 4),
                     "traffic": None if traffic is None else round(traffic),
                     "traffic_source": traffic_src,
                     "kernel_ms": round(kt[dom], 4), "algorithmic_ops": dom_flops, "ops_source": flops_src,
                     "note": "exact culling skips ~90% of the primitive evaluations the reference executes, so "
                             "reference-equivalent throughput can reach the VALU peak; valu_issue_util is the "
                             "hardware-side figure",
                     "valu_issue_util": valu_util, "valu_source": valu_src},
        "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
        "mesh": {"vertices": info.ctVertices, "triangles": info.ctTriangles, "passed_s1": info.ctPassedPrecheck,
                 "surface_mpus": info.ctSurfaceMPUs, "field_mpus": info.ctFieldMPUs, "per_rank": counts},
        "hbm_gbs_algorithmic": round((info.ctVertices * 36 + info.ctTriangles * 12) / (ms_step * 1e-3) / 1e9, 2),
    }
    if grp.rank == 0 and grp.world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(model, cs, N ** 3)
    if grp.rank == 0:
        print(json.dumps(out), flush=True)
    if grp.dist:
        grp.dist.destroy_process_group()
    poly.close()


if __name__ == "__main__":
    main()
