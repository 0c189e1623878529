#!/usr/bin/env python3
"""Benchmark: Mcells/s polygonized, 256^3 grid, 32-primitive BlobTree (BASELINE.json).

One step = one full polygonization of the C3 workload (32 prims, 31 ops
with Union/Dif, 256^3 cells over [-4,4]^3 = 50,653 MPUs) with the model already resident
in HBM: S1 precheck -> compaction -> per-MPU field cache, classification and vertex
ownership -> offsets -> vertices (root, colour, normal) -> triangles.  The compact mesh
stays in HBM.

N GPUs (one process per GPU: under torch.distributed.run, or `--gpus N` alone, which
spawns the N ranks itself before any HIP call): strong scaling by default, config C4 —
ONE 256^3 grid split into N contiguous MPU ranges of near-equal cost (the split comes
from one full planning run on every rank, deterministic, so all ranks agree without
communication); every step each rank polygonizes its range and the ranks exchange their
(MPUs, V, T, ...) totals with one RCCL all-gather on the library's stream (the only
collective: MPUs are independent, no halo).  value = 256^3 / max-over-ranks step time.
`--scaling weak` instead gives every rank its own grid (frame r of the animated tree).

Output: one JSON line on rank 0 (the driver's contract) with `roofline` for the dominant
kernel (hipEvent-timed on the library's stream) and `cpu_baseline` (the oracle, rank 0,
N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# HIP hands each process GPU_MAX_HW_QUEUES hardware queues (the box's default is 4) and maps
# streams onto them round-robin.  4 engines (one stream each) on queues of their own take the
# most steps per second (tools/rt_fresh.sh: C3 0.068 ms/step at >= 6 queues vs 0.080 with 2
# engines on 4; a 1/8 rank share 0.0165 vs 0.028); more than 4 concurrent streams is slower
# again.  Read at HIP init, so set here, before any HIP call: --hw-queues N wins, else at
# least HW_QUEUES_DEFAULT.
ENGINES_DEFAULT = 4
TIER_RUNS = 16        # OPT_TIER_RUNS: unchanged-model runs before the baked kernels (the library default)
TIER_HOLD = 1 << 30   # no tier-up while the structure kernels' pass is timed
HW_QUEUES_DEFAULT = 8
_hwq = None
for _i, _a in enumerate(sys.argv):
    if _a == "--hw-queues" and _i + 1 < len(sys.argv):
        _hwq = sys.argv[_i + 1]
if _hwq is None:
    _hwq = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4), HW_QUEUES_DEFAULT))
os.environ["GPU_MAX_HW_QUEUES"] = _hwq

from parsip_amd import costmodel, gpu, synth  # noqa: E402  (no HIP call at import)

VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md "Peak FP32 (vector)": 256 CU x 4 SIMD-32 x 2.4 GHz x 64 (FMA)
HBM_PEAK_GBS = 8000.0
# reference-priced ops above the VALU peak: not a utilisation (frac is then null)
FRAC_OVER_NOTE = (" (reference-priced ops / time exceeds the VALU peak: exact culling skips more of the tree "
                  "than the reference's op-box pruning, so the reference's op count is not this launch's work; "
                  "see valu_issue / the PMC profile for the hardware-side utilisation)")
METRIC = "Mcells/sec polygonized, 256^3 grid 32-prim BlobTree, at 1/2/4/8 MI355X"
# other configs are parity / scaling rehearsals, labelled by their own workload
METRIC_OTHER = "Mcells/sec polygonized, {n}^3 grid {p}-prim BlobTree ({config}), at {g} MI355X"
NOFMA_PEAK_TOPS = 78.6  # fp32 VALU lane-ops without FMA (-ffp-contract=off): 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside a launcher: start N rank processes (one per GPU) as
    children before this process touches a GPU, wait, return the worst exit code."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    # a rank that fails (e.g. no HIP device for it) would leave the others waiting in the
    # rendezvous forever: as torch.distributed.run does, end the remaining ranks then
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            return max(codes, key=abs)
        if any(c not in (None, 0) for c in codes):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return max((p.returncode for p in procs), key=abs)
        time.sleep(0.2)


class Group:
    """Barrier / max-reduce / broadcast across ranks over gloo (CPU).  torch.distributed is
    imported only for N > 1 and after the HIP library has initialised the device (the
    library's ROCm runtime is then the one loaded in the process)."""

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

    def broadcast_bytes(self, b: bytes | None) -> bytes:
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def allgather(self, vals, dtype="int64"):
        if not self.dist:
            return [list(vals)]
        import torch

        t = torch.tensor(list(vals), dtype=getattr(torch, dtype))
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]


def committed_profile(kind: str, jit: int):
    """Newest committed rocprofv3 summary of `kind` (profiles/rNN_<kind>.json) profiled on the
    kernels of OPT_JIT mode `jit` (the file's "jit"; files from before r04 carry none and were
    profiled with --jit 2)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{kind}.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            if int(d.get("jit", 2)) != jit:
                continue
            return d["kernels"], os.path.relpath(path, ROOT)
        except (OSError, ValueError, KeyError, TypeError):
            continue
    return None, None


def profile_entry(kernels, kernel: str, jit: int):
    if not kernels:
        return None
    for n in ([f"jit_{kernel[2:]}"] if jit else []) + [f"psgpu::{kernel}", kernel]:
        if n in kernels:
            return kernels[n]
    return None


def workload_ops(config: str):
    path = os.path.join(ROOT, "tests", "golden", "workload_ops.json")
    try:
        with open(path) as f:
            return json.load(f).get(config)
    except (OSError, ValueError):
        return None


def cpu_info():
    model, smt = "unknown", None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        smt = open("/sys/devices/system/cpu/smt/active").read().strip() == "1"
    except OSError:
        pass
    return model, smt


def host_cores():
    """Cores this process may run on: the affinity set, capped by a cgroup CPU quota if one
    is set (threads past the quota are throttled, not parallel); and the figures behind it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):  # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:  # cgroup v1
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(-(-quota // 1))))
    return cores, {"nproc": nproc, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
                   "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(model, cs, n_cells, config):
    """The oracle (oracle/psoracle.c, the CPU restatement of the reference: "port") on every
    core this process may use (host_cores), 2 warm-ups, then up to 10 timed runs within a
    bounded budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import psoracle

    psoracle.build()
    cores, why = host_cores()
    threads = int(os.environ.get("PSGPU_CPU_THREADS", cores))
    times = []
    for _ in range(2):  # warm-ups
        psoracle.polygonize(model, cs, threads=threads, keep=False)
    t_budget = float(os.environ.get("PSGPU_CPU_SECONDS", "12"))
    t_start = time.perf_counter()
    while len(times) < 10 and (time.perf_counter() - t_start) < t_budget:
        t0 = time.perf_counter()
        psoracle.polygonize(model, cs, threads=threads, keep=False)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    cpu_model, smt = cpu_info()
    return {"value": round(n_cells / med / 1e6, 3), "unit": "Mcells/s", "cores": threads, "kind": "port",
            "sample": f"full {config} polygonization x{len(times)} after 2 warm-ups (median {med * 1e3:.1f} ms, "
                      f"best {min(times) * 1e3:.1f} ms) by oracle/psoracle.c, the plain-C restatement of the "
                      f"reference (PS_Polygonizer.cpp; the reference binary is not built here), {threads} threads = "
                      f"the cores this process may use (affinity set, capped by the cgroup CPU quota)",
            "cpu_model": cpu_model, "smt_active": smt, **why}


def latency_single(poly, cs, reps=30):
    """One engine, one polygonization at a time (enqueue + device chain + host sync): what a
    blocking caller or a frame-at-a-time editor sees.  Median / best over `reps` runs."""
    poly.run(cs)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        poly.run(cs)
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e3, 4), round(min(t) * 1e3, 4)


def latency_single_parts(device, model, cs, jit, parts=2, reps=30):
    """latency_single for ONE polygonization split into `parts` cost-balanced MPU ranges on
    `parts` streams of the same device (psgpu_group over [device] * parts): the ranges'
    kernel chains overlap each other's tails.  The parts' meshes stay separate, concatenating
    in range order to the single-context mesh (psgpu_group_gather assembles one buffer)."""
    g = gpu.Group([device] * parts)
    try:
        g.set_option(gpu.OPT_JIT, gpu.JIT_BAKED if jit == gpu.JIT_TIERED else jit)
        g.set_model(model)
        for _ in range(3):
            info, _ = g.run(cs)
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            g.run(cs)
            t.append(time.perf_counter() - t0)
        return {"median": round(float(np.median(t)) * 1e3, 4), "best": round(min(t) * 1e3, 4), "parts": parts,
                "vertices": info.ctVertices, "triangles": info.ctTriangles,
                "note": f"one polygonization at a time as {parts} cost-balanced MPU ranges on {parts} streams of one "
                        "device (psgpu_group), host-timed (enqueue + kernel chains + sync)"}
    finally:
        g.close()


def blocking_contract(polys, config="C2", reps=24):
    """The reference's own blocking contract, PCIe-inclusive: Polygonize into the caller's
    PolyMPUs (PS_Polygonizer.h:386-391 as SimdPoly::run calls it, PS_HighPerformanceRender.cpp:
    373-376): model upload, polygonization, mesh download and the scatter into the sparse
    21.5-KB-per-MPU PolyMPUs layout.  `polys`: {name: engine}, each one context
    (gpu.Polygonizer: what psgpu::Polygonize / gpu.Polygonize run on) or a gpu.Group of parts of
    the device; their calls alternate, so every engine sees the same host and link conditions
    (some boxes run a few calls in 24 several times slower: DESIGN.md §4 "Blocking").  C3 has
    50,653 MPUs, past the reference's MAX_MPU_COUNT (24,000), so its PolyMPUs array is allocated
    with room for them (1.09 GB).  Per engine: median, best and p90 over `reps` calls after 2
    warm-ups."""
    from parsip_amd import soa

    model, cs, n = synth.make_config(config)
    ct_need = gpu.count_mpus(cs, *model.bbox)
    out = np.zeros(max(soa.MAX_MPU_COUNT, ct_need), soa.MPU_DTYPE)
    for _ in range(2):
        for poly in polys.values():
            rc, ct, _ = poly.polygonize_mpus(cs, model, out)
            assert rc == 1 and ct == ct_need, (rc, ct)
    t = {k: [] for k in polys}
    for _ in range(reps):
        for k, poly in polys.items():
            t0 = time.perf_counter()
            poly.polygonize_mpus(cs, model, out)
            t[k].append(time.perf_counter() - t0)
    res = {}
    for k, poly in polys.items():
        med = float(np.median(t[k]))
        engine = (f"psgpu_group_polygonize_mpus over {poly.n} parts of one device"
                  if isinstance(poly, gpu.Group) else "psgpu_polygonize_mpus on one context (the drop-ins' default)")
        res[k] = {"config": f"{config}: {model.ct_prims}-prim BlobTree, {n}^3 cells, {ct_need} MPUs",
                  "ms": round(med * 1e3, 3), "best_ms": round(min(t[k]) * 1e3, 3),
                  "p90_ms": round(float(np.percentile(t[k], 90)) * 1e3, 3), "calls": reps,
                  "mcells_per_s": round(n ** 3 / med / 1e6, 2), "engine": engine,
                  "note": "end to end (SoA upload, the kernel chains, compact-mesh download over PCIe, host scatter "
                          "into PolyMPUs); never the bench value"}
    return res


class Engine:
    """One device context over the rank's MPU range [begin, end) (parts == 1), or a group of
    `parts` cost-balanced sub-ranges on as many streams of the device."""

    def __init__(self, device, model, cs, args, begin, end, costs, poly=None):
        self.cs, self.begin, self.end, self.parts = cs, begin, end, max(1, args.parts)
        self.comm = None
        self.owns = poly is None
        if self.parts == 1:
            self.p = poly if poly is not None else gpu.Polygonizer(device)
            self.obj = self.p
        else:
            self.p = None
            self.obj = gpu.Group([device] * self.parts)
        if args.engines > 1:  # engines share the CUs: half the persistent waves each (1.8 % faster at 4)
            self.obj.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, args.vertex_blocks or 8)
            self.obj.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, args.finish_blocks or 4)
        else:
            if args.vertex_blocks:
                self.obj.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, args.vertex_blocks)
            if args.finish_blocks:
                self.obj.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, args.finish_blocks)
        if poly is None or self.parts > 1:
            if args.no_cull:
                self.obj.set_option(gpu.OPT_CULLING, 0)
            self.obj.set_option(gpu.OPT_JIT, args.jit)
            if args.jit == gpu.JIT_TIERED:  # held until the structure kernels' pass is measured
                self.obj.set_option(gpu.OPT_TIER_RUNS, TIER_HOLD)
            self.obj.set_option(gpu.OPT_TREE_SPLIT, args.tree_split)
            if args.debug:
                self.obj.set_option(gpu.OPT_DEBUG, args.debug)
            self.obj.set_model(model)
        if self.parts > 1:
            self.obj.set_split(gpu.split_costs(costs[begin:end], self.parts, begin))

    def set_range(self, begin, end, costs):
        self.begin, self.end = begin, end
        if self.parts > 1:
            self.obj.set_split(gpu.split_costs(costs[begin:end], self.parts, begin))

    def polygonize(self):
        if self.p is not None:
            self.p.polygonize(self.cs, self.begin, self.end)
        else:
            self.obj.polygonize(self.cs)
        if self.comm:
            self.comm.exchange()

    def finish(self):
        """(totals, parts) of the last run: over all ranks when exchanging."""
        if self.comm:
            return self.comm.result()
        if self.p is not None:
            return self.p.finish(), None
        return self.obj.finish()

    def local_info(self):
        return self.p.finish() if self.p is not None else self.obj.finish()[0]

    def set_option(self, opt, val):
        self.obj.set_option(opt, val)

    def jit_wait(self):
        return self.obj.jit_wait()

    def jit_tier(self):
        return self.obj.jit_tier

    def event_times(self):
        """Per part of the last run: hipEvent ms per kernel (OPT_KERNEL_TIMING)."""
        if self.p is not None:
            self.p.finish()
            return [self.p.kernel_times()]
        self.obj.finish()
        return [self.obj.kernel_times(i) for i in range(self.parts)]

    def stamp_spans(self):
        """Per part of the last run: (device-clock spans per kernel, S2-evaluated MPUs), from
        the per-wave timeline (OPT_STAMPS)."""
        if self.p is not None:
            info = self.p.finish()
            return [(gpu.kernel_spans(self.p.stamps(), bool(info.launchFlags & gpu.LAUNCH_FRONT)), info.ctFieldMPUs)]
        _, parts = self.obj.finish()
        return [(gpu.kernel_spans(self.obj.stamps(i), bool(parts[i].info.launchFlags & gpu.LAUNCH_FRONT)),
                 parts[i].info.ctFieldMPUs) for i in range(self.parts)]

    def spans(self, raw=False):
        """(launches, kernels) device-clock spans in ms recorded since OPT_SPANS, every part
        (raw: (launches, kernels, {first wave start, last wave end}) in 100 MHz ticks)."""
        if self.p is not None:
            return self.p.spans(raw)
        return np.concatenate([self.obj.spans(i, raw) for i in range(self.parts)])

    def close(self):
        if self.comm:
            self.comm.close()
        if self.p is None or self.owns:
            self.obj.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="N>1: strong (default: one grid split over the ranks) or weak (a grid per rank)")
    ap.add_argument("--engines", type=int, default=ENGINES_DEFAULT,
                    help="per device: this many engines (device contexts, each on its own HIP stream) take the "
                         "steps in turn; each step is a complete polygonization of the rank's range, queued "
                         "without host sync, so one run's kernel tails overlap the other's bulk")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; at most 32)")
    ap.add_argument("--parts", "--streams", type=int, default=1, dest="parts",
                    help="per engine: the range as this many cost-balanced parts on as many streams")
    ap.add_argument("--rebalance", type=int, default=2,
                    help="strong scaling: rebalance the cost split this many times from the ranks' measured step "
                         "times before the timed steps (gpu.rebalance)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the single-polygonization latency and the blocking C2 Polygonize timing")
    ap.add_argument("--no-cull", action="store_true", help="disable exact primitive culling")
    ap.add_argument("--jit", type=int, default=None, choices=[0, 1, 2, 3],
                    help="0 interpreter, 1 kernels specialised per tree structure (default), 2 + parameters baked "
                         "in, 3 tiered: the structure kernels' pass, then the baked ones (tier-up forced before the "
                         "headline, which is timed and labelled on the tier reached)")
    ap.add_argument("--tree-split", type=int, default=None, choices=[0, 1, 2],
                    help="OPT_TREE_SPLIT: 1 walk the root's two subtrees in two waves per brick / MPU, 2 only on "
                         "launches that queue few MPUs (default: 2 for strong scaling over N > 1 ranks, whose "
                         "shares are small, else 0)")
    ap.add_argument("--debug", type=int, default=0, help=argparse.SUPPRESS)  # profiling ablations only
    ap.add_argument("--vertex-blocks", type=int, default=0, help=argparse.SUPPRESS)  # persistent grids (experiments)
    ap.add_argument("--finish-blocks", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # stdout carries exactly one line, the JSON result: anything libraries print there (gloo's
    # "[Gloo] Rank 0 is connected to ..." at connection time) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    grp = Group()
    if grp.world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={grp.world}: launch one process per GPU")
    scaling = args.scaling or ("strong" if grp.world > 1 else "weak")
    if args.jit is None:
        # the structure-specialised kernels: measured faster than the baked ones in the
        # 4-engine throughput regime since r04 (C3, 200 steps, 3 interleaved runs on one box:
        # 0.0563 vs 0.0590 ms/step, profiles/r04_tier_ab.txt); C5 changes its parameters every
        # frame, so it never leaves this tier anyway
        args.jit = gpu.JIT_STRUCTURE
    if args.tree_split is None:
        args.tree_split = 2 if scaling == "strong" and grp.world > 1 else 0

    # one process per GPU (LOCAL_RANK); PSGPU_BENCH_DEVICE pins every rank to one device
    # (multi-rank rehearsal on a one-GPU box: the count exchange then runs over gloo)
    pinned = os.environ.get("PSGPU_BENCH_DEVICE")
    device = int(pinned) if pinned is not None else grp.local
    ndev = gpu.device_count()
    if device >= ndev:
        sys.exit(f"bench.py: rank {grp.rank} needs HIP device {device} but {ndev} are visible "
                 "(PSGPU_BENCH_DEVICE=0 runs every rank on device 0: a one-GPU rehearsal)")
    poly = gpu.Polygonizer(device)  # HIP before torch
    grp.init()
    if args.no_cull:
        poly.set_option(gpu.OPT_CULLING, 0)
    poly.set_option(gpu.OPT_JIT, args.jit)
    if args.jit == gpu.JIT_TIERED:
        poly.set_option(gpu.OPT_TIER_RUNS, TIER_HOLD)
    poly.set_option(gpu.OPT_TREE_SPLIT, args.tree_split)
    if args.debug:
        poly.set_option(gpu.OPT_DEBUG, args.debug)

    frame = grp.rank if scaling == "weak" else 0
    model, cs, N = synth.make_config(args.config, frame=frame)
    t0 = time.perf_counter()
    poly.set_model(model, wait_jit=False)  # uploads the SoA; hiprtc compiles on a host thread
    t_model = time.perf_counter() - t0
    jit_on = poly.jit_wait() if args.jit else False
    t_jit = time.perf_counter() - t0
    n_mpus = gpu.count_mpus(cs, *model.bbox)

    full = None
    # the cost split: one full planning run on this rank's device (exact results, so every
    # rank computes the same split without communication)
    strong = scaling == "strong" and grp.world > 1
    nparts, neng = max(1, args.parts), max(1, args.engines)
    costs = None
    if strong or nparts > 1:
        poly.run(cs)
        full = poly.finish()
        costs = poly.mpu_costs()
    if strong:
        begin, end = gpu.rank_range(costs, grp.world, grp.rank)
    else:
        begin, end = 0, n_mpus
        full = None
    engines = [Engine(device, model, cs, args, begin, end, costs, poly if e == 0 else None) for e in range(neng)]
    exchange = None
    if strong:
        if pinned is None:  # one communicator per engine: its all-gathers stay on its stream
            err = None
            try:
                for e in engines:
                    uid = grp.broadcast_bytes(gpu.comm_unique_id() if grp.rank == 0 else None)
                    e.comm = gpu.Comm(e.obj, uid, grp.world, grp.rank)
            except gpu.PsgpuError as x:  # every rank learns whether all communicators exist
                err = x
            if grp.max(1.0 if err else 0.0) > 0.0:
                for e in engines:
                    if e.comm:
                        e.comm.close()
                    e.comm = None
                print(f"bench.py rank {grp.rank}: RCCL communicators unavailable ({err}); the totals "
                      "go over gloo after the timed steps", file=sys.stderr)
                exchange = "gloo all-gather after the timed steps (RCCL communicator creation failed)"
            else:
                exchange = "rccl all-gather of 8 words per rank per step (library stream)"
        else:
            exchange = "gloo all-gather after the timed steps (ranks share one device: RCCL needs distinct GPUs)"

    # measured-time load balancing (strong scaling): every rank times its range, the times
    # are all-gathered, and every rank derives the same new split (gpu.rebalance); the cost
    # model underprices surface-heavy regions, which otherwise set the max over ranks
    split_log = None
    if strong and args.rebalance > 0:
        bounds = [int(x) for x in gpu.split_costs(costs, grp.world)]
        split_log = {"initial": bounds, "rounds": []}
        comms = [e.comm for e in engines]
        for e in engines:
            e.comm = None  # no count exchange during calibration
        kcal = 40
        for it in range(args.rebalance):
            for k in range(2 * neng):
                engines[k % neng].polygonize()
            for e in engines:
                e.finish()
            grp.barrier()
            tc = time.perf_counter()
            for k in range(kcal):
                engines[k % neng].polygonize()
            for e in engines:
                e.finish()
            mine_t = (time.perf_counter() - tc) / kcal * 1e3
            times = [t[0] for t in grp.allgather([mine_t], dtype="float64")]
            bounds = [int(x) for x in gpu.rebalance(costs, bounds, times)]
            split_log["rounds"].append({"ms_per_step": [round(t, 4) for t in times], "new_bounds": bounds})
            begin, end = bounds[grp.rank], bounds[grp.rank + 1]
            for e in engines:
                e.set_range(begin, end, costs)
        for e, c in zip(engines, comms):
            e.comm = c
    # tiered kernels (OPT_JIT 3): the timed loop first on the structure kernels, then the
    # tier-up -- every engine has polygonized the unchanged model more than TIER_RUNS times, so
    # its next run starts the baked compile -- and the headline on the baked kernels
    tier = None
    if args.jit == gpu.JIT_TIERED:
        for k in range(max(args.warmup, neng)):
            engines[k % neng].polygonize()
        for e in engines:
            e.finish()
        grp.barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            engines[k % neng].polygonize()
        for e in engines:
            e.finish()
        grp.barrier()
        ms1 = grp.max(time.perf_counter() - t0) / args.steps * 1e3
        tiers1 = [e.jit_tier() for e in engines]
        # tier up now: every engine has run the unchanged model at least once, so with a
        # threshold of 1 its next run starts the baked compile (a short --steps never reaches
        # the library's default of TIER_RUNS runs per engine); wait for the swap
        for e in engines:
            e.set_option(gpu.OPT_TIER_RUNS, 1)
        tt = time.perf_counter()
        for k in range(neng):
            engines[k].polygonize()
        for e in engines:
            e.finish()
            e.jit_wait()
        t_tier = time.perf_counter() - tt
        tiers2 = [e.jit_tier() for e in engines]
        timed_jit = gpu.JIT_BAKED if all(t == 2 for t in tiers2) else gpu.JIT_STRUCTURE
        # every rank must time the same tier (a rank whose baked compile failed keeps the
        # structure kernels): the headline is labelled by the lowest tier over the ranks
        if grp.max(0.0 if timed_jit == gpu.JIT_BAKED else 1.0) > 0.0:
            timed_jit = gpu.JIT_STRUCTURE
        tier = {"structure_kernels": {"ms_per_step": round(ms1, 4),
                                      "value": round(N ** 3 * (grp.world if scaling == "weak" else 1) / (ms1 * 1e-3) / 1e6, 2),
                                      "tiers": tiers1},
                "tier_up_after_runs": 1, "baked_ready_s": round(t_tier, 3),
                "note": "the same K steps on the structure-specialised kernels (parameters read from the model in "
                        "HBM) before the tier-up; then every engine tiers up (OPT_TIER_RUNS 1: the library's "
                        f"default waits for {TIER_RUNS} unchanged runs) and the headline is timed on the tier in "
                        "config.tiers (2 = baked: parameters compiled in as literals); baked_ready_s = the tier-up "
                        "run to the kernels' swap (hiprtc compile or on-disk code-object cache)"}
    else:
        timed_jit = args.jit
    for k in range(max(args.warmup, neng)):
        engines[k % neng].polygonize()
    for e in engines:
        e.finish()
    grp.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):  # step k is one complete polygonization, on engine k mod E
        engines[k % neng].polygonize()
    t_enq = time.perf_counter()
    results = [e.finish() for e in engines]
    grp.barrier()
    t1 = time.perf_counter()
    dt = grp.max(t1 - t0)
    ms_step = dt / args.steps * 1e3
    cells_per_step = N ** 3 * (grp.world if scaling == "weak" else 1)
    value = cells_per_step / (ms_step * 1e-3) / 1e6
    info = results[0][0]
    mines = [e.local_info() for e in engines]
    mine = mines[0]
    if any((m.ctMPUs, m.ctVertices, m.ctTriangles) != (mine.ctMPUs, mine.ctVertices, mine.ctTriangles)
           for m in mines):
        sys.exit(f"bench.py rank {grp.rank}: the engines' last runs differ")

    counts = grp.allgather([mine.ctMPUs, mine.ctVertices, mine.ctTriangles])
    check = None
    if full is not None:  # the parts must add up to the full grid of the planning run
        tot = [sum(c[i] for c in counts) for i in range(3)]
        ok = tot == [full.ctMPUs, full.ctVertices, full.ctTriangles]
        if engines[0].comm:
            ok = ok and (info.ctMPUs, info.ctVertices, info.ctTriangles) == tuple(tot)
        check = {"parts_sum_to_full_grid": ok, "full": [full.ctMPUs, full.ctVertices, full.ctTriangles]}
        if not ok:
            sys.exit(f"bench.py rank {grp.rank}: parts {counts} do not add up to the full grid {check['full']}")

    # roofline pass 1: the timed steps again, identically (K steps alternating between the
    # engines, queued without host sync), with every launch recording its kernels' spans on
    # the device clock (first wave start -> last wave end: one 64-bit atomic min / max per
    # wave); per kernel, the average over all K launches
    per_engine = (args.steps + neng - 1) // neng + 1
    for e in engines:
        e.set_option(gpu.OPT_SPANS, per_engine)
    grp.barrier()
    for k in range(args.steps):
        engines[k % neng].polygonize()
    for e in engines:
        e.finish()
    spr = np.concatenate([e.spans(raw=True) for e in engines])  # (launches, kernels, {start, end})
    sp = (spr[:, :, 1] - spr[:, :, 0]) * 1e-5
    for e in engines:
        e.set_option(gpu.OPT_SPANS, 0)
    launches = len(sp)
    kt = {k: float(sp[:, i].mean()) for i, k in enumerate(gpu.STAMP_KERNELS)}
    # k_front (PSGPU_OPT_FRONT): k_precheck's and k_mpu's waves are the S1 and S2 blocks of ONE
    # launch; its span is theirs together
    front = bool(mine.launchFlags & gpu.LAUNCH_FRONT)
    if front:
        kt["k_front"] = float(((np.maximum(spr[:, 0, 1], spr[:, 1, 1]) - np.minimum(spr[:, 0, 0], spr[:, 1, 0]))
                               * 1e-5).mean())
    fmpus = sum(e.local_info().ctFieldMPUs for e in engines) / neng * launches / nparts
    # pass 2: hipEvent brackets around each kernel (they add the dispatch gap before each
    # launch), in bursts alternating between the engines; the sample is the run of the engine
    # that is not last in its burst
    for e in engines:
        e.set_option(gpu.OPT_KERNEL_TIMING, 1)
    kt_sum, ev_n = {}, 0
    reps = max(4, min(args.steps, 20))
    for rep in range(reps):
        order = engines[rep % neng:] + engines[:rep % neng]
        for k in range(3 * neng):
            order[k % neng].polygonize()
        for e in engines:
            e.finish()
        for ev in order[0].event_times():
            for k, v in ev.items():
                kt_sum[k] = kt_sum.get(k, 0.0) + v
            ev_n += 1
    for e in engines:
        e.set_option(gpu.OPT_KERNEL_TIMING, 0)
    ev_ms = {k: v / ev_n for k, v in kt_sum.items()}
    if front:  # the hipEvent pair before / after the one launch ("k_precheck"; "k_mpu" brackets nothing)
        ev_ms["k_front"] = ev_ms.pop("k_precheck", 0.0)
        ev_ms.pop("k_mpu", None)
    fused = int(os.environ.get("PSGPU_FUSED_SURFACE", "2"))
    for e in engines:
        e.set_option(gpu.OPT_STAMPS, 1 << 17)
        if fused == 2:  # the timed regime's launches: a lone run would otherwise fuse k_vertex + k_finish
            e.set_option(gpu.OPT_FUSED_SURFACE, 1 if mine.launchFlags & gpu.LAUNCH_SURFACE else 0)
    # the same launches with the device to themselves (engine 0 alone): the per-kernel
    # figure without the other engine's kernels sharing the CUs
    solo_sum, solo_n, solo_fm = {}, 0, 0
    for _ in range(reps):
        engines[0].polygonize()
        for spn, fm in engines[0].stamp_spans():
            for k, v in spn.items():
                solo_sum[k] = solo_sum.get(k, 0.0) + v
            solo_fm += fm
            solo_n += 1
    for e in engines:
        e.set_option(gpu.OPT_STAMPS, 0)
        if fused == 2:
            e.set_option(gpu.OPT_FUSED_SURFACE, 2)
    solo = {k: v / solo_n for k, v in solo_sum.items()}
    single = mine
    # the dominant kernel: the longest launch with the device to itself (the replay spans of
    # concurrent engines stretch whichever kernel overlaps the other engine's work); with
    # k_front, its S1 / S2 wave spans are reported but the launch is k_front
    launch_names = [k for k in solo if not (front and k in ("k_precheck", "k_mpu"))]
    dom = max(launch_names, key=solo.get) if launch_names else max(kt, key=kt.get)
    # lane-evaluations one launch processes, on average (SURVEY.md §8(d) units) ...
    launch_evals = {"k_precheck": 8 * single.ctMPUs / nparts, "k_mpu": 512 * fmpus / launches,
                    "k_vertex": 4 * single.ctVertices / nparts, "k_finish": 4 * single.ctVertices / nparts}
    launch_evals["k_front"] = launch_evals["k_precheck"] + launch_evals["k_mpu"]
    # ... times the fp32 ops per lane-evaluation of that stage that the reference executes on
    # this input (its own op-box pruning included; the oracle's counters priced by
    # parsip_amd/costmodel.py, tests/golden/workload_ops.json); else the unpruned figure
    wops = workload_ops(args.config) if scaling == "weak" or grp.world == 1 else None
    unpruned = costmodel.ops_per_eval(model)

    def eval_price(k):  # fp32 ops per lane-evaluation of stage k, and where the figure comes from
        if wops and wops.get("vertices") == single.ctVertices and k in wops:
            ref_evals = {"k_precheck": 8 * mine.ctMPUs, "k_mpu": 512 * wops["passed_s1"],
                         "k_vertex": 4 * wops["vertices"], "k_finish": 4 * wops["vertices"]}[k]
            return wops[k] / ref_evals, "tests/golden/workload_ops.json (reference-executed ops per eval)"
        return unpruned, "costmodel.ops_per_eval (unpruned tree)"
    if dom == "k_front":  # S1's and S2's evaluations, each at its stage's price
        (pp, per_src), (pm, _) = eval_price("k_precheck"), eval_price("k_mpu")
        alg_ops = launch_evals["k_precheck"] * pp + launch_evals["k_mpu"] * pm
        per_eval = alg_ops / launch_evals["k_front"]
    else:
        per_eval, per_src = eval_price(dom)
        alg_ops = launch_evals[dom] * per_eval
    # the launch duration: hipEvent pairs on the engine's stream in the timed regime (the
    # contract's measure; it agrees with rocprofv3's mean for the same command), the
    # device-clock span of the replay beside it
    dur = ev_ms.get(dom) or kt[dom]
    achieved = alg_ops / (dur * 1e-3) / 1e12
    # the committed PMC / traffic passes of the tier that was timed (tools/gpu_round.sh profiles
    # the bench command twice: --jit 2, the baked kernels -> rNN_pmc.json / rNN_traffic.json;
    # --jit 1, the structure kernels -> rNN_pmc_structure.json / rNN_traffic_structure.json;
    # each file records the jit mode it ran)
    prof_ok = args.config == "C3" and grp.world == 1 and (nparts, neng) == (1, ENGINES_DEFAULT) and timed_jit in (1, 2)
    suffix = "" if timed_jit == gpu.JIT_BAKED else "_structure"
    pmc, pmc_src = committed_profile("pmc" + suffix, timed_jit)
    pe = profile_entry(pmc, dom, timed_jit) if prof_ok else None
    tr, tr_src = committed_profile("traffic" + suffix, timed_jit)
    te = profile_entry(tr, dom, timed_jit) if prof_ok else None
    lk = {"bound": "valu", "pipe": "fp32 VALU (no MFMA: scalar field evaluation; SURVEY.md §8(d))",
            "kernel": dom, "achieved": round(achieved, 3), "peak": NOFMA_PEAK_TOPS, "unit": "T op/s",
            "frac": round(achieved / NOFMA_PEAK_TOPS, 4),
            "traffic": round(te["traffic_bytes"]) if te and "traffic_bytes" in te else None,
            "traffic_source": tr_src if te else None,
            # the bytes the launch must move (k_mpu: its records and counts out, its queue in)
            "traffic_required": (round(8 * single.ctVertices / nparts + 8 * single.ctTriangles / nparts
                                       + 8 * single.ctMPUs / nparts + 20 * fmpus / launches)
                                 if dom == "k_mpu" else None),
            "traffic_required_note": "k_mpu: 8 B vertex key per vertex + 8 B triangle record per triangle + "
                                     "8 B count per MPU written, 4 B queue entry + 16 B culling mask per "
                                     "S2-evaluated MPU read" if dom == "k_mpu" else None,
            "kernel_ms": round(dur, 4), "kernel_ms_source": "hipEvent pair around each launch on its engine's "
            "stream, the engines' steps queued in bursts as in the timed loop (mean over the bursts)",
            "kernel_ms_span": round(kt[dom], 4), "kernel_ms_span_source": "device-clock span per launch (first "
            "wave start to last wave end, s_memrealtime), averaged over an identical replay of the K timed steps",
            "launches_timed": launches,
            "lane_evals": round(launch_evals[dom]),
            "ops_per_eval": round(per_eval, 1), "ops_per_eval_source": per_src, "algorithmic_ops": round(alg_ops),
            "note": "per launch: achieved = the lane-evaluations one launch performs (k_mpu: 512 x S2-evaluated "
                    "MPUs of its part; k_front: k_precheck's 8 per MPU + k_mpu's, each at its stage's price) x "
                    "the reference's fp32 ops per evaluation / its duration in the timed "
                    "regime (engines alternating, queued: the launches of the other engines share the CUs); "
                    "'isolated' is the same launch with the device to itself. Exact per-wave "
                    "culling skips part of those ops, so valu_issue (executed VALU instructions x 2 cycles per "
                    "wave64 on SIMD-32 / launch cycles, PMC pass of this command) is the hardware-side "
                    "utilisation"}
    lk["kernels_ms"] = {k: {"span": round(kt[k], 4), "hipevent": round(ev_ms.get(k, 0.0), 4),
                              "isolated": round(solo.get(k, 0.0), 4)} for k in kt}
    if dom in solo:
        solo_evals = dict(launch_evals, k_mpu=512 * solo_fm / solo_n,
                          k_front=launch_evals["k_precheck"] + 512 * solo_fm / solo_n)[dom]
        a_solo = solo_evals * per_eval / (solo[dom] * 1e-3) / 1e12
        lk["isolated"] = {"kernel_ms": round(solo[dom], 4), "achieved": round(a_solo, 3),
                            "frac": round(a_solo / NOFMA_PEAK_TOPS, 4),
                            "note": "engine 0 alone on the device (no concurrent engine), same launches"}
        if a_solo > NOFMA_PEAK_TOPS:
            lk["isolated"]["frac"] = None
            lk["isolated"]["note"] += FRAC_OVER_NOTE
    if achieved > NOFMA_PEAK_TOPS:
        lk["frac"] = None
        lk["note"] += ";" + FRAC_OVER_NOTE
    if pe and "SQ_INSTS_VALU" in pe:
        lk["valu_issue"] = round(pe["SQ_INSTS_VALU"] * 2 / (dur * 1e-3 * 2.4e9 * 1024), 4)
        if dom in solo and "isolated" in lk:
            lk["isolated"]["valu_issue"] = round(pe["SQ_INSTS_VALU"] * 2 / (solo[dom] * 1e-3 * 2.4e9 * 1024), 4)
        lk["valu_source"] = pmc_src
    if te and "avg_us" in te:
        lk["rocprof_avg_us"] = te["avg_us"]
    # primary figure: the executed VALU work of a whole step against the device's VALU issue
    # capacity over ms_per_step (verdict r02): per-step VALU instructions = sum over the
    # step's kernels of (mean SQ_INSTS_VALU per launch x launches per step) from the
    # committed PMC pass of this command; one wave64 VALU instruction occupies a SIMD-32 for
    # 2 cycles, so issue = instr x 2 / (step seconds x 2.4 GHz x 1024 SIMDs), <= 1 by
    # construction; the same work in lane-ops (instr x 64, inactive lanes included) against the
    # no-FMA fp32 ceiling (78.6 T op/s; the FMA peak 157.3 TFLOP/s does not apply to
    # -ffp-contract=off code) is the same fraction.
    step = None
    if pmc and prof_ok:
        ks = {k: v for k, v in pmc.items() if "SQ_INSTS_VALU" in v and "probe" not in k}
        first = profile_entry(pmc, "k_precheck", timed_jit) or profile_entry(pmc, "k_front", timed_jit)
        steps_prof = (first or {}).get("launches")
        if ks and steps_prof:
            instr = sum(v["SQ_INSTS_VALU"] * v.get("launches", steps_prof) for v in ks.values()) / steps_prof
            sec = ms_step * 1e-3
            issue = instr * 2 / (sec * 2.4e9 * 1024)
            lane_tops = instr * 64 / sec / 1e12
            tr_step = None
            tfirst = (profile_entry(tr, "k_precheck", timed_jit) or profile_entry(tr, "k_front", timed_jit)) if tr else None
            if tfirst and tfirst.get("calls"):  # launches per step from the kernel-trace call counts
                tr_step = sum(v.get("traffic_bytes", 0.0) * v.get("calls", tfirst["calls"]) / tfirst["calls"]
                              for k, v in tr.items() if "probe" not in k)
            step = {"bound": "valu", "kernel": "whole step (" + ", ".join(sorted(ks)) + ")",
                    "achieved": round(lane_tops, 3), "peak": NOFMA_PEAK_TOPS, "unit": "T op/s",
                    "frac": round(lane_tops / NOFMA_PEAK_TOPS, 4), "valu_issue": round(issue, 4),
                    "traffic": round(tr_step) if tr_step else None,
                    "traffic_unit": "HBM bytes per step (sum of the kernels' FETCH_SIZE x 2 + WRITE_SIZE)",
                    "valu_instr_per_step": round(instr),
                    "source": pmc_src, "traffic_source": tr_src if tr_step else None,
                    "peaks": {"no_fma_lane_ops_tops": NOFMA_PEAK_TOPS, "fma_tflops": VALU_PEAK_TFLOPS,
                              "hbm_gbs": HBM_PEAK_GBS},
                    "note": "executed work per step: sum over the step's kernels of SQ_INSTS_VALU per launch x "
                            "launches per step (committed PMC pass of this command), x 64 lanes / ms_per_step "
                            "(inactive lanes counted: an upper bound on lane-ops); frac = that / 78.6 T op/s, the "
                            "fp32 VALU ceiling without FMA (the code is built with -ffp-contract=off), which "
                            "equals valu_issue = instr x 2 cycles / (step x 2.4 GHz x 1024 SIMD-32). The "
                            "reference-priced per-launch figure of the dominant kernel is 'per_launch'"}
    roof = step if step else dict(lk)
    roof["per_launch"] = lk

    # what the timed steps ran, per engine: 0 interpreter, 1 structure kernels, 2 baked kernels
    tiers_timed = [e.jit_tier() for e in engines]
    if args.jit and not jit_on:
        kernels_label = "interpreter (jit unavailable)"
    elif args.jit == gpu.JIT_TIERED:
        kernels_label = ("jit-tiered: baked tier" if timed_jit == gpu.JIT_BAKED
                         else "jit-tiered: structure tier (the baked kernels were not ready)")
    else:
        kernels_label = ["interpreter", "jit-structure", "jit-baked"][args.jit]
    out = {
        "metric": METRIC if args.config == "C3" else METRIC_OTHER.format(
            n=N, p=model.ct_prims, config=args.config, g=grp.world),
        "value": round(value, 2),
        "unit": "Mcells/s",
        "n_gpus": grp.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: {args.config} BlobTree from std::mt19937(42) as in the reference probe (SURVEY.md §6, §8(d))",
        "config": {"workload": (f"{args.config}: {model.ct_prims}-prim/{model.ct_ops}-op BlobTree, {N}^3 cells, "
                                f"{n_mpus} MPUs")
                               + (" split over the ranks (C4)" if full is not None else "")
                               + (", a grid per rank (frame = rank)" if scaling == "weak" and grp.world > 1 else ""),
                   "grid": N, "mpus": n_mpus, "prims": model.ct_prims, "ops": model.ct_ops,
                   "parallelism": f"{scaling}-{grp.world}gpu", "engines_per_gpu": neng, "parts_per_engine": nparts,
                   "streams_per_gpu": neng * nparts,
                   "persistent_blocks_per_cu": [args.vertex_blocks or (8 if neng > 1 else 16),
                                                args.finish_blocks or (4 if neng > 1 else 8)],
                   "grids": "k_vertex / k_finish: a wave per batch of the last run's vertices + 1/8, at most "
                            "the persistent grids" if os.environ.get("PSGPU_GRID_FIT", "1") != "0" else "persistent",
                   "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                   "step": "one complete polygonization of the rank's MPU range (S1-S6: k_precheck + k_mpu, "
                           "one launch when launch_flags says k_front, then k_vertex + k_finish, or k_surface); "
                           "steps alternate between the engines and are queued without host sync",
                   "launch_flags": {"k_front": front, "tree_split": bool(mine.launchFlags & gpu.LAUNCH_TREE_SPLIT),
                                    "k_surface": bool(mine.launchFlags & gpu.LAUNCH_SURFACE)},
                   "mpu_range_rank0": [begin, end] if grp.rank == 0 else None,
                   "exchange": exchange, "culling": not args.no_cull, "tree_split": args.tree_split,
                   "fused_surface": ("auto: k_vertex + k_finish as one launch when both take their quad layouts"
                                     if args.tree_split and os.environ.get("PSGPU_FUSED_SURFACE", "2") != "0"
                                     else "off"),
                   "kernels": kernels_label, "tiers": tiers_timed, "set_model_s": round(t_model, 4),
                   "jit_ready_s": round(t_jit, 3),
                   "host_enqueue_ms": round((t_enq - t0) * 1e3, 4)},
        "roofline": roof,
        "kernel_ms_per_launch": {k: round(v, 4) for k, v in kt.items()},
        "kernel_ms_per_launch_hipevent": {k: round(v, 4) for k, v in ev_ms.items()},
        "kernel_ms_per_launch_isolated": {k: round(v, 4) for k, v in solo.items()},
        "mesh": {"vertices": info.ctVertices, "triangles": info.ctTriangles, "passed_s1": info.ctPassedPrecheck,
                 "surface_mpus": info.ctSurfaceMPUs, "field_mpus": info.ctFieldMPUs, "per_rank": counts},
        "hbm_gbs_algorithmic": round((mine.ctVertices * 36 + mine.ctTriangles * 12) / (ms_step * 1e-3) / 1e9, 2),
    }
    if tier:
        out["config"]["tiered"] = tier
    if check:
        out["check"] = check
    if split_log:
        out["config"]["split"] = dict(split_log, note="cost split (psgpu_split_costs) refined from all-gathered "
                                      "measured step times before the timed steps (gpu.rebalance)")
    if grp.rank == 0 and grp.world == 1 and not args.no_extras:
        lat = latency_single(engines[0].p if engines[0].p is not None else poly, cs)
        out["latency_ms_single"] = {"median": lat[0], "best": lat[1],
                                    "note": "one engine, one polygonization at a time, host-timed "
                                            "(enqueue + kernel chain + sync): a blocking caller's latency"}
        out["latency_ms_single_parts"] = latency_single_parts(device, model, cs, args.jit)
        # the drop-ins' blocking contract (psgpu::Polygonize / gpu.Polygonize: one context), C2
        # and the headline's C3; beside it C3 on a 2-part group of the device (shorter kernels,
        # the same whole call: DESIGN.md §4 "Blocking")
        out["blocking_polygonize_mpus"] = blocking_contract({"one": poly}, "C2")["one"]
        bg = gpu.Group([device, device])
        try:
            bg.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
            bg.set_option(gpu.GROUP_OPT_MIN_PART_MPUS, gpu.BLOCKING_MIN_PART_MPUS)
            bg.set_option(gpu.OPT_JIT, args.jit)
            b3 = blocking_contract({"one": poly, "2parts": bg}, "C3")  # calls alternate
            out["blocking_polygonize_mpus_c3"] = b3["one"]
            out["blocking_polygonize_mpus_c3_2parts"] = b3["2parts"]
        finally:
            bg.close()
    if grp.rank == 0 and grp.world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(model, cs, N ** 3, args.config)
    if grp.rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    for e in engines:
        e.close()
    if grp.dist:
        grp.dist.destroy_process_group()
    poly.close()


if __name__ == "__main__":
    main()
