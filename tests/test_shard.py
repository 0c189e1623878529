"""Multi-rank partition of the MPU lattice on CPU, through the product's
own split: psgpu_split_costs (host-only C-ABI, loads without a GPU) and the rank arithmetic
bench.py uses (gpu.rank_range, gpu.exclusive_bases).  world_size-2 gloo processes each
polygonize their contiguous MPU range with the oracle standing in for the device, exchange
(MPUs, V, T) counts and must reassemble the single-process mesh exactly."""
import os
import socket

import numpy as np

from parsip_amd import gpu


def oracle_costs(stats) -> np.ndarray:
    """Per-MPU lane-evaluation costs in psgpu_mpu_costs' units from the oracle's statistics
    (columns: passed S1, evals, V, T, overflow): 8 for S1, 512 for an S2 cache, 8 per
    vertex (the oracle proves nothing empty)."""
    return (8 + 512 * (stats[:, 0] != 0) + 8 * stats[:, 2].astype(np.int64)).astype(np.uint32)


def test_split_covers_in_order_and_balances():
    rng = np.random.default_rng(0)
    w = np.where(rng.uniform(size=10000) < 0.3, 512, 8).astype(np.uint32)
    w[:2000] = 8  # empty corner of the box
    for world in (1, 2, 3, 8):
        r = [gpu.rank_range(w, world, k) for k in range(world)]
        assert r[0][0] == 0 and r[-1][1] == len(w)
        assert all(a[1] == b[0] for a, b in zip(r[:-1], r[1:]))
        loads = [int(w[a:b].sum()) for a, b in r]
        assert max(loads) - min(loads) <= 2 * 512 + 8
    assert [gpu.rank_range(np.zeros(0, np.uint32), 2, k) for k in range(2)] == [(0, 0), (0, 0)]
    # the group form splits a sub-range starting at `begin`
    b = gpu.split_costs(w[100:900], 3, 100)
    assert b[0] == 100 and b[-1] == 900 and np.all(np.diff(b.astype(np.int64)) >= 0)


def test_exclusive_bases():
    off = gpu.exclusive_bases([[10, 100, 150], [5, 40, 60], [7, 0, 0]])
    np.testing.assert_array_equal(off, [[0, 0, 0], [10, 100, 150], [15, 140, 210]])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import psoracle
    import torch
    import torch.distributed as dist

    from parsip_amd import gpu, synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, cs, _ = synth.make_config("C2")
        # the planning run (bench.py: one full run on every rank, deterministic) -> costs
        plan = psoracle.polygonize(model, cs, threads=2)
        begin, end = gpu.rank_range(oracle_costs(plan.stats), world, rank)
        om = psoracle.polygonize(model, cs, begin, end, threads=2)
        mine = torch.tensor([end - begin, len(om.pos), len(om.tris)], dtype=torch.int64)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        counts = [c.tolist() for c in allc]
        # bench.py's check: the parts add up to the full grid of the planning run
        assert [sum(c[i] for c in counts) for i in range(3)] == [len(plan.stats), len(plan.pos), len(plan.tris)]
        off = gpu.exclusive_bases(counts)
        gt = np.asarray(om.global_tris(), np.int64) + int(off[rank][1])
        parts = [None] * world
        dist.all_gather_object(parts, (om.stats, om.pos, gt, (begin, end)))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_reassemble(oracle):
    import torch.multiprocessing as mp

    from parsip_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    model, cs, _ = synth.make_config("C2")
    full = oracle.polygonize(model, cs, threads=4)
    # a cost-balanced split, not the even one: the empty corner of the box weighs less
    (b0, e0), (b1, e1) = parts[0][3], parts[1][3]
    assert b0 == 0 and e0 == b1 and e1 == len(full.stats) and e0 != len(full.stats) // 2
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), full.stats)
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]).view(np.uint32), full.pos.view(np.uint32))
    np.testing.assert_array_equal(np.concatenate([p[2] for p in parts]), full.global_tris())


def test_rebalance_moves_work_off_the_slow_rank():
    """gpu.rebalance (bench.py's measured-time balancing): a rank that measured slower than its
    cost share gets a smaller range; equal times keep the split; the ranges stay a contiguous
    cover in order."""
    rng = np.random.default_rng(1)
    c = rng.integers(8, 600, size=20000).astype(np.uint32)
    b = gpu.split_costs(c, 4)
    same = gpu.rebalance(c, b, [1.0, 1.0, 1.0, 1.0])
    assert np.all(np.abs(same.astype(np.int64) - b.astype(np.int64)) <= 2)
    nb = gpu.rebalance(c, b, [1.0, 2.0, 1.0, 1.0])  # rank 1 took twice as long
    assert nb[0] == 0 and nb[-1] == len(c) and np.all(np.diff(nb.astype(np.int64)) >= 0)
    assert nb[2] - nb[1] < b[2] - b[1]
    # predicted times under the measured rates are now closer to equal
    rate = np.zeros(len(c))
    for r, t in enumerate([1.0, 2.0, 1.0, 1.0]):
        rate[b[r]:b[r + 1]] = t / c[b[r]:b[r + 1]].sum()
    pred = [float((c[nb[r]:nb[r + 1]] * rate[nb[r]:nb[r + 1]]).sum()) for r in range(4)]
    assert max(pred) / min(pred) < 1.05
