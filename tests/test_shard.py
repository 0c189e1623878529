"""Multi-rank partition of the MPU lattice (parsip_amd/shard.py) on CPU:
world_size-2 gloo processes, each polygonizing its contiguous MPU range with the oracle
standing in for its device, exchange (MPUs, V, T) counts and must reassemble the
single-process mesh exactly."""
import os
import socket

import numpy as np
import pytest

from parsip_amd import shard


def test_even_ranges_cover_in_order():
    for n in (0, 1, 7, 50653):
        for w in (1, 2, 3, 8):
            r = shard.mpu_ranges(n, w)
            assert r[0][0] == 0 and r[-1][1] == n and len(r) == w
            assert all(a[1] == b[0] for a, b in zip(r[:-1], r[1:]))
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 1


def test_weighted_ranges_balance():
    rng = np.random.default_rng(0)
    w = np.where(rng.uniform(size=10000) < 0.3, 512.0, 8.0)
    w[:2000] = 8.0  # empty corner of the box
    r = shard.mpu_ranges(len(w), 4, w)
    assert r[0][0] == 0 and r[-1][1] == len(w)
    loads = [w[a:b].sum() for a, b in r]
    assert max(loads) / min(loads) < 1.05


def test_exclusive_offsets():
    off = shard.exclusive_offsets([[10, 100, 150], [5, 40, 60], [7, 0, 0]])
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

    from parsip_amd import shard, synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, cs, _ = synth.make_config("C2")
        n = psoracle.count_mpus(cs, *model.bbox)
        begin, end = shard.mpu_ranges(n, world)[rank]
        om = psoracle.polygonize(model, cs, begin, end, threads=2)
        mine = torch.tensor([end - begin, len(om.pos), len(om.tris)], dtype=torch.int64)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        off = shard.exclusive_offsets([c.tolist() for c in allc])
        gt = shard.globalize_triangles(om.global_tris(), off[rank][1])
        parts = [None] * world
        dist.all_gather_object(parts, (om.stats, om.pos, gt))
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
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), full.stats)
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]).view(np.uint32), full.pos.view(np.uint32))
    np.testing.assert_array_equal(np.concatenate([p[2] for p in parts]), full.global_tris())
