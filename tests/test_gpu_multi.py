"""One grid over several parts, on the HIP path.

The reference's Polygonize fans the MPU list over every core in one call
(PS_Polygonizer.cpp:379-382); psgpu_group_* fans it over device contexts and
psgpu_comm_* exchanges the parts' counts over RCCL when there is one process per GPU.
On the one-GPU test box the parts share device 0 (a group may put several parts on one
device); the reassembled mesh must equal the committed single-device oracle digests.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from parity_util import assert_bits_equal, assert_mesh_matches, mesh_digests
from parsip_amd import gpu, soa, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _stats4(polys_stats):
    st = np.concatenate(polys_stats)
    return np.stack([st["passedPrecheck"], st["ctFieldEvals"], st["ctVertices"], st["ctTriangles"]], axis=1)


def _group_stats(group):
    return [group_ctx_stats(group, p) for p in range(group.n)]


def group_ctx_stats(group, part):
    """PsMpuStats of one part through the C-ABI (psgpu_download_stats on its context)."""
    L = gpu.load()
    info, parts = group.finish()
    n = parts[part].info.ctMPUs
    st = np.zeros(max(n, 1), soa.MPU_STATS_DTYPE)
    rc = L.psgpu_download_stats(group.context_ptr(part), st.ctypes.data)
    assert rc == soa.RET_SUCCESS
    return st[:n]


@pytest.fixture(scope="module")
def group8():
    assert gpu.device_count() > 0, "no HIP device visible"
    g = gpu.Group([0] * 8)
    yield g
    g.close()


def test_group_c3_eight_balanced_parts_equal_golden(group8):
    """C4 rehearsal: C3 as 8 cost-balanced ranges (planning run + split), reassembled."""
    model, cs, _ = synth.make_config("C3")
    group8.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
    group8.set_model(model)
    info, parts = group8.run(cs)
    bounds = group8.split()
    assert bounds[0] == 0 and bounds[-1] == info.ctMPUs == 50653
    assert all(parts[p].mpuBegin == bounds[p] and parts[p].mpuEnd == bounds[p + 1] for p in range(8))
    # balanced by cost: lane-evaluations per part within 15 % of the mean
    evals = np.array([p.info.ctLaneEvals for p in parts], np.float64)
    assert evals.max() / evals.mean() < 1.15, evals
    dig = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["C3"]
    mesh = group8.download()
    got = mesh_digests(_stats4(_group_stats(group8)), mesh.pos, mesh.nrm, mesh.col, mesh.local_tris())
    assert got == dig
    # the device gather (peer copies + rebase kernel) equals the host reassembly
    d = group8.gather(0)
    import ctypes

    L = gpu.load()
    V, T = info.ctVertices, info.ctTriangles
    pos = np.zeros((V, 3), np.float32)
    tris = np.zeros((T, 3), np.uint32)
    offs = np.zeros(info.ctMPUs + 1, np.uint64)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(pos.ctypes.data, d.pos, pos.nbytes, 2) == 0
    assert hip.hipMemcpy(tris.ctypes.data, d.tris, tris.nbytes, 2) == 0
    assert hip.hipMemcpy(offs.ctypes.data, d.mpuOffsets, offs.nbytes, 2) == 0
    assert_bits_equal(pos, mesh.pos, "gathered positions")
    np.testing.assert_array_equal(tris, mesh.tris)
    np.testing.assert_array_equal((offs & 0xFFFFFFFF).astype(np.int64), mesh.vertex_offsets)
    np.testing.assert_array_equal((offs >> 32).astype(np.int64), mesh.triangle_offsets)
    assert L is not None


def test_print_thread_results_one_entry_per_part(oracle):
    """PrintThreadResults over a 2-part group (two contexts = two workers) after two runs of
    C2: entry k holds part k's MPUs and MPUs with triangles (summed, / ctAttempts), in the
    order the parts first finished; the sums are the oracle's MPUs and surface MPUs."""
    m, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(m, cs, threads=8)
    g = gpu.Group([0, 0])
    try:
        g.set_model(m)
        gpu.PrintThreadResults(1, echo=False)  # clear what earlier tests left
        for _ in range(2):
            info, parts = g.run(cs)
        n = gpu.thread_result_count()
        assert n == 2
        pr, cr = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        assert gpu.PrintThreadResults(2, pr, cr) == 2
        assert gpu.thread_result_count() == 0
        assert list(pr) == [parts[k].info.ctMPUs for k in range(2)]
        assert list(cr) == [parts[k].info.ctSurfaceMPUs for k in range(2)]
        assert int(pr.sum()) == len(om.stats) and int(cr.sum()) == int((om.stats[:, 3] > 0).sum())
    finally:
        g.close()


@pytest.mark.parametrize("policy", [gpu.BALANCE_EVEN, gpu.BALANCE_EVERY_RUN])
def test_group_c2_policies_match_oracle(group8, oracle, policy):
    model, cs, _ = synth.make_config("C2")
    group8.set_option(gpu.GROUP_OPT_BALANCE, policy)
    group8.set_model(model)
    for _ in range(2):  # EVERY_RUN re-splits after the first finish
        group8.run(cs)
    mesh = group8.download()
    om = oracle.polygonize(model, cs, threads=8)
    st = np.concatenate(_group_stats(group8))
    assert_mesh_matches(mesh, st, om)


def test_group_plan_in_chunks_equals_one_run(gpu_poly, monkeypatch):
    """The planning run goes in chunks of fewer MPUs than one run takes (2^26; lowered here
    to 1,000 so C2's 6,859 MPUs plan in 7 runs): the split equals the one-run plan's."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    gpu_poly.run(cs)
    want = [int(x) for x in gpu.split_costs(gpu_poly.mpu_costs(), 3)]
    monkeypatch.setenv("PSGPU_PLAN_CHUNK_MPUS", "1000")
    g = gpu.Group([0] * 3)
    try:
        g.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
        g.set_model(model)
        info, _ = g.run(cs)
        assert [int(x) for x in g.split()] == want
        assert info.ctVertices == gpu_poly.finish().ctVertices
    finally:
        g.close()


def test_group_min_part_mpus(oracle):
    """PSGPU_GROUP_OPT_MIN_PART_MPUS (the blocking drop-ins' 16,384): C2's 6,859 MPUs run as one
    chain on part 0 (part 1 empty), 2 x 1,000 splits it; the mesh is the oracle's either way."""
    model, cs, _ = synth.make_config("C2")
    g = gpu.Group([0, 0])
    try:
        g.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
        g.set_option(gpu.GROUP_OPT_MIN_PART_MPUS, gpu.BLOCKING_MIN_PART_MPUS)
        g.set_model(model)
        info, parts = g.run(cs)
        assert [int(x) for x in g.split()] == [0, 6859, 6859]
        assert parts[1].info.ctMPUs == 0 and info.ctMPUs == 6859
        om = oracle.polygonize(model, cs, threads=8)
        assert_mesh_matches(g.download(), np.concatenate(_group_stats(g)), om)
        g.set_option(gpu.GROUP_OPT_MIN_PART_MPUS, 1000)
        info, parts = g.run(cs)
        b = [int(x) for x in g.split()]
        assert 0 < b[1] < 6859 and b[2] == 6859
        assert_mesh_matches(g.download(), np.concatenate(_group_stats(g)), om)
        rc, ct, mpus = g.polygonize_mpus(cs, model)
        assert rc == soa.RET_SUCCESS and ct == 6859
        np.testing.assert_array_equal(mpus["ctVertices"][:ct], om.stats[:, 2])
        np.testing.assert_array_equal(mpus["ctTriangles"][:ct], om.stats[:, 3])
    finally:
        g.close()


def test_group_fixed_split_with_empty_parts(group8, oracle):
    model, cs, _ = synth.make_config("C2")
    n = gpu.count_mpus(cs, *model.bbox)
    group8.set_model(model)
    group8.set_split([0, 0, 17, 17, n // 2, n // 2 + 1, n - 3, n, n])
    info, parts = group8.run(cs)
    assert [p.mpuEnd - p.mpuBegin for p in parts] == [0, 17, 0, n // 2 - 17, 1, n - 3 - n // 2 - 1, 3, 0]
    mesh = group8.download()
    om = oracle.polygonize(model, cs, threads=8)
    assert_mesh_matches(mesh, np.concatenate(_group_stats(group8)), om)


def test_group_export_polympus_equals_single_context(group8, gpu_poly):
    model, cs, _ = synth.make_config("C2")
    group8.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
    group8.set_model(model)
    group8.run(cs)
    a = group8.export_polympus()
    gpu_poly.set_model(model)
    gpu_poly.run(cs)
    b = gpu_poly.export_polympus()
    assert a.tobytes() == b.tobytes()
    # the reference capacity of PolyMPUs (24,000) is too small for 50,653 MPUs: -4, no export
    model3, cs3, _ = synth.make_config("C3")
    group8.set_model(model3)
    group8.run(cs3)
    with pytest.raises(gpu.PsgpuError) as e:
        group8.export_polympus(capacity=soa.MAX_MPU_COUNT)
    assert e.value.code == -4


def test_group_blocking_c3_two_parts_equals_single_context(gpu_poly):
    """The blocking export at C3 (several ~1 MB pieces per part, the second part's packing
    queued behind the first's, one pass of the scatter threads over both parts) fills PolyMPUs
    byte for byte as one context does, call after call."""
    model, cs, _ = synth.make_config("C3")
    n = gpu.count_mpus(cs, *model.bbox)
    g = gpu.Group([0, 0])
    try:
        g.set_option(gpu.GROUP_OPT_BALANCE, gpu.BALANCE_PLAN)
        a = np.zeros(n, soa.MPU_DTYPE)
        b = np.zeros(n, soa.MPU_DTYPE)
        for _ in range(2):
            rc, ct, _ = g.polygonize_mpus(cs, model, a)
            assert rc == soa.RET_SUCCESS and ct == n
            rc, ct, _ = gpu_poly.polygonize_mpus(cs, model, b)
            assert rc == soa.RET_SUCCESS and ct == n
            assert a.tobytes() == b.tobytes()
        assert int(b["ctTriangles"].sum()) == 520224
    finally:
        g.close()


def test_rccl_exchange_single_rank(gpu_poly):
    """The RCCL path of the multi-process form at world size 1 (one GPU on this box)."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    comm = gpu.Comm(gpu_poly, gpu.comm_unique_id(), 1, 0)
    try:
        for _ in range(3):
            gpu_poly.polygonize(cs)
            comm.exchange()
        total, parts = comm.result()
        info = gpu_poly.finish()
        assert (total.ctMPUs, total.ctVertices, total.ctTriangles, total.ctPassedPrecheck) == \
            (info.ctMPUs, info.ctVertices, info.ctTriangles, info.ctPassedPrecheck)
        assert parts[0].vertexBase == 0 and parts[0].mpuEnd == info.ctMPUs
    finally:
        comm.close()


def test_rccl_exchange_after_rerun_single_rank(gpu_poly):
    """A run whose k_mpu grid fell short (test hook: debug bit 20, one block) exchanges
    incomplete totals; finish() re-runs it with the full grid, the ranks agree on a second
    exchange, and the result carries the complete totals."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    comm = gpu.Comm(gpu_poly, gpu.comm_unique_id(), 1, 0)
    try:
        gpu_poly.polygonize(cs)
        comm.exchange()
        total, _ = comm.result()
        assert not comm.reexchanged()
        ref = (total.ctMPUs, total.ctVertices, total.ctTriangles)
        gpu_poly.set_option(gpu.OPT_DEBUG, 1 << 20)
        gpu_poly.polygonize(cs)
        comm.exchange()
        total, _ = comm.result()
        assert comm.reexchanged()
        assert (total.ctMPUs, total.ctVertices, total.ctTriangles) == ref
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        comm.close()


def test_rccl_result_after_failed_finish_single_rank(gpu_poly):
    """A rank whose finish fails (test hook: debug bit 21) still enters the collective flag
    all-reduce and returns the failure; the communicator stays usable for the next step."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    comm = gpu.Comm(gpu_poly, gpu.comm_unique_id(), 1, 0)
    try:
        gpu_poly.polygonize(cs)
        comm.exchange()
        ref, _ = comm.result()
        gpu_poly.set_option(gpu.OPT_DEBUG, 1 << 21)
        gpu_poly.polygonize(cs)
        comm.exchange()
        with pytest.raises(gpu.PsgpuError) as e:
            comm.result()
        assert e.value.code == -6
        gpu_poly.polygonize(cs)
        comm.exchange()
        total, _ = comm.result()
        assert not comm.reexchanged()
        assert (total.ctMPUs, total.ctVertices, total.ctTriangles) == (ref.ctMPUs, ref.ctVertices, ref.ctTriangles)
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        comm.close()


_TWO_RANK = r"""
import os, sys
sys.path.insert(0, os.environ["PSGPU_ROOT"])
rank = int(sys.argv[1])
from parsip_amd import gpu, synth
poly = gpu.Polygonizer(rank)
import torch.distributed as dist
dist.init_process_group("gloo", rank=rank, world_size=2)
model, cs, _ = synth.make_config("C2")
poly.set_model(model)
poly.run(cs)
full = poly.finish()
b = gpu.split_costs(poly.mpu_costs(), 2)
obj = [gpu.comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
comm = gpu.Comm(poly, obj[0], 2, rank)
if rank == 1:  # only this rank's finish re-runs: both must still agree and exchange again
    poly.set_option(gpu.OPT_DEBUG, 1 << 20)
poly.polygonize(cs, int(b[rank]), int(b[rank + 1]))
comm.exchange()
total, parts = comm.result()
assert comm.reexchanged(), rank
assert (total.ctMPUs, total.ctVertices, total.ctTriangles) == (full.ctMPUs, full.ctVertices, full.ctTriangles)
if rank == 0:  # only this rank's finish fails: both ranks return an error, neither blocks
    poly.set_option(gpu.OPT_DEBUG, 1 << 21)
poly.polygonize(cs, int(b[rank]), int(b[rank + 1]))
comm.exchange()
try:
    comm.result()
    raise AssertionError(f"rank {rank}: result() succeeded after rank 0's finish failed")
except gpu.PsgpuError as e:
    assert e.code == -6, (rank, e.code)
poly.polygonize(cs, int(b[rank]), int(b[rank + 1]))  # and the next step works on both
comm.exchange()
total, parts = comm.result()
assert (total.ctMPUs, total.ctVertices, total.ctTriangles) == (full.ctMPUs, full.ctVertices, full.ctTriangles)
comm.close()
poly.close()
dist.destroy_process_group()
print("ok", rank)
"""


def test_rccl_two_ranks_one_rerun(tmp_path):
    """Two ranks over RCCL where only rank 1's finish re-runs: the re-exchange is agreed
    collectively, so neither rank blocks and both get the re-run's totals; then only rank
    0's finish fails and both ranks return the error instead of blocking (needs 2 GPUs)."""
    if gpu.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL ranks on distinct devices)")
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    script = tmp_path / "two_rank.py"
    script.write_text(_TWO_RANK)
    env = dict(os.environ, PSGPU_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    procs = [subprocess.Popen([sys.executable, str(script), str(r)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()  # the contract: stdout is the JSON line and nothing else
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


def test_bench_contract_one_gpu():
    out = _bench(["--steps", "5", "--warmup", "1", "--no-cpu"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 5 and out["warmup"] == 1
    assert out["mesh"]["vertices"] == 339820 and out["mesh"]["triangles"] == 520224
    assert 0 < out["roofline"]["frac"] <= 1 and out["roofline"]["bound"] == "valu"
    assert out["value"] > 0


def test_bench_two_ranks_strong_split_one_device():
    """`bench.py --gpus 2` spawns its two ranks itself; pinned to device 0 they split the one
    256^3 grid and their parts must add up to the full grid (checked inside the bench)."""
    out = _bench(["--gpus", "2", "--steps", "5", "--warmup", "1", "--no-cpu"], {"PSGPU_BENCH_DEVICE": "0"})
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["check"]["parts_sum_to_full_grid"] is True
    per = out["mesh"]["per_rank"]
    assert sum(p[1] for p in per) == 339820 and sum(p[2] for p in per) == 520224
    assert sum(p[0] for p in per) == 50653


@pytest.mark.parametrize("seed", [0, 4, 9, 13, 19, 38])
def test_group_fuzz_random_splits(group8, oracle, seed):
    """The fuzz trees (tests/test_gpu_fuzz.py) over 8 parts of one device at random split
    points (empty parts included): the reassembled mesh is the oracle's, and the device gather
    (peer copies + rebase kernel) equals it."""
    import ctypes

    import test_gpu_fuzz as fz

    model, cs = fz.fuzz_case(seed)[:2]
    n = gpu.count_mpus(cs, *model.bbox)
    rng = np.random.default_rng(seed)
    inner = sorted(int(x) for x in rng.integers(0, n + 1, 7))
    group8.set_model(model)
    group8.set_split([0] + inner + [n])
    info, parts = group8.run(cs)
    assert [p.mpuBegin for p in parts] == [0] + inner and info.ctMPUs == n
    mesh = group8.download()
    om = oracle.polygonize(model, cs, threads=8)
    assert_mesh_matches(mesh, np.concatenate(_group_stats(group8)), om)
    V, T = info.ctVertices, info.ctTriangles
    if V == 0:
        return
    d = group8.gather(0)
    pos = np.zeros((V, 3), np.float32)
    tris = np.zeros((T, 3), np.uint32)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(pos.ctypes.data, d.pos, pos.nbytes, 2) == 0
    assert hip.hipMemcpy(tris.ctypes.data, d.tris, tris.nbytes, 2) == 0
    assert_bits_equal(pos, mesh.pos, "gathered positions")
    np.testing.assert_array_equal(tris, mesh.tris)
