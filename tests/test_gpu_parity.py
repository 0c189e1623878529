"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical inputs.

Bar (north_star): MPU lattice, S1/S2 decisions, per-MPU vertex and
triangle counts, vertex order and triangle indices bit-exact; positions bit-exact
(north_star allows 1e-5); normals and colours bit-exact against the oracle's IEEE
1/sqrt (the reference's _mm_rsqrt_ps is CPU-vendor specific: see test_oracle.py for
the 2e-3 normal tolerance against that variant).
"""
import json
import os

import numpy as np
import pytest

from parity_util import assert_bits_equal, assert_mesh_matches, mesh_digests
from parsip_amd import gpu, soa, synth
from parsip_amd.soa import NodeType

pytestmark = pytest.mark.gpu


def run_both(poly, oracle, model, cs, begin=0, end=None, cull=1, jit=1, vwide=2, split=0):
    poly.set_option(gpu.OPT_CULLING, cull)
    poly.set_option(gpu.OPT_JIT, jit)
    poly.set_option(gpu.OPT_VERTEX_WIDE, vwide)
    poly.set_option(gpu.OPT_TREE_SPLIT, split)
    # a forced k_vertex layout must run k_vertex (a lone run otherwise takes k_surface)
    poly.set_option(gpu.OPT_FUSED_SURFACE, 2 if vwide == 2 else 0)
    poly.set_model(model)
    assert poly.jit_active == bool(jit)
    poly.run(cs, begin, end)
    gm = poly.download()
    gs = poly.stats()
    om = oracle.polygonize(model, cs, begin, 0xFFFFFFFF if end is None else end, threads=8)
    return gm, gs, om


@pytest.mark.parametrize("name", ["C1", "C2"])
@pytest.mark.parametrize("cull", [0, 1])
@pytest.mark.parametrize("jit", [0, 1])
def test_configs_bit_exact(gpu_poly, oracle, name, cull, jit):
    model, cs, _ = synth.make_config(name)
    gm, gs, om = run_both(gpu_poly, oracle, model, cs, cull=cull, jit=jit)
    assert len(gm.pos) > 0
    assert_mesh_matches(gm, gs, om)


def test_c1_reference_counts(gpu_poly):
    """C1 is PRNG-independent; SURVEY.md §6/§8(d) record the reference's own output for it
    (the survey compiled PS_Polygonizer.cpp): 125 MPUs, 109 past S1, 1,326 V, 2,024 T."""
    model, cs, _ = synth.make_config("C1")
    gpu_poly.set_model(model)
    info = gpu_poly.run(cs)
    assert (info.ctMPUs, info.ctPassedPrecheck, info.ctVertices, info.ctTriangles) == (125, 109, 1326, 2024)


@pytest.mark.parametrize("name", ["C1", "C2", "C3"])
def test_reference_counts_and_golden_digests(gpu_poly, name):
    """Counts recorded from the reference and the committed oracle digests
    (tests/golden/oracle_digests.json): full-output parity without running the oracle."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    ref = json.load(open(os.path.join(gdir, "reference_probe.json")))[name]
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))[name]
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_model(model)
    info = gpu_poly.run(cs)
    assert (info.ctMPUs, info.ctPassedPrecheck, info.ctVertices, info.ctTriangles) == \
        (ref["mpus"], ref["passed_s1"], ref["vertices"], ref["triangles"])
    gm, gs = gpu_poly.download(), gpu_poly.stats()
    st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
    assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig


@pytest.mark.parametrize("name", ["C2", "C3"])
@pytest.mark.parametrize("jit", [0, 1])
def test_finish_layouts_golden(gpu_poly, name, jit):
    """k_finish one lane per vertex (OPT_FINISH_QUAD 0), a quad (1) or a pair (3) of lanes per
    vertex and the per-run choice (2; the second run sees the first run's vertex count) all reproduce
    the committed oracle digests."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))[name]
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_option(gpu.OPT_JIT, jit)
    gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 0)  # k_finish itself (a lone run would take k_surface)
    gpu_poly.set_model(model)
    try:
        for mode in (0, 1, 3, 2, 2):
            gpu_poly.set_option(gpu.OPT_FINISH_QUAD, mode)
            gpu_poly.run(cs)
            gm, gs = gpu_poly.download(), gpu_poly.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig, (name, jit, mode)
    finally:
        gpu_poly.set_option(gpu.OPT_FINISH_QUAD, 2)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)
        gpu_poly.set_option(gpu.OPT_JIT, 1)


@pytest.mark.parametrize("name", ["C2", "C3"])
@pytest.mark.parametrize("jit", [0, 1])
def test_vertex_layouts_golden(gpu_poly, name, jit):
    """k_vertex a quad of lanes per vertex (OPT_VERTEX_WIDE 0), one lane per vertex walking its
    4 edge samples (1; the interpreter keeps the quad layout) and the per-run choice (2; the
    second run sees the first run's vertex count) all reproduce the committed oracle digests."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))[name]
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_option(gpu.OPT_JIT, jit)
    gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 0)  # k_vertex itself (a lone run would take k_surface)
    gpu_poly.set_model(model)
    try:
        for mode in (0, 1, 2, 2):
            gpu_poly.set_option(gpu.OPT_VERTEX_WIDE, mode)
            gpu_poly.run(cs)
            gm, gs = gpu_poly.download(), gpu_poly.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig, (name, jit, mode)
    finally:
        gpu_poly.set_option(gpu.OPT_VERTEX_WIDE, 2)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)
        gpu_poly.set_option(gpu.OPT_JIT, 1)


@pytest.mark.parametrize("name", ["C2", "C3", "C5"])
def test_tree_split_golden(gpu_poly, name):
    """k_precheck / k_mpu with the walk split at the root (OPT_TREE_SPLIT 1: two waves per brick
    / MPU, values combined through LDS) reproduce the committed oracle digests, then the
    unsplit kernels on the same context do again (C5: against the unsplit run)."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    digs = json.load(open(os.path.join(gdir, "oracle_digests.json")))
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_model(model)
    seen = []
    try:
        for split in (1, 1, 0):
            gpu_poly.set_option(gpu.OPT_TREE_SPLIT, split)
            gpu_poly.jit_wait()  # enabling the split compiles the split kernels
            assert gpu_poly.jit_active
            gpu_poly.run(cs)
            gm, gs = gpu_poly.download(), gpu_poly.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            seen.append(mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()))
    finally:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
    assert seen[0] == seen[1] == seen[2]
    if name in digs:
        assert seen[0] == digs[name]


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_fused_surface_golden(gpu_poly, name):
    """k_vertex + k_finish as one launch (OPT_FUSED_SURFACE 1; the small-launch kernels compile
    with OPT_TREE_SPLIT) reproduce the committed oracle digests; on a 1/8 cost share the
    automatic choice (2) takes the fused kernel from the second run on (no k_vertex waves in the
    timeline) and equals the two-kernel run."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))[name]
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_model(model)

    def digest():
        gm, gs = gpu_poly.download(), gpu_poly.stats()
        st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
        return mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris())
    try:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 1)
        gpu_poly.jit_wait()  # the split option compiles the small-launch kernels
        for mode in (1, 3):  # the quad and the one-lane-per-vertex k_surface
            gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, mode)
            for _ in range(2):
                info = gpu_poly.run(cs)
                assert info.launchFlags & gpu.LAUNCH_SURFACE
                assert digest() == dig, mode
        b = gpu_poly.plan_split(cs, 8)
        lo, hi = int(b[3]), int(b[4])
        got = {}
        for mode in (0, 2):
            gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, mode)
            gpu_poly.run(cs, lo, hi)
            gpu_poly.set_option(gpu.OPT_STAMPS, 1 << 15)
            gpu_poly.run(cs, lo, hi)
            vertex_waves = len(gpu_poly.stamps()["k_vertex"])
            gpu_poly.set_option(gpu.OPT_STAMPS, 0)
            got[mode] = digest()
            assert (vertex_waves == 0) == (mode == 2), (mode, vertex_waves)
        assert got[0] == got[2] and got[0]["vertices"] > 0
    finally:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)


@pytest.mark.parametrize("hook,fused", [(gpu.DEBUG_SURFACE_LATE_SCAN, 1), (gpu.DEBUG_LOOKBACK_TIMEOUT, 1),
                                        (gpu.DEBUG_LOOKBACK_TIMEOUT, 0)])
def test_protocol_error_reruns_two_kernels(gpu_poly, capfd, hook, fused):
    """An in-kernel wait that gives up does not fail the call: k_surface's waves waiting for a
    late offsets scan (hook 25: the scan blocks count themselves done ~40 us late, the waves
    give up after a few spins), or a look-back that times out (hook 26, in k_surface's scan
    blocks or k_vertex's) flag the run, and psgpu_finish re-runs it once as k_vertex +
    k_finish: RET_SUCCESS and the committed C2 oracle digests.  The hooks apply to one run."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))["C2"]
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)

    def digest():
        gm, gs = gpu_poly.download(), gpu_poly.stats()
        st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
        return mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris())
    try:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 1)
        gpu_poly.jit_wait()
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, fused)
        gpu_poly.run(cs)  # sizes the buffers; no hook
        capfd.readouterr()
        gpu_poly.set_option(gpu.OPT_DEBUG, hook)
        info = gpu_poly.run(cs)  # raises PsgpuError on anything but RET_SUCCESS
        err = capfd.readouterr().err
        assert "re-running as separate launches" in err, err
        assert ("k_surface" in err) == (fused == 1)
        assert (info.ctVertices, info.ctTriangles) == (32541, 50034)
        assert digest() == dig
        gpu_poly.run(cs)  # the hook is spent: no error, no re-run
        assert "protocol error" not in capfd.readouterr().err
        assert digest() == dig
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)


@pytest.mark.parametrize("name,split", [("C2", 1), ("C3", 1), ("C3", 2)])
def test_front_golden(gpu_poly, name, split):
    """k_precheck + k_mpu as one launch (OPT_FRONT 1: the S2 blocks take S1's survivors as its
    waves publish them, no grid barrier) reproduce the committed oracle digests, with the split
    kernels (jit_front_s) and without (jit_front: the split option 2 compiles the small-launch
    kernels, and a first run of the lattice does not take the split); a k_mpu grid too short
    for the sub-queues (hook, one run) is re-run with the grid they need; on a 1/8 cost share
    the automatic choice (2) takes k_front and equals the separate launches."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))[name]
    model, cs, _ = synth.make_config(name)
    gpu_poly.set_model(model)

    def digest():
        gm, gs = gpu_poly.download(), gpu_poly.stats()
        st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
        return mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris())
    try:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, split)
        gpu_poly.jit_wait()  # the split option compiles the small-launch kernels
        gpu_poly.set_option(gpu.OPT_FRONT, 1)
        gpu_poly.run(1.5 * cs)  # another lattice first: the next run has no queue history
        for k in range(3):
            if k == 1:
                gpu_poly.set_option(gpu.OPT_DEBUG, 1 << 20)  # a grid of one row of S2 blocks
            info = gpu_poly.run(cs)
            assert info.launchFlags & gpu.LAUNCH_FRONT, info.launchFlags
            assert bool(info.launchFlags & gpu.LAUNCH_TREE_SPLIT) == (split == 1)
            assert bool(info.launchFlags & gpu.LAUNCH_RERUN) == (k == 1)
            assert digest() == dig, k
        b = gpu_poly.plan_split(cs, 8)
        lo, hi = int(b[3]), int(b[4])
        got = {}
        for mode in (0, 2):
            gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 2)
            gpu_poly.set_option(gpu.OPT_FRONT, mode)
            gpu_poly.run(cs, lo, hi)
            info = gpu_poly.run(cs, lo, hi)
            assert bool(info.launchFlags & gpu.LAUNCH_FRONT) == (mode == 2), (mode, info.launchFlags)
            got[mode] = digest()
        assert got[0] == got[2] and got[0]["vertices"] > 0
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FRONT, 2)


def test_front_protocol_error_reruns(gpu_poly, capfd):
    """k_front's S2 waves give up on entries published late (hook 27: the S1 blocks publish
    ~40 us late, the pollers stop after a few polls): the run is flagged, and finish re-runs it
    as separate launches -- RET_SUCCESS and the C2 oracle digests."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))["C2"]
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    try:
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 1)
        gpu_poly.jit_wait()
        gpu_poly.set_option(gpu.OPT_FRONT, 1)
        gpu_poly.run(cs)
        capfd.readouterr()
        gpu_poly.set_option(gpu.OPT_DEBUG, gpu.DEBUG_FRONT_LATE_S1)
        info = gpu_poly.run(cs)
        err = capfd.readouterr().err
        assert "(k_front" in err and "re-running as separate launches" in err, err
        assert not info.launchFlags & gpu.LAUNCH_FRONT and info.launchFlags & gpu.LAUNCH_RERUN
        gm, gs = gpu_poly.download(), gpu_poly.stats()
        st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
        assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig
        info = gpu_poly.run(cs)  # the hook is spent
        assert info.launchFlags & gpu.LAUNCH_FRONT and not info.launchFlags & gpu.LAUNCH_RERUN
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FRONT, 2)


def test_front_epoch_wrap(gpu_poly):
    """k_front tags its queue entries with the run's epoch + 1 and takes an entry whose ready word
    holds that tag; at epoch 0xffffffff the tag would be 0, the value of every ready word no run
    has written.  Hook (debug bit 28): the context starts 3 runs short of the wrap; the runs up
    to it and the ones after the context restarts its counter sets at epoch 0 all reproduce the
    C2 oracle digests."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))["C2"]
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    try:
        gpu_poly.set_option(gpu.OPT_FRONT, 1)
        gpu_poly.run(cs)
        gpu_poly.set_option(gpu.OPT_DEBUG, gpu.DEBUG_EPOCH_NEAR_WRAP)
        for k in range(5):  # epochs 0xfffffffc, 0xfffffffd, 0xfffffffe, then 0, 1
            info = gpu_poly.run(cs)
            assert info.launchFlags & gpu.LAUNCH_FRONT and not info.launchFlags & gpu.LAUNCH_RERUN, k
            gm, gs = gpu_poly.download(), gpu_poly.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig, k
    finally:
        gpu_poly.set_option(gpu.OPT_DEBUG, 0)
        gpu_poly.set_option(gpu.OPT_FRONT, 2)


def test_engines_pipelined_c3_golden():
    """The bench's pipelining: 4 contexts take 12 C3 polygonizations in turn, queued without
    host synchronisation (bench.py's timed loop); every context's last mesh equals the
    committed oracle digests, so the queued runs do not disturb each other."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    dig = json.load(open(os.path.join(gdir, "oracle_digests.json")))["C3"]
    model, cs, _ = synth.make_config("C3")
    ps = [gpu.Polygonizer(0) for _ in range(4)]
    try:
        for p in ps:
            p.set_model(model)
            p.run(cs)  # sizes the buffers
        for k in range(12):
            ps[k % 4].polygonize(cs)
        for p in ps:
            p.finish()
            gm, gs = p.download(), p.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == dig
    finally:
        for p in ps:
            p.close()


def test_contexts_on_host_threads():
    """Four host threads, one context each (a host driving several polygonizers from its own
    worker threads): ctypes releases the GIL inside the library, so model uploads with their
    compile requests for the same two trees, polygonizations, finishes and downloads run
    concurrently; half the threads start on the interpreter while the shared compile is still
    running.  Every mesh equals its committed oracle digests, and each context's entry of the
    thread results counts its own runs."""
    import threading

    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    digs = json.load(open(os.path.join(gdir, "oracle_digests.json")))
    runs = 5
    errors, done = [], []

    def work(i):
        name = "C2" if i % 2 == 0 else "C3"
        model, cs, _ = synth.make_config(name)
        p = gpu.Polygonizer(0)
        try:
            p.set_model(model, wait_jit=i < 2)
            for k in range(runs):
                p.run(cs)
                gm, gs = p.download(), p.stats()
                st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]],
                              axis=1)
                if mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) != digs[name]:
                    errors.append((i, k, "digest"))
            done.append(i)
        except Exception as e:  # reported by the main thread
            errors.append((i, repr(e)))
        finally:
            p.close()

    gpu.PrintThreadResults(1, echo=False)  # clears the entries of earlier tests
    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a host thread did not finish"
    assert not errors, errors
    assert sorted(done) == [0, 1, 2, 3]
    n = gpu.thread_result_count()
    assert n == 4, n
    proc, crossed = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    assert gpu.PrintThreadResults(runs, proc, crossed, echo=False) == 4
    want = sorted(gpu.count_mpus(c, *m.bbox) for m, c, _ in (synth.make_config(x) for x in ("C2", "C2", "C3", "C3")))
    assert sorted(proc.tolist()) == want
    assert (crossed > 0).all() and (crossed < proc).all()


def test_engines_different_models_interleaved():
    """Contexts holding different trees (C2, C3: different generated kernels) queued in turn
    without host sync each reproduce their own oracle digests."""
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    digs = json.load(open(os.path.join(gdir, "oracle_digests.json")))
    cfg = ["C2", "C3", "C2", "C3"]
    ps = [gpu.Polygonizer(0) for _ in cfg]
    try:
        css = []
        for p, name in zip(ps, cfg):
            model, cs, _ = synth.make_config(name)
            p.set_model(model)
            p.run(cs)
            css.append(cs)
        for k in range(16):
            ps[k % 4].polygonize(css[k % 4])
        for p, name in zip(ps, cfg):
            p.finish()
            gm, gs = p.download(), p.stats()
            st = np.stack([gs["passedPrecheck"], gs["ctFieldEvals"], gs["ctVertices"], gs["ctTriangles"]], axis=1)
            assert mesh_digests(st, gm.pos, gm.nrm, gm.col, gm.local_tris()) == digs[name], name
    finally:
        for p in ps:
            p.close()


def test_c3_full_size(gpu_poly, oracle):
    """Headline workload (256^3, 32 prims, pruning live) against the oracle, in full."""
    model, cs, _ = synth.make_config("C3")
    gm, gs, om = run_both(gpu_poly, oracle, model, cs)
    assert_mesh_matches(gm, gs, om)


@pytest.mark.parametrize("jit", [0, 1, 2])
def test_c3_interpreter_and_jit(gpu_poly, oracle, jit):
    model, cs, _ = synth.make_config("C3")
    gm, gs, om = run_both(gpu_poly, oracle, model, cs, jit=jit)
    assert_mesh_matches(gm, gs, om)


@pytest.mark.parametrize("layout", ["default", "vwide", "split"])
@pytest.mark.parametrize("seed", range(6))
def test_random_trees(gpu_poly, oracle, seed, layout):
    """Random trees (every op type, matrices on odd seeds); "vwide" forces k_vertex's
    lane-per-vertex layout, whose op-box pruning groups a lane's 4 edge samples; "split" walks
    the root's two subtrees in two waves in k_precheck / k_mpu (trees whose root is a binary
    op over two ops; the others run unsplit)."""
    ops = [NodeType.BLEND, NodeType.UNION, NodeType.INTERSECT, NodeType.DIF, NodeType.SMOOTHDIF,
           NodeType.RICCIBLEND, NodeType.WARPTWIST, NodeType.GRADIENTBLEND]
    model = synth.random_model(seed, n_prims=3 + 3 * seed, op_types=ops, matrices=seed % 2 == 1)
    cs = float(np.float32(4.0 / 48))
    try:
        gm, gs, om = run_both(gpu_poly, oracle, model, cs, jit=[1, 2, 0][seed % 3],
                              vwide=1 if layout == "vwide" else 2, split=1 if layout == "split" else 0)
    finally:
        gpu_poly.set_option(gpu.OPT_VERTEX_WIDE, 2)
        gpu_poly.set_option(gpu.OPT_TREE_SPLIT, 0)
        gpu_poly.set_option(gpu.OPT_FUSED_SURFACE, 2)
    assert_mesh_matches(gm, gs, om)


def test_max_size_tree(gpu_poly, oracle):
    """The SoA limits: 128 primitives (cull masks' high word, 8-bit child ids) and 127 ops,
    every primitive type and op, matrices; interpreter kernels (the generated kernels of a
    128-primitive tree take ~2 minutes of hiprtc)."""
    ops = [NodeType.BLEND, NodeType.UNION, NodeType.INTERSECT, NodeType.DIF, NodeType.SMOOTHDIF,
           NodeType.RICCIBLEND]
    types = [NodeType.POINT, NodeType.LINE, NodeType.CYLINDER, NodeType.CUBE, NodeType.DISC, NodeType.RING,
             NodeType.TRIANGLE]
    model = synth.random_model(99, n_prims=128, types=types, op_types=ops, matrices=True)
    assert int(model.prims["ctPrims"][0]) == 128 and int(model.ops["ctOps"][0]) == 127
    cs = float(np.float32(4.0 / 40))
    for cull in (1, 0):
        gm, gs, om = run_both(gpu_poly, oracle, model, cs, cull=cull, jit=0)
        assert len(gm.pos) > 10000
        assert_mesh_matches(gm, gs, om)


def test_disc_ring_triangle_null(gpu_poly, oracle):
    """Every primitive switch case incl. rsqrt users and the no-case default."""
    types = [NodeType.DISC, NodeType.RING, NodeType.POINT, NodeType.TRIANGLE, NodeType.CUBE]
    model = synth.random_model(11, n_prims=10, types=types)
    cs = float(np.float32(4.0 / 40))
    gm, gs, om = run_both(gpu_poly, oracle, model, cs)
    assert_mesh_matches(gm, gs, om)


def test_mpu_range_partition(gpu_poly, oracle):
    """Contiguous MPU ranges (the multi-GPU split) concatenate to the full result."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_model(model)
    gpu_poly.run(cs)
    full = gpu_poly.download()
    n = gpu_poly.finish().ctMPUs
    cuts = [0, n // 3, n // 2 + 17, n]
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        gpu_poly.run(cs, a, b)
        parts.append(gpu_poly.download())
    pos = np.concatenate([p.pos for p in parts])
    assert_bits_equal(pos, full.pos, "partitioned positions")
    lt = np.concatenate([p.local_tris() for p in parts])
    np.testing.assert_array_equal(lt, full.local_tris())
    om = oracle.polygonize(model, cs, cuts[1], cuts[2], threads=8)
    gpu_poly.run(cs, cuts[1], cuts[2])
    assert_mesh_matches(gpu_poly.download(), gpu_poly.stats(), om)


def test_range_limit(gpu_poly, oracle):
    """A range holds < 2^26 MPUs (the 8-B triangle record's slot field); a larger one is a
    parameter error before any buffer is sized, and the context still polygonizes after."""
    model, cs, _ = synth.make_config("C1")
    gpu_poly.set_model(model)
    small = np.float32(cs / 128)  # C1's box at 4096^3 cells: 585^3 MPUs
    n = gpu.count_mpus(small, *model.bbox)
    assert n > 1 << 26
    for end in (None, 1 << 26):
        with pytest.raises(gpu.PsgpuError) as e:
            gpu_poly.polygonize(float(small), 0, end)
        assert e.value.code == soa.RET_PARAM_ERROR
    gm, gs, om = run_both(gpu_poly, oracle, model, cs)
    assert_mesh_matches(gm, gs, om)


def test_field_probe_quads(gpu_poly, oracle):
    model, cs, _ = synth.make_config("C3")
    gpu_poly.set_model(model)
    rng = np.random.default_rng(3)
    # quads of 4 z-consecutive points like S2, plus scattered quads
    base = rng.uniform(-4, 4, (4096, 3)).astype(np.float32)
    pts = np.repeat(base, 4, axis=0)
    pts[:, 2] += np.tile(np.arange(4, dtype=np.float32) * np.float32(1 / 32), 4096)
    g = gpu_poly.field_values(pts, mode=0)
    o = oracle.field_value(model, pts[:, 0], pts[:, 1], pts[:, 2])
    assert_bits_equal(g, o, "fieldValue (4-lane groups)")


def test_field_probe_colour(gpu_poly, oracle):
    model, cs, _ = synth.make_config("C3")
    gpu_poly.set_model(model)
    rng = np.random.default_rng(5)
    pts = rng.uniform(-3, 3, (2048, 3)).astype(np.float32)
    f, c = gpu_poly.field_values(pts, mode=2)
    rep = np.repeat(pts, 4, axis=0)
    of, oc = oracle.field_value_and_color(model, rep[:, 0], rep[:, 1], rep[:, 2])
    assert_bits_equal(f, of[::4], "fieldValueAndColor field")
    assert_bits_equal(c, oc[::4], "fieldValueAndColor colour")


def test_drop_in_polygonize(gpu_poly, oracle):
    """psgpu_polygonize_mpus fills the reference PolyMPUs layout (21,524-B MPUs)."""
    model, cs, _ = synth.make_config("C2")
    rc, ct, mpus = gpu.Polygonize(cs, model)
    assert rc == soa.RET_SUCCESS and ct == 6859
    om = oracle.polygonize(model, cs, threads=8)
    np.testing.assert_array_equal(mpus["ctVertices"][:ct], om.stats[:, 2])
    np.testing.assert_array_equal(mpus["ctTriangles"][:ct], om.stats[:, 3])
    np.testing.assert_array_equal(mpus["ctFieldEvals"][:ct], om.stats[:, 1])
    origins = soa.mpu_origins(cs, *model.bbox)
    assert_bits_equal(mpus["bboxLo"][:ct], origins, "MPU origins")
    voff = om.vertex_offsets
    toff = om.triangle_offsets
    for i in np.flatnonzero(om.stats[:, 2])[:200]:
        nv, nt = om.stats[i, 2], om.stats[i, 3]
        assert_bits_equal(mpus["vPos"][i, :nv * 3].reshape(-1, 3), om.pos[voff[i]:voff[i] + nv], "vPos")
        np.testing.assert_array_equal(mpus["triangles"][i, :nt * 3].reshape(-1, 3), om.tris[toff[i]:toff[i] + nt])
    # reference error code for an empty model
    empty = soa.Model.empty()
    assert gpu.Polygonize(cs, empty)[0] == soa.RET_PARAM_ERROR


def test_drop_in_polygonize_threads(oracle):
    """gpu.Polygonize from three host threads at once: each thread gets its own default context
    (as parsip_gpu.hpp's default_context()), every call fills PolyMPUs as the oracle does."""
    import threading

    model, cs, _ = synth.make_config("C2")
    om = oracle.polygonize(model, cs, threads=8)
    res, errors = {}, []

    def work(i):
        try:
            for k in range(2):
                rc, ct, mpus = gpu.Polygonize(cs, model)
                res[(i, k)] = (rc, ct, mpus["ctVertices"][:ct].copy(), mpus["ctTriangles"][:ct].copy(),
                               mpus["vPos"][:ct].tobytes())
        except Exception as e:  # reported by the main thread
            errors.append((i, repr(e)))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts) and not errors, errors
    assert len(res) == 6
    first = res[(0, 0)]
    for (i, k), (rc, ct, v, t, pos) in res.items():
        assert rc == soa.RET_SUCCESS and ct == 6859, (i, k)
        np.testing.assert_array_equal(v, om.stats[:, 2])
        np.testing.assert_array_equal(t, om.stats[:, 3])
        assert pos == first[4], (i, k)


def test_scene_train(gpu_poly, oracle):
    """The reference's own scene file (95 transformed prims, n-ary ops binarized) through
    the linearizer: matrices on every primitive, Ricci / Difference / Union / Blend."""
    from parsip_amd import blobtree, scene

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_corrected.scene")
    code, model = blobtree.linearize_blobtree(blobtree.binarize(scene.load_scene(path)[0]))
    assert code == 0
    gm, gs, om = run_both(gpu_poly, oracle, model, 0.2)
    assert len(gm.pos) > 10000
    assert_mesh_matches(gm, gs, om)


@pytest.mark.parametrize("cap", [64, 5000])
def test_capacity_overflow_regrows(gpu_poly, oracle, cap):
    """Compact mesh / work queues far too small: kernels must not write past them, and
    finish() grows the buffers and repeats the run (C5-sized meshes take this path)."""
    model, cs, _ = synth.make_config("C2")
    gpu_poly.set_option(gpu.OPT_CAPACITY, cap)
    gm, gs, om = run_both(gpu_poly, oracle, model, cs)
    assert_mesh_matches(gm, gs, om)


def test_graph_replay_and_frames(gpu_poly, oracle):
    """hipGraph replay of the launch sequence across model updates of one structure
    (an animation: C2 frames 0..3), each frame bit-exact to the oracle."""
    gpu_poly.set_option(gpu.OPT_GRAPH, 1)
    try:
        for f in range(4):
            model, cs, _ = synth.make_config("C2", frame=f)
            gm, gs, om = run_both(gpu_poly, oracle, model, cs)
            assert_mesh_matches(gm, gs, om)
    finally:
        gpu_poly.set_option(gpu.OPT_GRAPH, 0)


def test_c5_animation_frame(gpu_poly, oracle):
    """The 512^3, 64-primitive animated workload (C5), one frame against the oracle."""
    model, cs, _ = synth.make_config("C5", frame=7)
    gm, gs, om = run_both(gpu_poly, oracle, model, cs)
    assert len(gm.pos) > 1_000_000
    assert_mesh_matches(gm, gs, om)


def test_animation_driver(gpu_poly, oracle):
    from parsip_amd import animate

    seen = []
    anim = animate.Animation(gpu_poly, lambda f: synth.make_config("C2", frame=f)[0], synth.make_config("C2")[1])
    out = anim.run(3, sink=lambda f, mesh: seen.append((f, len(mesh.pos))), download=True)
    gpu_poly.set_option(gpu.OPT_GRAPH, 0)
    assert out["frames"] == 3 and [f for f, _ in seen] == [0, 1, 2]
    model, cs, _ = synth.make_config("C2", frame=2)
    om = oracle.polygonize(model, cs, threads=8)
    assert seen[2][1] == len(om.pos)


def test_tiered_kernels(oracle):
    """PSGPU_OPT_JIT 3: the structure kernels serve at once; once the model has stayed unchanged
    for OPT_TIER_RUNS runs the baked kernels take over (bit-exact); an animation frame (new
    parameters, same structure) is back on the structure kernels at its first run, without
    waiting for a compile; the same model again keeps the baked tier."""
    p = gpu.Polygonizer(0)
    try:
        p.set_option(gpu.OPT_JIT, gpu.JIT_TIERED)
        p.set_option(gpu.OPT_TIER_RUNS, 3)
        model, cs, _ = synth.make_config("C2")
        om = oracle.polygonize(model, cs, threads=8)
        p.set_model(model)
        assert p.jit_tier == 1
        for k in range(3):
            p.run(cs)
            assert_mesh_matches(p.download(), p.stats(), om)
        p.jit_wait()  # the third run started the baked compile
        assert p.jit_tier == 2
        p.run(cs)
        assert_mesh_matches(p.download(), p.stats(), om)
        p.set_model(model)  # the same bytes: nothing to recompile, the tier stays
        assert p.jit_tier == 2
        frame, cs1, _ = synth.make_config("C2", frame=3)
        p.set_model(frame, wait_jit=False)  # the structure kernels are loaded: no compile
        assert p.jit_tier == 1 and not p.jit_pending
        p.run(cs1)
        assert_mesh_matches(p.download(), p.stats(), oracle.polygonize(frame, cs1, threads=8))
    finally:
        p.close()
