"""Comparison helpers shared by the parity tests (GPU path vs the CPU oracle)."""
import numpy as np


def bits_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise bit equality of fp32 arrays; any NaN equals any NaN (x86 and CDNA
    produce different default-NaN payloads)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def assert_bits_equal(a, b, what: str):
    eq = bits_equal(a, b)
    if not eq.all():
        bad = np.argwhere(~eq)
        i = tuple(bad[0])
        raise AssertionError(f"{what}: {len(bad)} of {eq.size} differ; first at {i}: gpu {a[i]!r} oracle {b[i]!r}")


def assert_mesh_matches(gmesh, gstats, omesh, normals_atol: float | None = None, colours: bool = True):
    """GPU compact mesh + per-MPU stats vs the oracle's per-MPU output (same MPU range)."""
    ost = omesh.stats
    assert len(gstats) == len(ost), "MPU count"
    np.testing.assert_array_equal(gstats["passedPrecheck"], ost[:, 0], err_msg="S1 precheck decisions")
    np.testing.assert_array_equal(gstats["ctFieldEvals"], ost[:, 1], err_msg="ctFieldEvals")
    np.testing.assert_array_equal(gstats["ctVertices"], ost[:, 2], err_msg="per-MPU vertex counts")
    np.testing.assert_array_equal(gstats["ctTriangles"], ost[:, 3], err_msg="per-MPU triangle counts")
    np.testing.assert_array_equal(gmesh.vertex_offsets, omesh.vertex_offsets, err_msg="per-MPU vertex offsets")
    np.testing.assert_array_equal(gmesh.triangle_offsets, omesh.triangle_offsets, err_msg="per-MPU triangle offsets")
    assert gmesh.pos.shape == omesh.pos.shape
    assert gmesh.tris.shape == omesh.tris.shape
    np.testing.assert_array_equal(gmesh.local_tris(), omesh.tris, err_msg="triangles (MPU-local ids)")
    assert_bits_equal(gmesh.pos, omesh.pos, "vertex positions")
    if normals_atol is None:
        assert_bits_equal(gmesh.nrm, omesh.nrm, "normals")
    else:
        ok = np.isclose(gmesh.nrm, omesh.nrm, atol=normals_atol, rtol=0) | (np.isnan(gmesh.nrm) & np.isnan(omesh.nrm))
        assert ok.all(), f"normals beyond {normals_atol}: {np.count_nonzero(~ok)}"
    if colours:
        assert_bits_equal(gmesh.col, omesh.col, "vertex colours")


def _canon(a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a, np.float32).copy()
    a[np.isnan(a)] = np.float32(np.nan)
    return a.view(np.uint32).astype("<u4").tobytes()


def mesh_digests(stats4, pos, nrm, col, tris_local) -> dict:
    """SHA-256 digests of a mesh in MPU order; stats4 = (passed, evals, V, T) per MPU."""
    import hashlib

    h = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    st = np.ascontiguousarray(stats4, np.uint32)
    return {"vertices": int(len(pos)), "triangles": int(len(tris_local)),
            "passed_s1": int(np.count_nonzero(st[:, 0])),
            "stats_sha256": h(st.astype("<u4").tobytes()),
            "pos_sha256": h(_canon(pos)), "nrm_sha256": h(_canon(nrm)), "col_sha256": h(_canon(col)),
            "tris_sha256": h(np.ascontiguousarray(tris_local, np.uint16).astype("<u2").tobytes())}
