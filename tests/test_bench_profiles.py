"""bench.py's roofline reads the committed PMC / traffic summaries of the kernel tier it timed
(verdict r03: the baked tier's counters must never price a structure-tier step).  CPU only:
the selection logic over synthetic profile files."""
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def bench(tmp_path, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")  # bench sets it at import: restored after the test
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # no HIP call at import
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(mod, "ROOT", str(tmp_path))
    return mod


def _write(tmp_path, name, jit, instr):
    d = {"kernels": {"jit_mpu": {"SQ_INSTS_VALU": instr, "launches": 1}}}
    if jit is not None:
        d["jit"] = jit
    (tmp_path / "profiles" / name).write_text(json.dumps(d))


def test_profile_of_the_timed_tier(bench, tmp_path):
    _write(tmp_path, "r03_pmc.json", None, 1.0)       # before r04: no "jit", profiled with --jit 2
    _write(tmp_path, "r04_pmc.json", 2, 2.0)
    _write(tmp_path, "r04_pmc_structure.json", 1, 3.0)
    k, src = bench.committed_profile("pmc", 2)
    assert src.endswith("r04_pmc.json") and k["jit_mpu"]["SQ_INSTS_VALU"] == 2.0
    k, src = bench.committed_profile("pmc_structure", 1)
    assert src.endswith("r04_pmc_structure.json") and k["jit_mpu"]["SQ_INSTS_VALU"] == 3.0
    # a file whose recorded tier differs is never used for another tier
    assert bench.committed_profile("pmc", 1) == (None, None)
    assert bench.committed_profile("pmc_structure", 2) == (None, None)


def test_old_profiles_count_as_baked(bench, tmp_path):
    _write(tmp_path, "r03_pmc.json", None, 1.0)
    k, src = bench.committed_profile("pmc", 2)
    assert src.endswith("r03_pmc.json")
    assert bench.committed_profile("pmc", 1) == (None, None)


def test_profile_entry_names(bench):
    kernels = {"jit_mpu": {"a": 1}, "psgpu::k_mpu": {"a": 2}}
    assert bench.profile_entry(kernels, "k_mpu", 1) == {"a": 1}
    assert bench.profile_entry(kernels, "k_mpu", 0) == {"a": 2}
    assert bench.profile_entry(None, "k_mpu", 1) is None
