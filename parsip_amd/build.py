"""Build the gfx950 shared library in-tree (parsip_amd/libparsip_gpu.so).

hipcc cross-compiles for gfx950 without a GPU.  Parity-critical flags:
``-ffp-contract=off`` (no FMA contraction: the reference's SSE code has none) and no
fast-math, so fp32 division and sqrt stay correctly rounded and denormals IEEE.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libparsip_gpu.so")
SOURCES = ["psgpu_kernels.hip", "psgpu_host.cpp"]
HEADERS = ["psgpu_model.h", "psgpu_launch.h", os.path.join("..", "..", "include", "parsip_gpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PSGPU_ARCH", "gfx950")
FLAGS = ["-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-std=c++17", "-Wall",
         f"--offload-arch={ARCH}"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [HIPCC, *FLAGS, *[os.path.join(CSRC, s) for s in SOURCES], "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
