"""Register, LDS and scratch use of every generated (hiprtc) kernel, and the occupancy they
allow on gfx950 -- no GPU needed: the code objects are compiled host-only
(psgpu_jit_compile) and their AMDGPU metadata read with llvm-readelf.

Occupancy rules (MI355X_MICROARCH.md "Register files", "Residency"): 256-thread blocks (one
wave per SIMD each); waves/SIMD by VGPRs = min(8, 512 // alloc), alloc = VGPR + AGPR rounded
up to 8; blocks/CU by SGPRs = min(8, 800 // (ceil(sgpr / 16) * 16 + 16)); blocks/CU by LDS =
163840 // (static + dynamic LDS); at most 8 blocks (32 waves) per CU.  k_mpu's dynamic LDS is
the host's mpu_lds_bytes(0) = 4 MPUs x 4,864 B (psgpu_device.h kLdsMpu), half that for the
tree-split k_mpu (2 MPUs per block); the others take none.

Static instruction mix per kernel from llvm-objdump (VALU = v_* except v_readlane /
v_readfirstlane / v_writelane counted as VALU too; s_nop; s_waitcnt; packed fp32).

Usage: python tools/kernel_resources.py [--configs C3,C5] [--out profiles/r05_kernel_resources.json]
       [--variant name=ENV=VALUE[;ENV=VALUE]] ...
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LLVM = "/opt/rocm/lib/llvm/bin"
K_LDS_MPU = 4864            # psgpu_device.h kLdsMpu (6400 with PSGPU_MPU_MAPS 1)
MPU_DYNAMIC_LDS = 4 * K_LDS_MPU  # mpu_lds_bytes(0), kMpusPerBlock = 4 (PSGPU_MPU_WAVES 1)
MPU_S_DYNAMIC_LDS = 2 * K_LDS_MPU  # the tree-split k_mpu: 2 MPUs per block
ROLE = {"jit_precheck": "k_precheck", "jit_mpu": "k_mpu", "jit_vertex": "k_vertex (quad, 16/wave)",
        "jit_vertex_w": "k_vertex (wide, 64/wave)", "jit_finish": "k_finish (64/wave)",
        "jit_finish_q": "k_finish (quad, 16/wave)", "jit_finish_p": "k_finish (pair, 32/wave)",
        "jit_precheck_s": "k_precheck (tree split)", "jit_mpu_s": "k_mpu (tree split)",
        "jit_surface": "k_vertex + k_finish in one launch (small launches, quad layouts)", "jit_probe": "probe"}


def parse_metadata(co: str) -> dict:
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    out = {}
    for block in re.split(r"\n  - \.agpr_count:", txt)[1:]:
        block = ".agpr_count:" + block

        def field(name, cast=int):
            m = re.search(r"\n?\s*\." + re.escape(name) + r":\s+(\S+)", block)
            return cast(m.group(1)) if m else None
        name = field("name", str)
        out[name] = {"vgpr": field("vgpr_count"), "agpr": field("agpr_count"), "sgpr": field("sgpr_count"),
                     "lds_static": field("group_segment_fixed_size"),
                     "scratch": field("private_segment_fixed_size"),
                     "vgpr_spill": field("vgpr_spill_count"), "sgpr_spill": field("sgpr_spill_count")}
    return out


def instruction_mix(co: str) -> dict:
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                         check=True).stdout
    mix, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\w+)>:", line)
        if m:
            cur = m.group(1)
            mix[cur] = {"instructions": 0, "valu": 0, "s_nop": 0, "s_waitcnt": 0, "v_pk_fp32": 0, "dpp": 0,
                        "code_bytes": 0, "load_x2_sc1": 0, "load_sc1": 0, "store_sc1": 0}
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+(\w+)", line)
        if not m or "//" not in line:
            continue
        op = m.group(1)
        d = mix[cur]
        d["instructions"] += 1
        words = re.search(r"//\s*([0-9A-F]+):((?:\s[0-9A-F]{8})+)", line)
        if words:
            d["code_bytes"] += 4 * len(words.group(2).split())
        if op.startswith("v_"):
            d["valu"] += 1
            if op.startswith(("v_pk_add_f32", "v_pk_mul_f32", "v_pk_fma_f32", "v_pk_mov_b32")):
                d["v_pk_fp32"] += 1
            if "_dpp" in op or "row_" in line or "quad_perm" in line:
                d["dpp"] += 1
        elif op.startswith("global_load") and re.search(r"\bsc1\b", line.split("//")[0]):
            # agent-scope loads: the offsets-scan look-back and k_surface's offsets reads
            # (surface_offs), k_front's entries, masks and ready words -- they must bypass the
            # non-coherent caches
            d["load_sc1"] += 1
            if op == "global_load_dwordx2":
                d["load_x2_sc1"] += 1
        elif op.startswith("global_store") and re.search(r"\bsc1\b", line.split("//")[0]):
            d["store_sc1"] += 1  # write-through stores: k_front's published entries, masks, ready words
        elif op == "s_nop":
            d["s_nop"] += 1
        elif op == "s_waitcnt":
            d["s_waitcnt"] += 1
    return mix


def occupancy(r: dict, dynamic_lds: int) -> dict:
    alloc = -(-(r["vgpr"] + (r["agpr"] or 0)) // 8) * 8
    by_vgpr = min(8, 512 // alloc)
    by_sgpr = min(8, 800 // (-(-r["sgpr"] // 16) * 16 + 16))
    lds = (r["lds_static"] or 0) + dynamic_lds
    by_lds = min(8, 163840 // lds) if lds else 8
    blocks = min(8, by_vgpr, by_sgpr, by_lds)
    limiter = min((("vgpr", by_vgpr), ("sgpr", by_sgpr), ("lds", by_lds), ("waves/CU cap", 8)), key=lambda t: t[1])[0]
    return {"vgpr_alloc": alloc, "lds_per_block": lds, "blocks_per_cu_by_vgpr": by_vgpr,
            "blocks_per_cu_by_sgpr": by_sgpr, "blocks_per_cu_by_lds": by_lds, "waves_per_simd": blocks,
            "limited_by": limiter}


def compile_variant(config: str, mode: int, env: dict) -> dict:
    from parsip_amd import gpu, synth
    model = synth.make_config(config)[0]
    saved = {k: os.environ.get(k) for k in env}
    with tempfile.TemporaryDirectory() as d:
        os.environ["PSGPU_JIT_CACHE"] = d
        os.environ.update(env)
        try:
            gpu.jit_compile(model, mode)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        cos = [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".co")]
        assert len(cos) == 1, cos
        meta = parse_metadata(cos[0])
        mix = instruction_mix(cos[0])
    out = {}
    for name, r in sorted(meta.items()):
        out[name] = {"role": ROLE.get(name, name), **r,
                     **occupancy(r, MPU_DYNAMIC_LDS if name == "jit_mpu" else MPU_S_DYNAMIC_LDS if name == "jit_mpu_s" else 0),
                     **mix.get(name, {})}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C5")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_kernel_resources.json"))
    ap.add_argument("--variant", action="append", default=[],
                    help="name=ENV=VALUE[;ENV=VALUE]: an extra structure-tier compile with that environment")
    a = ap.parse_args()
    res = {"generator": "tools/kernel_resources.py (host-only hiprtc compile, llvm-readelf / llvm-objdump)",
           "rules": __doc__.split("Usage:")[0].strip()}
    variants = [("structure", 1 | 4, {}), ("baked", 2, {})]
    for v in a.variant:
        name, _, rest = v.partition("=")
        env = dict(kv.split("=", 1) for kv in rest.split(";") if kv)
        variants.append((name, 1, env))
    for cfg in a.configs.split(","):
        res[cfg] = {}
        for name, mode, env in variants:
            res[cfg][name] = {"mode": mode, "env": env, "kernels": compile_variant(cfg, mode, env)}
            for k, r in res[cfg][name]["kernels"].items():
                print(f"{cfg:3s} {name:12s} {k:15s} vgpr {r['vgpr']:3d} sgpr {r['sgpr']:3d} lds {r['lds_per_block']:6d} "
                      f"scratch {r['scratch']:4d} -> {r['waves_per_simd']} waves/SIMD ({r['limited_by']}); "
                      f"VALU {r.get('valu', 0):6d} s_nop {r.get('s_nop', 0):5d} waitcnt {r.get('s_waitcnt', 0):5d} "
                      f"code {r.get('code_bytes', 0)} B", flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
