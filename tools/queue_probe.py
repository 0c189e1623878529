"""Which set-up detail makes E engines fast or slow (C3, full grid): an extra idle planning
context (EXTRA=1), a first sizing run per engine (PRERUN=1), torch.distributed gloo
initialised in the process (TORCH=1).  Prints ms/step for K queued steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gpu, synth  # noqa: E402

E = int(os.environ.get("ENGINES", "4"))
model, cs, N = synth.make_config("C3")
n = gpu.count_mpus(cs, *model.bbox)
ps = []
X = os.environ.get("EXTRA", "0")  # 1: a context before the engines, run once; 2: created only


def make_extra():
    extra = gpu.Polygonizer(0)
    if X in ("1", "3"):
        extra.set_model(model)
        extra.run(cs)
        extra.finish()
    return extra


if X in ("1", "2"):
    keep = make_extra()
if os.environ.get("TORCH", "0") == "1":
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("gloo", rank=0, world_size=1)
VB, FB = int(os.environ.get("VB", "0")), int(os.environ.get("FB", "0"))  # persistent grids (blocks per CU)
for _ in range(E):
    p = gpu.Polygonizer(0)
    if VB:
        p.set_option(gpu.OPT_VERTEX_BLOCKS_PER_CU, VB)
    if FB:
        p.set_option(gpu.OPT_FINISH_BLOCKS_PER_CU, FB)
    p.set_model(model)
    if os.environ.get("PRERUN", "0") == "1":
        p.run(cs, 0, n)
        p.finish()
    ps.append(p)
if X == "3":  # 3: created and run after the engines
    keep = make_extra()
for k in range(max(20, E)):
    ps[k % E].polygonize(cs, 0, n)
for p in ps:
    p.finish()
for rep in range(3):
    K = 400
    t0 = time.perf_counter()
    for k in range(K):
        ps[k % E].polygonize(cs, 0, n)
    for p in ps:
        p.finish()
    dt = (time.perf_counter() - t0) / K * 1e3
    print(f"E={E} EXTRA={os.environ.get('EXTRA', '0')} PRERUN={os.environ.get('PRERUN', '0')} "
          f"TORCH={os.environ.get('TORCH', '0')} q={os.environ.get('GPU_MAX_HW_QUEUES')} VB={VB} FB={FB}: {dt:.4f} ms/step", flush=True)
