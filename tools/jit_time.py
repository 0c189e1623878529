"""Time the hiprtc specialisation of one model's tree kernels (no GPU needed).
Usage: python tools/jit_time.py C3|C5|scene [mode]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PSGPU_JIT_CACHE", "/tmp/psgpu_jit_time_%d" % time.time_ns())

from parsip_amd import blobtree, gpu, scene, synth  # noqa: E402

name = sys.argv[1]
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 1
if name == "scene":
    path = os.path.join(ROOT, "tests", "golden", "train_corrected.scene")
    code, model = blobtree.linearize_blobtree(blobtree.binarize(scene.load_scene(path)[0]))
else:
    model = synth.make_config(name)[0]
t = time.time()
n = gpu.jit_compile(model, mode)
print(f"{name} prims={model.ct_prims} ops={model.ct_ops} code={n} B compile={time.time() - t:.1f} s", flush=True)
