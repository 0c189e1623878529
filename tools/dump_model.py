"""Write a config's model for tools/engine_threads: PsSoaBlobPrims, PsSoaPrimMatrices,
PsSoaBlobOps bytes, then the cell size (float32).  Usage: python tools/dump_model.py C3 out.bin"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import synth  # noqa: E402

model, cs, _ = synth.make_config(sys.argv[1])
with open(sys.argv[2], "wb") as f:
    f.write(model.prims.tobytes() + model.mats.tobytes() + model.ops.tobytes() + np.float32(cs).tobytes())
