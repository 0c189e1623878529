"""Debug helper: run the compat mode on the train scene and save the mesh (npz)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parsip_amd import gui, scene  # noqa: E402

cs = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
root = scene.load_scene(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                     "train_corrected.scene"))[0]
code, tree = gui.compact_blobtree(root)
p = gui.ParsipOptimized(0)
p.setup(tree, tree.root_octree, 0, cs, 0.5)
p.run()
m = p.exportMesh()
f, c = p.field_values(m.pos)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/gui_dump.npz", pos=m.pos, nrm=m.nrm, col=m.col, tris=m.tris, probe_f=f, probe_c=c)
print("saved", len(m.pos))
p.close()
