import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import numpy as np
import psoracle
from parsip_amd import gpu, synth
from parity_util import bits_equal
model, cs, _ = synth.make_config('C3')
om = psoracle.polygonize(model, cs, threads=16)
p = gpu.Polygonizer(0)
for jit, cull in [(1, 1), (0, 1), (1, 0), (0, 0)]:
    p.set_option(gpu.OPT_JIT, jit); p.set_option(gpu.OPT_CULLING, cull); p.set_model(model)
    p.run(cs); gm = p.download()
    bad = np.flatnonzero(~bits_equal(gm.nrm, om.nrm).all(axis=1))
    print('jit', jit, 'cull', cull, 'bad vertices', bad[:10])
    for v in bad[:4]:
        q = om.pos[v]
        d = np.float32(0.001)
        pts = np.array([q, q + [d, 0, 0], q + [0, d, 0], q + [0, 0, d]], np.float32)
        rep = np.repeat(pts, 4, axis=0)
        of = psoracle.field_value(model, rep[:, 0], rep[:, 1], rep[:, 2])[::4]
        gf = p.field_values(rep, mode=0)[::4]
        g1 = p.field_values(pts, mode=1) if True else None
        print('  v', v, 'pos', q.tolist(), 'gpu n', gm.nrm[v].tolist(), 'orc n', om.nrm[v].tolist())
        print('    oracle f', of.tolist(), '\n    gpu quad f', gf.tolist(), '\n    gpu mode1 f', np.asarray(g1).tolist())
p.close()
