"""Offline estimate (oracle only, no GPU): how many of C3's S1 bricks (2x2x2 MPUs, one k_precheck
wave) hold only survivors whose 8 MPU corners straddle the iso value 0.5 -- MPUs a conservative
field bound can never prove empty, so the bound walk is wasted on them.
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ('oracle', 'tests', '')]
import psoracle, numpy as np
from parsip_amd import synth, soa
m,cs,n=synth.make_config('C3')
om=psoracle.polygonize(m,cs,threads=8)
st=om.stats
org=soa.mpu_origins(cs,*m.bbox).astype(np.float32)
side=np.float32(cs)*np.float32(7)
pts=[]
for c in range(8):
    X,Y,Z=c&1,(c>>1)&1,c>>2
    pts.append(org+np.array([X,Y,Z],np.float32)*side)
P=np.stack(pts,1).reshape(-1,3)
f=psoracle.field_value(m,P[:,0],P[:,1],P[:,2]).reshape(-1,8)
passed=st[:,0]>0
straddle=(f>=0.5).any(1)&(f<0.5).any(1)
surface=st[:,2]>0
print('passed',passed.sum(),'straddle',straddle.sum(),'straddle&passed',(straddle&passed).sum(),'surface',surface.sum(),'straddle&~surface',(straddle&~surface).sum())
idx=np.arange(len(st)); i=idx//(37*37); j=(idx//37)%37; k=idx%37
brick=(i//2)*19*19+(j//2)*19+(k//2)
allstr=0; withsurv=0
for b in np.unique(brick):
    sel=brick==b
    sv=passed[sel]
    if sv.any():
        withsurv+=1
        if straddle[sel][sv].all(): allstr+=1
print('bricks with survivors',withsurv,'all survivors straddle',allstr)
