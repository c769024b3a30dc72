"""Neighbour tests per ROR candidate: the tile pass's order (bins counting-sorted, the candidate's own bin row
then the rows above and below, 4-record batches, stop at need = 3) against bins sorted by z with a |dz| <= r window per
bin (nine ranges), on 20 000 random clip-box candidates of the C2 cloud. usage: python tools/ror_tests_sim.py"""
import sys, numpy as np
import os; sys.path[:0]=[os.path.dirname(os.path.abspath(__file__))]
import orchard
cfg=orchard.CONFIGS['C2']
xyz=orchard.xyz(orchard.generate(cfg)).astype(np.float32)
poly=orchard.polygon(cfg)
r=0.2; r2=np.float32(r*r); cs=r*1.001
bx0,bx1=poly[:,0].min()-r,poly[:,0].max()+r; by0,by1=poly[:,1].min()-r,poly[:,1].max()+r
m=(xyz[:,2]>=-0.6)&(xyz[:,2]<=0.7)&(xyz[:,0]>=bx0)&(xyz[:,0]<=bx1)&(xyz[:,1]>=by0)&(xyz[:,1]<=by1)
P=xyz[m]
bx=((P[:,0]-bx0)/cs).astype(np.int64); by=((P[:,1]-by0)/cs).astype(np.int64)
nbx=bx.max()+1
key=by*nbx+bx
order=np.argsort(key,kind='stable')
P=P[order]; key=key[order]; bx=bx[order]; by=by[order]
starts=np.searchsorted(key, np.arange(key.max()+nbx*2+8))
cand=np.where((P[:,2]>=-0.4)&(P[:,2]<=0.5)&(P[:,0]>=bx0+r)&(P[:,0]<=bx1-r)&(P[:,1]>=by0+r)&(P[:,1]<=by1-r))[0]
rng=np.random.default_rng(1); samp=rng.choice(cand, 20000, replace=False)
need=3
def tests_current(i):
    p=P[i]; cnt=0; t=0
    for dy in (0,-1,1):
        b=(by[i]+dy)*nbx+bx[i]-1
        lo,hi=starts[b],starts[b+3]
        k=lo
        while k<hi and cnt<need:
            q=P[k:min(k+4,hi)]
            d=q-p; d2=(d[:,0]*d[:,0]+d[:,1]*d[:,1])+d[:,2]*d[:,2]
            cnt+=int((d2<=r2).sum()); t+=4; k+=4
        if cnt>=need: break
    return t, cnt>=need
# z-sorted bins: within each bin sort by z; scan own bin row's 3 bins' z-windows then others
Pz=P.copy()
zs=np.empty(len(P),np.float32)
for b in range(len(starts)-1):
    pass
def tests_z(i, Zsorted_bins):
    p=P[i]; cnt=0; t=0
    for dy in (0,-1,1):
        for dx in (0,-1,1):
            b=(by[i]+dy)*nbx+bx[i]+dx
            lo,hi=starts[b],starts[b+1]
            if hi<=lo: continue
            zz=Zsorted_bins[lo:hi,2]
            a=lo+np.searchsorted(zz, p[2]-r, 'left'); e=lo+np.searchsorted(zz, p[2]+r, 'right')
            k=a
            while k<e and cnt<need:
                q=Zsorted_bins[k:min(k+4,e)]
                d=q-p; d2=(d[:,0]*d[:,0]+d[:,1]*d[:,1])+d[:,2]*d[:,2]
                cnt+=int((d2<=r2).sum()); t+=4; k+=4
            if cnt>=need: break
        if cnt>=need: break
    return t, cnt>=need
# build z-sorted copy: sort by (key, z)
o2=np.lexsort((P[:,2], key)); Zs=P[o2]
# map sample indices: positions differ; use point values (find each sample's point in Zs is not needed: p is the value)
tc=[tests_current(i) for i in samp]
tz=[tests_z(i, Zs) for i in samp]
print("current: mean tests %.1f, kept %.3f" % (np.mean([a for a,_ in tc]), np.mean([b for _,b in tc])))
print("z-window: mean tests %.1f, kept %.3f" % (np.mean([a for a,_ in tz]), np.mean([b for _,b in tz])))
print("points per bin (nonempty) %.1f" % np.mean(np.diff(starts)[np.diff(starts)>0]))
