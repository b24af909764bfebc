"""Candidates per row of k_neigh3's trimmed bin-rows against bin sizes (x and y/z separately),
on a jittered sc lattice with spacing 1 and cutoff 3 (C5's h = 3 dx, skin 0): the per-row
candidate count and the number of bin-rows looked up.  A sizing model for the list builders'
bins (profiles/r06/qbx/README.md); CPU only.  usage: python tools/bin_candidates.py"""
import numpy as np
rng=np.random.default_rng(1)
cut=3.0
L=40
g=np.arange(L)+0.5
X=np.stack(np.meshgrid(g,g,g,indexing='ij'),-1).reshape(-1,3)+rng.normal(0,0.01,(L**3,3))
def count(bx,byz,R):
    nbx=int(L/bx); bx=L/nbx; nb=int(L/byz); byz=L/nb
    cx=np.floor(X[:,0]/bx).astype(int); cy=np.floor(X[:,1]/byz).astype(int); cz=np.floor(X[:,2]/byz).astype(int)
    cnt=np.zeros((nb,nb,nbx),int); np.add.at(cnt,(cz,cy,cx),1)
    tot=0;N=300;rows=0
    idx=rng.choice(np.where(np.all((X>10)&(X<L-10),1))[0],N)
    for i in idx:
        xi=X[i]; c=(int(xi[0]/bx),int(xi[1]/byz),int(xi[2]/byz))
        for dz in range(-R,R+1):
            for dy in range(-R,R+1):
                bz,by=c[2]+dz,c[1]+dy
                def gap(v,bb,cc):
                    if bb==cc: return 0.0
                    edge=(bb+1)*byz if bb<cc else bb*byz
                    return max((v-edge) if bb<cc else (edge-v),0)
                gz=gap(xi[2],bz,c[2]); gy=gap(xi[1],by,c[1])
                d2=gy*gy+gz*gz
                if d2>cut*cut: continue
                rows+=1
                ext=np.sqrt(cut*cut-d2)
                bx0=int(np.floor((xi[0]-ext)/bx)); bx1=int(np.floor((xi[0]+ext)/bx))
                tot+=cnt[bz,by,bx0:bx1+1].sum()
    return tot/N, rows/N
for bx,byz,R in ((1.5,1.5,2),(0.5,1.5,2),(0.75,1.5,2),(0.5,1.0,3),(1.0,1.0,3)):
    print(bx,byz,R,count(bx,byz,R))
