"""Host emulation of the split sweep's error sources on the lpsc.yaml box (N = 16384,
k-d or caller order): f32 vs f64 accumulation inside a k-tile and across tiles, A
rounded to f32, f32 strtrs.  CPU only (numpy/scipy, ~2 min, ~12 GB):
    python tools/r3_emulate_accumulation.py 16384 kd"""
import numpy as np, time, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import oracle as O
from safe_bayesian_optimization_amd.terrain import synthetic_box
import scipy.linalg as sla
from scipy.linalg import lapack
n=int(sys.argv[1]); order=sys.argv[2]
wl=synthetic_box(n,1000,1000,seed=0)
h=wl.hyper
x=wl.x.astype(np.float32); y=wl.y.astype(np.float32)
def kd(p, off):
    if off+len(p)<=64: return sorted(p)
    xs=x[p]; ys=y[p]
    c = x if (xs.max()-xs.min())>=(ys.max()-ys.min()) else y
    cnt=len(p); left=(off+cnt//2+32)//64*64-off; left=min(max(left,64-off),cnt-1)
    ps=sorted(p,key=lambda i:(c[i],i))
    return kd(ps[:left],off)+kd(ps[left:],(off+left)%64)
if order=="kd":
    sys.setrecursionlimit(10000)
    perm=np.array(kd(list(range(n)),0))
    x=x[perm]; y=y[perm]
K=O.rbf_fill_f32(x,y,h.length_scale,h.sf2,h.sn2).reshape(n,n)
L,info=lapack.spotrf(K,lower=1); assert info==0
L=np.tril(L); del K
L64=L.astype(np.float64)
Li=sla.solve_triangular(L64,np.eye(n),lower=True)
A32=(h.sf2*Li).astype(np.float32); A64=A32.astype(np.float64)
del Li
rng=np.random.default_rng(7)
sel=rng.choice(wl.qx.size,512,replace=False)
qx=wl.qx[sel].astype(np.float32); qy=wl.qy[sel].astype(np.float32)
X=x.astype(np.float64)[:,None]; Y=y.astype(np.float64)[:,None]
E=np.exp(-((X-qx.astype(np.float64)[None])**2+(Y-qy.astype(np.float64)[None])**2)/(2*h.length_scale**2))
Vt=sla.solve_triangular(L64,h.sf2*E,lower=True)
var_t=h.sf2-(Vt*Vt).sum(0)
def rep(name,V):
    var=h.sf2-(np.asarray(V,np.float64)**2).sum(0)
    print(f"{order} {name:44s} nrel {np.abs(var-var_t).max()/np.abs(var_t).max():.3e}",flush=True)
Ef=E.astype(np.float32)
rep("A f32 exact arith", A64@Ef.astype(np.float64))
acc32=np.zeros((n,512),np.float32); acc64=np.zeros((n,512))
for k0 in range(0,n,64):
    p=(A32[:,k0:k0+64]@Ef[k0:k0+64])
    acc32+=p; acc64+=p.astype(np.float64)
rep("f32 tile + f32 outer", acc32)
rep("f32 tile + f64 outer", acc64)
acc32=np.zeros((n,512),np.float32)
for k0 in range(0,n,64):
    acc32+=(A64[:,k0:k0+64]@Ef[k0:k0+64].astype(np.float64)).astype(np.float32)
rep("f64 tile + f32 outer", acc32)
V=sla.solve_triangular(L,(h.sf2*E).astype(np.float32),lower=True)
rep("strtrs f32", V)
