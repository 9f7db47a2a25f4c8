"""How much tighter the per-piece level bounds are than the |A|_F ones, on a C2-sized factor in
Hilbert order (numpy/torch, CPU): medians of old/new for the 0->1 and 1->2 increments.
  python tools/plane_norm_gain.py"""
import sys; sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import numpy as np
from safe_bayesian_optimization_amd import synthetic
import torch
def bf16(x):
    t=torch.from_numpy(np.ascontiguousarray(x,np.float32)).to(torch.bfloat16).to(torch.float32)
    return t.numpy()
def hilbert_d(n, x, y):
    d=np.zeros_like(x); s=n//2
    x=x.copy(); y=y.copy()
    while s>0:
        rx=((x & s)>0).astype(np.int64); ry=((y & s)>0).astype(np.int64)
        d+= s*s*((3*rx)^ry)
        # rotate
        m=(ry==0)
        flip=m&(rx==1)
        x[flip]=s-1-x[flip]; y[flip]=s-1-y[flip]
        tmp=x[m].copy(); x[m]=y[m]; y[m]=tmp
        s//=2
    return d
N=2048
wl=synthetic(N,8,seed=0)
side=wl.x.max()
xi=(wl.x/side*1023).astype(np.int64); yi=(wl.y/side*1023).astype(np.int64)
o=np.argsort(hilbert_d(1024,xi,yi),kind='stable')
x=wl.x[o]; y=wl.y[o]
d2=(x[:,None]-x[None,:])**2+(y[:,None]-y[None,:])**2
K=np.exp(-d2/(2*0.16))+0.1*np.eye(N)
L=np.linalg.cholesky(K)
A=np.linalg.inv(L).astype(np.float32)
A0=bf16(A); r1=A-A0; A1=bf16(r1); r2=r1-A1; A2=bf16(r2)
rat2=[];rat1=[];rat0=[]
for I in range(N//256):
    for t in range((I+1)*4):
        T=A[I*256:(I+1)*256, t*64:(t+1)*64]
        fro=np.linalg.norm(T)
        if fro==0: continue
        sp=np.linalg.norm(T,2)
        s1=np.linalg.norm(A1[I*256:(I+1)*256, t*64:(t+1)*64],2)
        s2=np.linalg.norm(A2[I*256:(I+1)*256, t*64:(t+1)*64],2)
        old0=3.1*2**-16*fro; new0=s2*1.002+2**-9*1.002*s1+2**-18*(sp+2**-9*fro)
        old1=2.03*2**-8*fro; new1=s1*1.002+2**-9*1.002*(sp+2**-9*fro)
        rat0.append(old0/new0); rat1.append(old1/new1); rat2.append(fro/sp)
for nm,r in (("inc0 old/new",rat0),("inc1 old/new",rat1),("fro/spec",rat2)):
    r=np.array(r); print(nm, "median %.1f  p10 %.1f p90 %.1f min %.1f"%(np.median(r),np.percentile(r,10),np.percentile(r,90),r.min()))
