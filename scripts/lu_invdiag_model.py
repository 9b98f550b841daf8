"""Numpy model behind bo_lu.hip's solve: the residual |A X - I| of inv(A) from LU with partial pivoting,
with the 16 x 16 diagonal blocks applied by substitution (getrs) or as explicit inverses (rocBLAS
trsm's method, the device solve), against LAPACK's gesv, on C3-like kernel matrices at fitted and
bench length scales (cond 1e4 .. 2e19)."""
import numpy as np, scipy.linalg as sl
rng=np.random.default_rng(0)
def make(n, ls, pv, seed):
    r=np.random.default_rng(seed)
    side=1024
    lin=r.choice(side*side, size=n, replace=False)
    x=np.stack([lin//side, lin%side],1).astype(float)
    d=((x[:,None,:]-x[None,:,:])**2).sum(-1)
    return pv*np.exp(-0.5*d/ls**2)+1e-6*np.eye(n)
def blocked_inv(A, nb=16, inv_diag=True):
    n=A.shape[0]
    lu,piv=sl.lu_factor(A)
    L=np.tril(lu,-1)+np.eye(n); U=np.triu(lu)
    P=np.eye(n)
    perm=np.arange(n)
    for i,p in enumerate(piv): perm[[i,p]]=perm[[p,i]]
    W=np.eye(n)[perm]   # P I
    # forward
    for s in range(0,n,nb):
        e=min(n,s+nb)
        Lss=L[s:e,s:e]
        if inv_diag: W[s:e]=np.linalg.inv(Lss)@W[s:e]  # inv via LAPACK (substitution on identity)
        else: W[s:e]=sl.solve_triangular(Lss,W[s:e],lower=True,unit_diagonal=True)
        W[e:]-=L[e:,s:e]@W[s:e]
    for s in reversed(range(0,n,nb)):
        e=min(n,s+nb)
        Uss=U[s:e,s:e]
        if inv_diag: W[s:e]=sl.solve_triangular(Uss,np.eye(e-s),lower=False)@W[s:e]
        else: W[s:e]=sl.solve_triangular(Uss,W[s:e],lower=False)
        W[:s]-=U[:s,s:e]@W[s:e]
    return W
for n,ls,pv in ((512,680.,2e9),(512,25.,3e3),(512,400.,2e9),(300,400.,2e9)):
    A=make(n,ls,pv,n)
    ref=np.linalg.inv(A)
    rr=np.abs(A@ref-np.eye(n)).max()
    r1=np.abs(A@blocked_inv(A,inv_diag=False)-np.eye(n)).max()
    r2=np.abs(A@blocked_inv(A,inv_diag=True)-np.eye(n)).max()
    print(f"n={n} ls={ls} cond={np.linalg.cond(A):.1e} gesv {rr:.2e} subst {r1:.2e} invdiag {r2:.2e} ratio {r2/rr:.1f}")
