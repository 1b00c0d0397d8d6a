"""CPU float32 emulation of the Winograd forms' rounding error (F(2x2), F(3x3) on two point sets,
F(4x4)) against a float64 conv, and the split of that error between the fp32 GEMM accumulation and
the fp32 transforms.  Study tool (round 6); numpy only.

    python tools/wino_error_emulation.py
"""
import numpy as np
from fractions import Fraction as F
rng=np.random.default_rng(0)
def f2():
    BT=np.array([[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]],float)
    G=np.array([[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]])
    AT=np.array([[1,1,1,0],[0,1,-1,-1]],float); return AT,G,BT,2
def f4():
    BT=np.array([[4,0,-5,0,1,0],[0,-4,-4,1,1,0],[0,4,-4,-1,1,0],[0,-2,-1,2,1,0],[0,2,-1,-2,1,0],[0,4,0,-5,0,1]],float)
    G=np.array([[1/4,0,0],[-1/6,-1/6,-1/6],[-1/6,1/6,-1/6],[1/24,1/12,1/6],[1/24,-1/12,1/6],[0,0,1]])
    AT=np.array([[1,1,1,1,1,0],[0,1,-1,2,-2,0],[0,1,1,4,4,0],[0,1,-1,8,-8,1]],float); return AT,G,BT,4
def f3a():  # points 0,1,-1,2
    AT=np.array([[1,1,1,1,0],[0,1,-1,2,0],[0,1,1,4,1]],float)
    G=np.array([[1/2,0,0],[1/2,1/2,1/2],[1/6,-1/6,1/6],[1/6,1/3,2/3],[0,0,1]])
    BT=np.array([[2,-1,-2,1,0],[0,2,1,-1,0],[0,-2,3,-1,0],[0,-1,0,1,0],[0,2,-1,-2,1]],float); return AT,G,BT,3
def f3b():  # points 0,1,-1,1/2
    AT=np.array([[1,1,1,1,0],[0,1,-1,.5,0],[0,1,1,.25,1]],float)
    G=np.array([[1,0,0],[1/2,1/2,1/2],[1/6,-1/6,1/6],[8/3,4/3,2/3],[0,0,1/2]])
    BT=np.array([[1,-2,-1,2,0],[0,-1,1,2,0],[0,-1,3,-2,0],[0,1,0,-1,0],[0,1,-2,-1,2]],float); return AT,G,BT,3
def conv_ref(x,w):  # x [H,W,Ci] (padded 1), w [Co,3,3,Ci] -> [H,W,Co], float64
    H,W,Ci=x.shape; xp=np.pad(x,((1,1),(1,1),(0,0)))
    y=np.zeros((H,W,w.shape[0]))
    for ky in range(3):
        for kx in range(3):
            y+=xp[ky:ky+H,kx:kx+W,:]@w[:,ky,kx,:].T
    return y
def conv_fp32(x,w):
    H,W,Ci=x.shape; xp=np.pad(x,((1,1),(1,1),(0,0))).astype(np.float32)
    y=np.zeros((H,W,w.shape[0]),np.float32)
    for ky in range(3):
        for kx in range(3):
            y+=(xp[ky:ky+H,kx:kx+W,:]@w[:,ky,kx,:].T.astype(np.float32)).astype(np.float32)
    return y
def wino(x,w,mat):
    AT,G,BT,m=mat; n=m+2
    H,W,Ci=x.shape; Co=w.shape[0]
    TY=-(-H//m); TX=-(-W//m)
    xp=np.zeros((TY*m+2,TX*m+2,Ci),np.float32); xp[1:H+1,1:W+1]=x
    # U = G g G^T in double, rounded to fp32
    U=np.einsum('ik,ckld,jl->ijcd',G,w,G).astype(np.float32)   # [n,n,Co,Ci]
    # V = BT D B in fp32
    D=np.stack([np.stack([xp[m*ti:m*ti+n,m*tj:m*tj+n] for tj in range(TX)]) for ti in range(TY)]).astype(np.float32) # [TY,TX,n,n,Ci]
    BT32=BT.astype(np.float32)
    V=np.einsum('ik,abklc->abilc',BT32,D).astype(np.float32)
    V=np.einsum('abilc,jl->abijc',V,BT32).astype(np.float32)
    M=np.einsum('abijc,ijoc->abijo',V,U).astype(np.float32)  # fp32 GEMM
    AT32=AT.astype(np.float32)
    Y=np.einsum('pi,abijo->abpjo',AT32,M).astype(np.float32)
    Y=np.einsum('abpjo,qj->abpqo',Y,AT32).astype(np.float32)
    Y=Y.transpose(0,2,1,3,4).reshape(TY*m,TX*m,Co)[:H,:W]
    return Y
H=W=24; Ci=256; Co=64
x=np.maximum(rng.standard_normal((H,W,Ci)),0).astype(np.float32)
w=(rng.standard_normal((Co,3,3,Ci))*np.sqrt(2/(9*Ci))).astype(np.float32)
ref=conv_ref(x.astype(np.float64),w.astype(np.float64))
mx=np.abs(ref).max()
print('fp32 direct', np.abs(conv_fp32(x,w)-ref).max()/mx)
for name,mat in (('F2',f2()),('F3a',f3a()),('F3b',f3b()),('F4',f4())):
    print(name, np.abs(wino(x,w,mat)-ref).max()/mx)
def wino_mixed(x,w,mat,gemm64=False,tr64=False):
    AT,G,BT,m=mat; n=m+2
    H,W,Ci=x.shape; Co=w.shape[0]
    TY=-(-H//m); TX=-(-W//m)
    dt_tr=np.float64 if tr64 else np.float32
    xp=np.zeros((TY*m+2,TX*m+2,Ci),np.float64); xp[1:H+1,1:W+1]=x
    U=np.einsum('ik,ckld,jl->ijcd',G,w.astype(np.float64),G).astype(np.float32).astype(np.float64 if gemm64 else np.float32)
    D=np.stack([np.stack([xp[m*ti:m*ti+n,m*tj:m*tj+n] for tj in range(TX)]) for ti in range(TY)]).astype(dt_tr)
    V=np.einsum('ik,abklc->abilc',BT.astype(dt_tr),D).astype(dt_tr)
    V=np.einsum('abilc,jl->abijc',V,BT.astype(dt_tr)).astype(dt_tr)
    if gemm64: M=np.einsum('abijc,ijoc->abijo',V.astype(np.float32).astype(np.float64),U)
    else: M=np.einsum('abijc,ijoc->abijo',V.astype(np.float32),U.astype(np.float32)).astype(np.float32)
    M=M.astype(dt_tr)
    Y=np.einsum('pi,abijo->abpjo',AT.astype(dt_tr),M).astype(dt_tr)
    Y=np.einsum('abpjo,qj->abpqo',Y,AT.astype(dt_tr)).astype(dt_tr)
    return Y.transpose(0,2,1,3,4).reshape(TY*m,TX*m,Co)[:H,:W]
for name,mat in (('F2',f2()),('F3a',f3a()),('F3b',f3b()),('F4',f4())):
    e1=np.abs(wino_mixed(x,w,mat,gemm64=True)-ref).max()/mx
    e2=np.abs(wino_mixed(x,w,mat,tr64=True)-ref).max()/mx
    print(name,'gemm exact, fp32 transforms',e1,' fp32 gemm, exact transforms',e2)
