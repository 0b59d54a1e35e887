"""Least-squares fit of the gemm_pipe cost model (csrc/kernels/bindings.cpp pipe_est_us) to bench_decode_gemm.py logs.

    python tools/fit_gemm_model.py   # reads profiles/r6/gemm_sweep_*_r6.log and fix_same_xcd_ab_*_r6.log

Prints the fitted constants, the worst residuals, and per (shape, rows) the model's pick against the measured best.
"""
import math
import re

import numpy as np
from scipy.optimize import least_squares
SH={"qkv":(6144,4096),"o":(4096,4096),"gate_up":(28672,4096),"down":(4096,14336)}
pts=[]
for f in ["profiles/r6/gemm_sweep_gate_up_r6.log","profiles/r6/gemm_sweep_qkv_r6.log","profiles/r6/gemm_sweep_o_down_r6.log","profiles/r6/fix_same_xcd_ab_gate_up_r6.log","profiles/r6/fix_same_xcd_ab_qkv_r6.log"]:
    for line in open(f):
        m=re.match(r"(\w+)\s+M=\s*(\d+)\s+(\S+)\s+([\d.]+) us/call.*\[impl 4 cfg (\d+) S (\d+)( fix)? est",line)
        if not m: continue
        sh,M,var,us,cfg,S,fix=m.groups()
        cfg=int(cfg)
        if cfg not in (8,9,10): continue
        op=var.split(":")[0]
        pts.append((sh,int(M),op,float(us),{8:256,9:192,10:128}[cfg],int(S),bool(fix)))
print(len(pts))
def model(p,sh,M,op,bm,S,fix):
    F,P,T0,a,W,R,Ts,Tn,Hn=p
    N,K=SH[sh]
    nbm=-(-M//bm); rows=min(bm,M); Kr=K/S
    wgs=nbm*(N//256)*S
    full=wgs//256; rem=wgs-256*full
    tw=T0+max((rows+256)*Kr*2/F, 2*bm*256*Kr/P)
    t=full*tw+(tw*(a+(1-a)*rem/256) if rem else 0)
    slot=bm*256*4
    if S>1:
        if fix: t+=slot/W+Ts+(S-1)*slot/R
        elif op=="split_norm": t+=slot/W+Tn+S*M*N*4/Hn
        else: t+=slot/W+Tn+(S*M*N*4+M*N*2)/Hn
    elif op=="split_norm": t+=Tn+M*N*10/Hn
    return t
def res(p):
    return [math.log(model(p,*x[:3],*x[4:]))-math.log(x[3]) for x in pts]
p0=[46e3,5.5e6,3,0.6,18e3,35e3,2,3,6e6]
lb=[10e3,1e6,0,0.2,5e3,5e3,0,0,1e6]; ub=[200e3,20e6,20,1,200e3,300e3,20,20,20e6]
r=least_squares(res,p0,bounds=(lb,ub))
print([round(v,3) for v in r.x])
e=np.array(res(r.x)); print("rms log err",np.sqrt((e**2).mean()), "max", np.abs(e).max())
for x,ei in sorted(zip(pts,e), key=lambda t:-abs(t[1]))[:12]:
    print(x, round(math.exp(ei),2))

# choices: model-best over pipe candidates vs measured-best among measured configs
p=r.x
def cands(sh,M,use):
    N,K=SH[sh]
    out=[]
    for bm in (256,192,128):
        for S in (1,2,4,8,16):
            if K%(128*S): break
            for fix in (False,True):
                if S==1 and fix: continue
                if S>1 and not fix and use=="plain":
                    op="out"   # slabs + reduce kernel
                else:
                    op="split_norm" if use=="slab" else "out"
                out.append(((bm,S,fix,op), model(p,sh,M,op,bm,S,fix)))
    return out
meas={}
for x in pts:
    key=(x[0],x[1]); meas.setdefault(key,[]).append((x[3],x[4],x[5],x[6],x[2]))
for (sh,M),v in sorted(meas.items()):
    use="slab" if sh in ("o","down") else "plain"
    c=min(cands(sh,M,use), key=lambda t:t[1])
    best=min(v)
    # measured time of the model's choice if measured
    mt=[t for t,bm,S,fix,op in v if (bm,S,fix)==c[0][:3]]
    print(f"{sh:8s} {M:5d} model pick {c[0]} est {c[1]:6.1f} | measured best {best[0]:6.1f} {best[1:]} | pick measured {mt[:1]}")
