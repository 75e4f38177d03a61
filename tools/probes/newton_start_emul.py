import numpy as np, sys
sys.path.insert(0,'/root/repo')
from mujoco_playground_amd import _lib
from mujoco_playground_amd.model import blob as B
from oracle.oracle import Oracle, controller
blob=_lib.load_blob("flat"); h=B.unpack_header(blob)
floss_dof=np.array([h.dof_frictionloss[i] for i in range(h.nv)])
o=Oracle(blob)

def rows(dg):
    J=dg['efc_J']; ef=dg['efc']; t=ef[:,0].astype(int); R=ef[:,2]; aref=ef[:,3]; D=1/R
    fl=np.zeros(len(t))
    for r in np.nonzero(t==1)[0]: fl[r]=floss_dof[np.argmax(np.abs(J[r]))]
    return J,t,R,D,aref,fl

def state_eval(a,M,a0,J,t,R,D,aref,fl):
    x=J@a-aref
    f=np.zeros_like(x); q=np.zeros(len(x),bool)
    for r in range(len(x)):
        if t[r]==0: f[r]=-D[r]*x[r]; q[r]=True
        elif t[r]==1:
            th=R[r]*fl[r]
            if x[r]<=-th: f[r]=fl[r]
            elif x[r]>=th: f[r]=-fl[r]
            else: f[r]=-D[r]*x[r]; q[r]=True
        elif x[r]<0: f[r]=-D[r]*x[r]; q[r]=True
    grad=M@(a-a0)-J.T@f
    # region id per row for 'changed' check
    reg=np.where(t==1, np.sign(np.where(x<=-R*fl,-1,np.where(x>=R*fl,1,0))), (x<0).astype(int))
    return x,q,grad,reg

def line_search(a,p,M,a0,J,t,R,D,aref,fl):
    x0=J@a-aref; Jp=J@p; Mp=M@p; pMp=p@Mp; pg0=Mp@(a-a0)
    bps=[]
    for r in range(len(x0)):
        if Jp[r]==0: continue
        if t[r] in (2,3):
            al=-x0[r]/Jp[r]
            if al>0: bps.append(al)
        elif t[r]==1:
            th=R[r]*fl[r]
            for v in ((-th-x0[r])/Jp[r],(th-x0[r])/Jp[r]):
                if v>0: bps.append(v)
    bps=sorted(bps); lo=0.0
    for k in range(len(bps)+1):
        hi=bps[k] if k<len(bps) else 1e300
        if hi<=lo: continue
        mid=0.5*(lo+hi) if k<len(bps) else lo+1.0
        g=0.0; hh=0.0
        for r in range(len(x0)):
            x=x0[r]+mid*Jp[r]; gg=0; h2=0
            if t[r]==0: gg=D[r]*x*Jp[r]; h2=D[r]*Jp[r]**2
            elif t[r]==1:
                th=R[r]*fl[r]
                if x<=-th: gg=-fl[r]*Jp[r]
                elif x>=th: gg=fl[r]*Jp[r]
                else: gg=D[r]*x*Jp[r]; h2=D[r]*Jp[r]**2
            elif x<0: gg=D[r]*x*Jp[r]; h2=D[r]*Jp[r]**2
            hh+=h2; g+=gg-h2*mid
        c1=pMp+hh; c0=pg0+g
        root=-c0/c1 if c1>0 else (1e300 if c0<0 else lo)
        if root<=lo: return lo
        if root<hi: return root
        lo=hi
    return lo

def newton(a,M,a0,rowsd,predict_mask=None,maxit=30):
    J,t,R,D,aref,fl=rowsd
    for it in range(maxit):
        x,q,grad,reg=state_eval(a,M,a0,*rowsd)
        qq=q if (it>0 or predict_mask is None) else predict_mask
        H=M+(J[qq].T*D[qq])@J[qq]
        p=-np.linalg.solve(H,grad)
        al=line_search(a,p,M,a0,*rowsd)
        an=a+al*p
        _,qn,_,regn=state_eval(an,M,a0,*rowsd)
        full=abs(al-1.0)<1e-9
        same=np.array_equal(regn,reg) if (it>0 or predict_mask is None) else np.array_equal(qn,predict_mask)
        a=an
        if (full and same) or np.abs(al*p).max()<=2e-6*max(np.abs(a).max(),1): return it+1,a
    return maxit,a

n=512
st=np.zeros((n,44)); o.reset(st,seed=3)
rng=np.random.default_rng(3)
A_its=[];B_its=[];C_its=[]
acts=[rng.uniform(-1,1,(n,2)).astype(np.float32) for _ in range(240)]
for k in range(200): o.step(st,acts[k],flags=3,seed=3)
for k in range(200,220):
    for e in range(n):
        s=st[e]; ctrl=controller(acts[k][e],1.0,1.0)
        dg=o.diag(s,ctrl,flags=1)
        if dg['nefc']==0: A_its.append(0);B_its.append(0);C_its.append(0);continue
        M=dg['qM']; a0=dg['qacc_smooth']; rd=rows(dg)
        ia,aa=newton(a0.copy(),M,a0,rd)
        warm=s[25:37]
        _,qw,_,_=state_eval(warm,M,a0,*rd)
        ib,ab=newton(a0.copy(),M,a0,rd,predict_mask=qw)
        ic,ac=newton(warm.copy(),M,a0,rd)
        A_its.append(ia);B_its.append(ib);C_its.append(ic)
    o.step(st,acts[k],flags=3,seed=3)
for nm,its in (("smooth",A_its),("smooth+predicted set",B_its),("warm start",C_its)):
    its=np.array(its); w=its.reshape(-1,8).max(axis=1)
    print(nm,"mean",its.mean().round(2),"hist",np.bincount(its)[:10],"wave8 max mean",w.mean().round(2),"hist",np.bincount(w)[:10])
