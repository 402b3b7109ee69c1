"""Pre-filter selectivity on the synthetic generators: % of centres passing the cardinal
test, cardinal + diagonal test, and the full segment test."""
import sys; import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, workloads
DX=[0,1,2,3,3,3,2,1,0,-1,-2,-3,-3,-3,-2,-1]; DY=[-3,-3,-2,-1,0,1,2,3,3,3,2,1,0,-1,-2,-3]
def stats(img,t,n):
    h,w=img.shape; I=img.astype(np.int16); c=I[3:h-3,3:w-3]
    def px(i): return I[3+DY[i]:h-3+DY[i], 3+DX[i]:w-3+DX[i]]
    b=[px(i)-c>t for i in range(16)]; d=[px(i)-c< -t for i in range(16)]
    def pair(f,ks): return (f[ks[0]]|f[ks[2]])&(f[ks[1]]|f[ks[3]])
    def tri(f,ks):
        a,b_,c_,d_=[f[k] for k in ks]; return (a&b_&(c_|d_))|(c_&d_&(a|b_))
    test=pair if n<12 else tri
    card=test(b,[0,4,8,12])|test(d,[0,4,8,12])
    diag_b=test(b,[2,6,10,14]); diag_d=test(d,[2,6,10,14])
    both=(test(b,[0,4,8,12])&diag_b)|(test(d,[0,4,8,12])&diag_d)
    def arc(f):   # some cyclic run of >= n set flags (segment test, numpy)
        out=np.zeros_like(f[0])
        for s_ in range(16):
            run=np.ones_like(f[0])
            for k in range(n): run&=f[(s_+k)%16]
            out|=run
        return out
    kp=int((arc(b)|arc(d)).sum())
    N=c.size
    return card.sum()/N*100, both.sum()/N*100, kp/N*100
for name,img in (("s1",workloads.s1_frame(3)),("s2",workloads.s2_frame(1)),("s3",workloads.s3_frame(2))):
    for t,n in ((16,9),(8,12),(30,9)):
        print(name,t,n,["%.2f%%"%v for v in stats(img,t,n)])
