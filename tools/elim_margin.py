"""Action elimination at Na = 20,000, on CPU: how many candidates can never be
eliminated per state for a given margin E (a candidate k is provably never the argmax again once
f(k) < max f - E, E = beta/(1-beta)*||dV|| >= 24*tol = 2.4e-4 over the whole solve).  Every 97th
state of each row, the objective of Aiyagari_VFI.m:70-83 at a near-converged V (the Na = 400
solution interpolated, as tests/test_vfi_gpu.py).  Tool only: uses the oracle."""
import numpy as np, sys
import os; sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from oracle import corc, np_oracle as no
cal = no.calib_aiyagari(Na=20000, shocks="rouwenhorst")
a, s, P = cal["a_grid"], cal["s"], cal["P"]
r=0.04; w = no.wage(r, 0.36, 0.08); beta=0.96; sig=5.0
c4 = no.calib_aiyagari(Na=400, shocks="rouwenhorst")
V4 = corc.vfi_solve(np.zeros((7, 400)), c4["a_grid"], c4["s"], c4["P"], r, w, beta, sig)["v_new"]
V = np.stack([np.interp(a, c4["a_grid"], V4[i]) for i in range(7)])
EV = beta * P @ V
Na=a.size
for E in (2.4e-4, 4.8e-4, 1e-2, 0.1):
    cnt=[]; span=[]
    for i in range(7):
        for j in range(0, Na, 97):
            coh=(1+r)*a[j]+w*s[i]
            kf=np.searchsorted(a, coh)  # a_k < coh
            c=coh-a[:kf]
            f=(c**(1-sig)-1)/(1-sig)+EV[i,:kf]
            fs=f.max()
            live=np.nonzero(f>=fs-E)[0]
            cnt.append(live.size); span.append(live[-1]-live[0]+1)
    print(f"E={E:g}: candidates never eliminable per state: median {int(np.median(cnt))} p90 {int(np.percentile(cnt,90))}; live interval median {int(np.median(span))} max {max(span)}")
