#!/usr/bin/env python3
"""FIR bit comparison (development tool): variants 0 (default), 7 (generic), 13 (matrix core), 14 (LDS-DMA
staging) against each other and the C oracle on 100,000 outputs."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from gsdr_amd import ops
from gsdr_amd.signals import lowpass_taps, uniform_iq
from oracle import oracle as o
D,T,N=4,127,100000
taps=lowpass_taps(T,0.1); x=uniform_iq((N-1)*D+T, seed=3)
tt=torch.from_numpy(taps).cuda(); xt=torch.from_numpy(x).cuda()
ys={v: ops.fir_variant(v, tt, xt, D, N).cpu().numpy() for v in (0, 7, 13, 14)}
ref=o.fir(taps,x,D,N)
for v,y in ys.items():
    print(v, "bitdiff vs generic:", int(np.sum(y.view(np.uint64)!=ys[7].view(np.uint64))), "vs oracle:", int(np.sum(y.view(np.uint64)!=ref.view(np.uint64))), "maxabs vs oracle", float(np.max(np.abs(y-ref))))
