import sys; sys.path.insert(0, '.')
import numpy as np, torch
from scipy import signal
from gsdr_amd import ops
from oracle import oracle as o
cuda = torch.device('cuda:0')
b, a = signal.butter(6, 0.1); b = b.astype(np.float32); a = a.astype(np.float32)
x = np.random.default_rng(7).uniform(-1, 1, 2000).astype(np.float32)
xd = torch.from_numpy(x).to(cuda)
xh = torch.zeros(6, device=cuda); yh = torch.zeros(6, device=cuda)
bd, ad = torch.from_numpy(b).to(cuda), torch.from_numpy(a).to(cuda)
want_all, _, _ = o.iir(b, a, x)
pos = 0
for m in (1, 2, 3, 127, 129, 500, 1238):
    gxh, gyh = xh.cpu().numpy().copy(), yh.cpu().numpy().copy()
    y = ops.iir(bd, ad, xd[pos:pos + m], xh, yh).cpu().numpy()
    want, _, _ = o.iir(b, a, x[pos:pos + m], gxh, gyh)       # oracle from the GPU's own history
    seq, = [o.iir_f32(b, a, x[pos:pos + m], gxh, gyh)]
    print(m, 'gpu-vs-oracle(same hist)', np.max(np.abs(y - want)), 'seq32-vs-oracle', np.max(np.abs(seq - want)),
          'gpu-vs-mono', np.max(np.abs(y - want_all[pos:pos+m])), 'hist err', np.max(np.abs(gyh - (want_all[:pos][::-1][:6] if pos >= 6 else gyh))))
    pos += m
y = ops.iir(bd, ad, xd).cpu().numpy()
print('mono gpu vs oracle', np.max(np.abs(y - want_all)), 'seq32', np.max(np.abs(o.iir_f32(b, a, x) - want_all)))
