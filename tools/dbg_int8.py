import sys; sys.path.insert(0, '.')
import numpy as np, torch
from gsdr_amd import ops
from oracle import oracle as o
cuda = torch.device('cuda:0')
v = np.arange(-128, 128, dtype=np.int8)
x = np.zeros(2 * 2 * 256, np.int8)
x[0::4], x[1::4] = v, v[::-1]
for D in (2, 3):
    y = ops.fir(torch.tensor([1.0], device=cuda), torch.from_numpy(x).to(cuda), D).cpu().numpy()
    want = o.int8_to_float(x).view(np.complex64)[0::D]
    print(D, y[:4], want[:4], np.sum(y != want[:y.size]))
conv = ops.int8_to_norm_float(torch.from_numpy(x).to(cuda)).cpu().numpy()
print('conv', conv[:8], o.int8_to_float(x)[:8])
