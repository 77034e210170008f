"""Time gsdrFirFC (D = 4, T = 127, 2^26 samples) with the input pointer offset by 0, 1 and 2 complex samples
(16-, 8- and 16-byte aligned) -- the cost of the per-sample staging path (development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device('cuda', 0)
n_in, T, D = (1 << 26) + 8, 127, 4
x = (torch.rand(2 * n_in, device=dev) * 2 - 1).view(torch.complex64)
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
stream = torch.cuda.current_stream(dev).cuda_stream
N = (n_in - 8 - T) // D + 1
y = torch.empty(N, dtype=torch.complex64, device=dev)
for off in (0, 1, 2, 0, 1):
    a = (D, taps.data_ptr(), T, x.data_ptr() + 8 * off, y.data_ptr(), N, 0, stream)
    for _ in range(20): abi.lib.gsdrFirFC(*a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100): abi.lib.gsdrFirFC(*a)
    e1.record(); torch.cuda.synchronize()
    print('offset', off, 'samples:', round(e0.elapsed_time(e1) / 100 * 1e3, 1), 'us')
