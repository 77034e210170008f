"""Time gsdrFirFF (real samples) and gsdrxFirFCInt8 (int8 I/Q) at D = 4, T = 127, 2^26 samples with the input
pointer offset by 0..3 elements -- the cost of the per-sample staging path these inputs take when the
tile start is not 16-byte aligned (development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device('cuda', 0)
n_in, T, D = (1 << 26) + 16, 127, 4
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
stream = torch.cuda.current_stream(dev).cuda_stream
N = (n_in - 16 - T) // D + 1


def timed(fn, args):
    for _ in range(20):
        assert fn(*args) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        fn(*args)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / 100 * 1e3, 1)


xf = torch.rand(n_in, device=dev) * 2 - 1
yf = torch.empty(N, dtype=torch.float32, device=dev)
for off in (0, 1, 2, 3, 0, 1, 2, 3):
    a = (D, taps.data_ptr(), T, xf.data_ptr() + 4 * off, yf.data_ptr(), N, 0, stream)
    us = timed(abi.lib.gsdrFirFF, a)
    print('FF offset', off, 'floats (', 4 * off, 'B):', us, 'us', flush=True)

xi = torch.randint(-128, 128, (2 * n_in,), dtype=torch.int8, device=dev)
yc = torch.empty(N, dtype=torch.complex64, device=dev)
for off in (0, 1, 2, 3, 0, 1, 2, 3):
    a = (D, taps.data_ptr(), T, xi.data_ptr() + 2 * off, yc.data_ptr(), N, 0, stream)
    us = timed(abi.lib.gsdrxFirFCInt8, a)
    print('Int8 offset', off, 'samples (', 2 * off, 'B):', us, 'us', flush=True)
