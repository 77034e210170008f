#!/usr/bin/env python3
"""Per-call floor of short calls (development tool): back-to-back launches timed with HIP events for
  * a 256-element gsdrMagnitude (one workgroup: the launch floor itself),
  * gsdrFmDemod / gsdrxFmDemodInt8 direct calls and gsdrxStream calls at 2^16 / 2^18 / 2^20 input samples.
Run under `rocprofv3 --kernel-trace --stats` to split each call into kernel time and the gap between kernels."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
lib = abi.lib
T, D = 127, 4
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
NI = 1 << 26
x = (torch.rand(2 * NI, device=dev) * 2 - 1).view(torch.complex64)
x8 = torch.randint(-100, 100, (2 * NI,), dtype=torch.int8, device=dev)
y = torch.empty(NI // D + 4096, dtype=torch.float32, device=dev)
REPS = int(os.environ.get("REPS", "400"))


def timed(fn, reps=REPS):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


xm = x[:256]
ym = torch.empty(256, dtype=torch.float32, device=dev)
print(f"gsdrMagnitude 256: {timed(lambda i: lib.gsdrMagnitude(xm.data_ptr(), ym.data_ptr(), 256, 0, st)):.2f} us", flush=True)
for size in (1 << 16, 1 << 18, 1 << 20):
    n = (size - T) // D
    k = NI // size
    t_fm = timed(lambda i: lib.gsdrFmDemod(1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T,
                                           x.data_ptr() + 8 * size * (i % k), y.data_ptr(), n, 0, st))
    t_i8 = timed(lambda i: lib.gsdrxFmDemodInt8(1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T,
                                                x8.data_ptr() + 2 * size * (i % k), y.data_ptr(), n, 0, st))
    res = [f"{size} samples: gsdrFmDemod {t_fm:.2f} us, gsdrxFmDemodInt8 {t_i8:.2f} us"]
    for fmt, buf, sb in ((0, x, 8), (1, x8, 2)):
        h = ctypes.c_void_p()
        assert lib.gsdrxStreamCreate(ctypes.byref(h), 1, fmt, D, taps.data_ptr(), T, 1e6, 0.0, 1e5, 2e4, 0, 0) == 0
        w = ctypes.c_size_t()
        t = timed(lambda i: lib.gsdrxStreamProcess(h, buf.data_ptr() + sb * size * (i % k), size, y.data_ptr(),
                                                   y.numel(), ctypes.byref(w), st))
        lib.gsdrxStreamDestroy(h)
        res.append(f"stream {'CS8' if fmt else 'CF32'} {t:.2f} us")
    print(", ".join(res), flush=True)
