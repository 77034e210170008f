"""Per-call cost of short float calls (development tool): config 2's complex64 channel through a gsdrxStream
(CF32 FIR, D = 4; then the FM chain) in 1 / 8 / 32 / 128 chunks a pass, against one gsdrFirFC / gsdrFmDemod
call (HIP events)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

D, T, N_IN = 4, 127, 67_108_987
N_OUT = (N_IN - T) // D + 1
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
g = torch.Generator(device=dev).manual_seed(3)
xs = [(torch.rand(2 * N_IN, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(2)]
y = torch.empty(N_OUT + 1024, dtype=torch.complex64, device=dev)


def timed(fn, args, reps):
    k = 0
    for _ in range(max(20, reps // 5)):
        assert fn(*args[k % len(args)]) == 0
        k += 1
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(*args[k % len(args)])
        k += 1
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = ["gsdrFirFC %.1f" % timed(abi.lib.gsdrFirFC, [(D, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(), N_OUT, 0, stream)
                                                    for x in xs], 60)]
written = ctypes.c_size_t()
f = ctypes.c_float
N_FM = (N_IN - T) // D
res.append("gsdrFmDemod %.1f" % timed(abi.lib.gsdrFmDemod, [(f(1e6), f(0.0), f(1e5), f(2e4), D, 0, taps.data_ptr(), T,
                                                             x.data_ptr(), y.data_ptr(), N_FM, 0, stream) for x in xs], 60))
for kind in (0, 1):
    for chunks in (1, 8, 32, 128):
        h = ctypes.c_void_p()
        assert abi.lib.gsdrxStreamCreate(ctypes.byref(h), kind, 0, D, taps.data_ptr(), T, f(1e6), f(0.0), f(1e5),
                                         f(2e4), 0, 0) == 0
        cs = N_IN // chunks
        args = []
        for x in xs:
            for c in range(chunks):
                n = cs if c < chunks - 1 else N_IN - cs * (chunks - 1)
                args.append((h, x.data_ptr() + 8 * cs * c, n, y.data_ptr(), y.numel(), ctypes.byref(written), stream))
        res.append("%s stream x%d %.1f" % ("fir" if kind == 0 else "fm", chunks,
                                           timed(abi.lib.gsdrxStreamProcess, args, 20 * chunks) * chunks))
        abi.lib.gsdrxStreamDestroy(h)
print(" | ".join(res), "(us per channel pass)")
