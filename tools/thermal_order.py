#!/usr/bin/env python3
"""Whether the config-5 kernels time slower after the power-capped FIR (development tool): AWGN modulate and
rectangular demod timed alone, then after 3 s of back-to-back headline FIR launches, then after a 2 s idle."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 24
ops.qpsk256_init(0, 1.0, 0)
syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
tx = torch.empty(n, dtype=torch.complex64, device=dev)
dec = torch.empty(n, dtype=torch.uint8, device=dev)
taps = torch.from_numpy(lowpass_taps(127, 0.1)).to(dev)
NI = 67_108_987
x = (torch.rand(2 * NI, device=dev) * 2 - 1).view(torch.complex64)
y = torch.empty(1 << 24, dtype=torch.complex64, device=dev)


def q5(label):
    res = []
    for fn in (lambda: ops.qpsk256_modulate_awgn(syms, 0, 0.02, 0x5EED0005, 0, out=tx),
               lambda: ops.qpsk256_demodulate(tx, 0, out=dec)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / 50)
    print(f"{label:28s} mod_awgn {res[0]:6.2f}  demod {res[1]:6.2f} us", flush=True)


def direct(label):
    """The same two entry points through the C-ABI directly (prebuilt ctypes arguments, as tools/ab_ref.py), and
    the host time per call of the ops wrapper."""
    from gsdr_amd.abi import lib

    st = torch.cuda.current_stream(dev).cuda_stream
    fa = (syms.data_ptr(), tx.data_ptr(), n, 0, 0.02, 0x5EED0005, 0, 0, st)
    fd = (tx.data_ptr(), dec.data_ptr(), n, 0, 0, st)
    res = []
    for f, a in ((lib.gsdrxQpsk256ModulateAwgn, fa), (lib.gsdrQpsk256Demodulate, fd)):
        f(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f(*a)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / 50)
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(50):
        ops.qpsk256_modulate_awgn(syms, 0, 0.02, 0x5EED0005, 0, out=tx)
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{label:28s} mod_awgn {res[0]:6.2f}  demod {res[1]:6.2f} us (direct C-ABI); ops wrapper host "
          f"{(h1 - h0) / 50 * 1e6:.1f} us a call", flush=True)


direct("direct, cold")
q5("cold")
q5("cold again")
t0 = time.time()
while time.time() - t0 < 3.0:
    for _ in range(50):
        ops.fir(taps, x, 4, out=y)
    torch.cuda.synchronize()
q5("after 3 s of FIR")
time.sleep(2.0)
q5("after 2 s idle")
direct("direct, after")
