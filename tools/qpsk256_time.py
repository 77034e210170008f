"""Time gsdrQpsk256Demodulate (both constellations) on 2^24 noisy symbols with HIP events
(development tool; bench.py reports the same figures under secondary.qpsk256). Optional arguments:
other builds of libgsdr.so to time side by side on the same box."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import ops  # noqa: E402


def time_lib(path, syms, dev, g):
    lib = ctypes.CDLL(path)
    lib.gsdrQpsk256InitConstellation.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p]
    lib.gsdrQpsk256Demodulate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_int32, ctypes.c_void_p]
    n = syms.numel()
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = []
    for ctype, sigma in ((0, 0.02), (1, 0.01)):
        ops.qpsk256_init(ctype, 1.0)
        assert lib.gsdrQpsk256InitConstellation(ctype, 1.0, 0, stream) == 0
        rx = ops.qpsk256_modulate(syms, ctype)
        rx += torch.randn(n, dtype=torch.complex64, device=dev, generator=g) * (sigma * np.sqrt(2.0))
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        args = (rx.data_ptr(), out.data_ptr(), n, ctype, 0, stream)
        for _ in range(200):
            lib.gsdrQpsk256Demodulate(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 500
        e0.record()
        for _ in range(reps):
            lib.gsdrQpsk256Demodulate(*args)
        e1.record()
        torch.cuda.synchronize()
        ser = float((out != syms).float().mean())
        res.append(f"type {ctype}: {e0.elapsed_time(e1) / reps * 1e3:.2f} us ser {ser:.5f}")
    print(os.path.relpath(path, ROOT), " | ".join(res))


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    syms = torch.randint(0, 256, (1 << 24,), dtype=torch.uint8, device=dev, generator=g)
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(p) for p in sys.argv[1:]]
    for rep in range(2):
        for p in libs:
            time_lib(p, syms, dev, g)


if __name__ == "__main__":
    main()
