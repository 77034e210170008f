"""Per-launch time of gsdrxFirFCInt8 / gsdrxFmDemodInt8 (decimation 4, T = 127) against the number of
outputs per call, back-to-back launches with pre-marshalled ctypes arguments, HIP events (development
tool: separates the matrix-core kernels' fixed per-launch cost from their streaming rate)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    D, T = 4, 127
    nmax = 1 << 24
    L = nmax * D + T + 8
    g = torch.Generator(device=dev).manual_seed(3)
    x8 = torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=dev, generator=g)
    taps = torch.from_numpy(lowpass_taps(T)).to(dev)
    yc = torch.empty(nmax, dtype=torch.complex64, device=dev)
    yf = torch.empty(nmax, dtype=torch.float32, device=dev)
    for n in (1 << 24, 1 << 22, 1 << 21, 1 << 20, 1 << 18, 1 << 16, 1 << 12):
        row = []
        for name in ("gsdrxFirFCInt8", "gsdrxFmDemodInt8"):
            fn = getattr(abi.lib, name)
            reps = max(20, min(2000, (1 << 26) // n))
            if name == "gsdrxFirFCInt8":
                args = [(D, taps.data_ptr(), T, x8.data_ptr() + 2 * D * ((k * n) % (nmax - n + 1)), yc.data_ptr(), n, 0,
                         stream) for k in range(4)]
            else:
                args = [(1.0e6, 0.0, 1.0e5, 2.0e4, D, 0, taps.data_ptr(), T,
                         x8.data_ptr() + 2 * D * ((k * n) % (nmax - n + 1)), yf.data_ptr(), n - 1, 0, stream)
                        for k in range(4)]
            for i in range(50):
                assert fn(*args[i % 4]) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(reps):
                fn(*args[i % 4])
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            row.append(f"{name} {us:9.2f} us ({n * D / us / 1e3:8.1f} GS/s)")
        print(f"N = 2^{n.bit_length() - 1:2d}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
