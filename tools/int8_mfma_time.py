"""Time gsdrxFirFCInt8Variant shapes (default 0 = packed-VALU polyphase, 40 = matrix cores) on config 2
from int8 I/Q (2^24 outputs, D = 4, T = 127), interleaved, HIP events (development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1:]] or [0, 40]
    dev = torch.device("cuda", 0)
    n, D, T = 1 << 24, 4, 127
    L = (n - 1) * D + T
    g = torch.Generator(device=dev).manual_seed(5)
    x8 = torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=dev, generator=g)
    taps = torch.from_numpy(lowpass_taps(T)).to(dev)
    out = torch.empty(n, dtype=torch.complex64, device=dev)
    for v in variants:
        for _ in range(100):
            ops.fir_variant(v, taps, x8, D, n, out=out)
    torch.cuda.synchronize()
    for rep in range(3):
        line = []
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(100):
                ops.fir_variant(v, taps, x8, D, n, out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 100 * 1e3
            line.append(f"v{v} {us:7.2f} us ({(2 * L + 8 * n) / us / 1e3:6.0f} GB/s alg)")
        print(" | ".join(line))


if __name__ == "__main__":
    main()
