#!/usr/bin/env python3
"""Kernel time of the D = 4 FIR tile shapes on short calls (development tool): gsdrxFirFCVariant 0 (WG 256,
R 4), 28 (WG 128, R 4), 24 (WG 64, R 4), 25 (WG 256, R 2), 26 (WG 256, R 1) at 2 M / 524 K / 131 K outputs
(a 64 M-sample channel cut in 8 / 32 / 128 stream calls), HIP events around back-to-back launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device("cuda", 0)
taps = torch.from_numpy(lowpass_taps(127, 0.1)).to(dev)
x = (torch.rand(2 * 67_108_987, device=dev) * 2 - 1).view(torch.complex64)
y = torch.empty(1 << 24, dtype=torch.complex64, device=dev)
for n in (2097156, 524289, 131073):
    res = []
    for v in (0, 28, 24, 25, 26):
        xs = [x[k * 4 * n: k * 4 * n + 4 * (n - 1) + 127] for k in range(7)]
        for i in range(20):
            ops.fir_variant(v, taps, xs[i % 7], 4, n, out=y[:n])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            ops.fir_variant(v, taps, xs[i % 7], 4, n, out=y[:n])
        e1.record()
        torch.cuda.synchronize()
        res.append(f"v{v} {e0.elapsed_time(e1) / 200 * 1e3:.1f}")
    print(f"N = {n}: " + " | ".join(res) + " us", flush=True)
