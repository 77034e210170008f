#!/usr/bin/env python3
"""int8 I/Q matrix-core FIR tile sizes on short calls (development tool, run under rocprofv3 --kernel-trace):
gsdrxFirFCInt8Variant 41 (default: 2,048-output tiles, 512 for calls under two rounds of slots), 42 (1,024) and
43 (512) at 2.1 M / 524 K / 131 K outputs (a 64 M-sample channel cut in 8 / 32 / 128 stream calls)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device("cuda", 0)
taps = torch.from_numpy(lowpass_taps(127, 0.1)).to(dev)
x = torch.randint(-100, 100, (2 * 67_108_987,), dtype=torch.int8, device=dev)
y = torch.empty(1 << 24, dtype=torch.complex64, device=dev)
for n in (2097156, 524289, 131073):
    xs = [x[2 * k * 4 * n: 2 * (k * 4 * n + 4 * (n - 1) + 127)] for k in range(7)]
    for v in (41, 42, 43):
        for i in range(220):
            ops.fir_variant(v, taps, xs[i % 7], 4, n, out=y[:n])
    torch.cuda.synchronize()
    print(f"N = {n} done", flush=True)
