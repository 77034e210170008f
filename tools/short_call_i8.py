#!/usr/bin/env python3
"""int8 I/Q matrix-core FIR tile shapes on short calls (development tool; also runs under rocprofv3
--kernel-trace): gsdrxFirFCInt8Variant 41 (default), 43 (512-output tiles, 3 workgroups a CU), 44 (512, 4 a CU),
45 (512, 3 a CU, two tiles in flight), 46 (512, 4 a CU, two in flight) at 2.1 M / 524 K / 131 K outputs (a 64 M-sample
channel cut in 8 / 32 / 128 stream calls) and 16.8 M (one call). Prints HIP-event time per call over back-to-back calls."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "41,43,44,45,46").split(",")]
dev = torch.device("cuda", 0)
taps = torch.from_numpy(lowpass_taps(127, 0.1)).to(dev)
x = torch.randint(-100, 100, (2 * 67_108_987,), dtype=torch.int8, device=dev)
y = torch.empty(1 << 24, dtype=torch.complex64, device=dev)
print("outputs   " + " ".join(f"{v:>8d}" for v in VARIANTS) + "   (us a call, min of 5 rounds)")
for n in (2097156, 524289, 131073, 16777216):
    k_max = max(1, min(7, (x.numel() // 2 - 127) // (4 * n)))
    xs = [x[2 * k * 4 * n: 2 * (k * 4 * n + 4 * (n - 1) + 127)] for k in range(k_max)]
    reps = max(20, min(200, (1 << 25) // n))
    res = []
    for v in VARIANTS:
        best = 1e30
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ops.fir_variant(v, taps, xs[0], 4, n, out=y[:n])
            e0.record()
            for i in range(reps):
                ops.fir_variant(v, taps, xs[i % k_max], 4, n, out=y[:n])
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
        res.append(best)
    print(f"{n:9d} " + " ".join(f"{r:8.2f}" for r in res), flush=True)
