#!/usr/bin/env python3
"""int8 multi-channel FM / AM (gsdrxFmDemodMulti / gsdrxAmDemodMulti, int8 I/Q, D = 4) per channel (development
tool): T = 132 takes one matrix-core chain launch per channel (the input read C times); T = 133 is
past the matrix-core chain's tap limit and takes the grouped float-engine kernel (input staged once for all
channels). One extra tap is < 1 % more work, so the two columns compare the two forms."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

dev = torch.device("cuda", 0)
L = 67_108_987
x = torch.randint(-100, 100, (2 * L,), dtype=torch.int8, device=dev)
print(f"{'mode':4s} {'C':>3s} {'T=132 us/ch':>12s} {'T=133 us/ch':>12s}")
for fm in (True, False):
    for C in (1, 8, 16):
        chans = [1e4 * (c - C / 2) for c in range(C)]
        res = []
        for T in (132, 133):
            taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
            N = (L - T) // 4 - 1
            if fm:
                run = lambda: ops.fm_demod_multi(x, taps, 1e6, 0.0, chans, [2e4] * C, 4, num_outputs=N)  # noqa: E731
            else:
                run = lambda: ops.am_demod_multi(x, taps, 1e6, 0.0, chans, 4, num_outputs=N)  # noqa: E731
            run()
            torch.cuda.synchronize()
            best = 1e30
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    y = run()
                    del y
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / 3 / C)
            res.append(best)
        print(f"{'FM' if fm else 'AM':4s} {C:3d} {res[0]:12.1f} {res[1]:12.1f}", flush=True)
