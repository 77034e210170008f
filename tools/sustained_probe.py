#!/usr/bin/env python3
"""Sustained-load probe (development tool): run each FC/D=4 variant back-to-back for many launches
(3 rotating input batches) and report the mean launch time per window of launches, so DVFS
(clock reduction under sustained power) shows up. Launches go through the C ABI directly (no
Python wrapper overhead), with a HIP event pair per window on the launch stream."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation variants (>= 100) exist only in the tuning-probe build (`make probes`)
os.environ.setdefault("GSDR_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build",
                                               "probes", "libgsdr_probes.so"))

import torch  # noqa: E402

from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

TAPS, D, N = 127, 4, 1 << 24
L = (N - 1) * D + TAPS
BYTES = 8 * L + 8 * N + 4 * TAPS

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,8,104,107,111")
ap.add_argument("--launches", type=int, default=400)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--cool", type=float, default=2.0, help="idle seconds before each variant")
ap.add_argument("--int8", action="store_true", help="int8 I/Q input (gsdrxFirFCInt8Variant)")
a = ap.parse_args()
if a.int8:
    BYTES = 2 * L + 8 * N + 4 * TAPS
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0x5EED)
if a.int8:
    xs = [torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=dev, generator=g) for _ in range(3)]
else:
    xs = [(torch.rand(2 * L, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(3)]
taps = torch.from_numpy(lowpass_taps(TAPS)).to(dev)
y = torch.empty(N, dtype=torch.complex64, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
fn = abi.lib.gsdrxFirFCInt8Variant if a.int8 else abi.lib.gsdrxFirFCVariant
for v in [int(s) for s in a.variants.split(",")]:
    argsets = [(v, D, taps.data_ptr(), TAPS, x.data_ptr(), y.data_ptr(), N, 0, stream) for x in xs]
    torch.cuda.synchronize()
    time.sleep(a.cool)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches // a.window + 1)]
    evs[0].record()
    for i in range(a.launches):
        rc = fn(*argsets[i % 3])
        assert rc == 0, rc
        if (i + 1) % a.window == 0:
            evs[(i + 1) // a.window].record()
    torch.cuda.synchronize()
    w = [evs[k].elapsed_time(evs[k + 1]) / a.window * 1e3 for k in range(len(evs) - 1)]
    print(f"variant {v:4d}: us/launch per {a.window}-launch window: " + " ".join(f"{t:6.1f}" for t in w)
          + f"   | steady {w[-1]:.1f} us = {BYTES / (w[-1] * 1e-6) / 1e9:.0f} GB/s", flush=True)
