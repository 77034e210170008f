#!/usr/bin/env python3
"""Tuning probe for the headline FIR (FC, D=4, T=127, 2^24 outputs): times gsdrxFirFCVariant tile
shapes and ablations (variants >= 100, see launch_fc_probe in gsdr_amd/csrc/fir.hip) interleaved in one process,
HIP events on the launch stream. Development tool; not part of the library."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation variants (>= 100) exist only in the tuning-probe build (`make probes`)
os.environ.setdefault("GSDR_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build",
                                               "probes", "libgsdr_probes.so"))

import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

TAPS, D, N = 127, 4, 1 << 24
L = (N - 1) * D + TAPS
BYTES = 8 * L + 8 * N + 4 * TAPS

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="0,1,3,4,5,8,24,28,104,107,111")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--fm", action="store_true", help="also time the fused FM chain")
ap.add_argument("--buffers", type=int, default=3, help="input buffers rotated per launch (3 x 537 MB defeats the 256 MB MALL)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0x5EED)
xs = [(torch.rand(2 * L, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(a.buffers)]
x = xs[0]
taps = torch.from_numpy(lowpass_taps(TAPS)).to(dev)
y = torch.empty(N, dtype=torch.complex64, device=dev)
variants = [int(v) for v in a.variants.split(",")]
res = {v: [] for v in variants}
for r in range(a.rounds):
    for v in variants:
        for i in range(2):
            ops.fir_variant(v, taps, xs[i % len(xs)], D, N, out=y)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(a.reps):
            ops.fir_variant(v, taps, xs[i % len(xs)], D, N, out=y)
        e.record()
        torch.cuda.synchronize()
        res[v].append(s.elapsed_time(e) / a.reps * 1e3)
print(f"{'variant':>8} {'us(min)':>9} {'us(med)':>9} {'alg GB/s':>9}")
for v in variants:
    t = sorted(res[v])
    print(f"{v:>8} {t[0]:9.2f} {t[len(t) // 2]:9.2f} {BYTES / (t[0] * 1e-6) / 1e9:9.1f}")
if a.fm:
    out = torch.empty(N - 1, dtype=torch.float32, device=dev)
    xf = x[: (N - 1) * D + TAPS]
    for _ in range(3):
        ops.fm_demod(xf, taps, 1e6, 0.0, 1e5, 2e4, D, 0, N - 1, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        ops.fm_demod(xf, taps, 1e6, 0.0, 1e5, 2e4, D, 0, N - 1, out=out)
    e.record()
    torch.cuda.synchronize()
    print(f"fm chain {s.elapsed_time(e) / a.reps * 1e3:.2f} us")
