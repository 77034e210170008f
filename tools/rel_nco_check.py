#!/usr/bin/env python3
"""Checks the tile-relative NCO probe (variant 127) against the default FM kernel (120) on config 3's
shape: the discriminator is invariant to a rotation common to a tile, so the outputs must agree to the
wrapped-angle bar. Development tool (probes build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GSDR_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build",
                                               "probes", "libgsdr_probes.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import fm_test_signal, lowpass_taps  # noqa: E402

TAPS, D, N = 127, 4, 1 << 22
L = (N - 1) * D + TAPS
dev = torch.device("cuda", 0)
x = torch.from_numpy(fm_test_signal(L, carrier=-0.1, seed=3)).to(dev)
taps = torch.from_numpy(lowpass_taps(TAPS)).to(dev)
outs = {}
for v in (120, 127, 128):
    y = torch.zeros(N, dtype=torch.complex64, device=dev)
    ops.fir_variant(v, taps, x, D, N, out=y)
    torch.cuda.synchronize()
    outs[v] = y.view(torch.float32)[: N - 1].cpu().numpy()
g = 7.957747
for v in (127, 128):
    d = np.remainder(outs[v] - outs[120] + np.pi * g, 2 * np.pi * g) - np.pi * g
    print(f"variant {v} vs default: max wrapped diff / (pi g) = {np.max(np.abs(d)) / (np.pi * g):.3e}")
