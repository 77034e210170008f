"""Development probe: FM chain (config 3 shape) accuracy vs the oracle and sustained per-launch time.
The NCO implementation is taken from GSDR_NCO_IMPL by the library (probe switch)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gsdr_amd import abi, ops
from gsdr_amd.signals import fm_test_signal, lowpass_taps
from oracle import oracle as orc

ap = argparse.ArgumentParser()
ap.add_argument("--launches", type=int, default=800)
ap.add_argument("--window", type=int, default=100)
ap.add_argument("--mode", default="fm")
a = ap.parse_args()
dev = torch.device("cuda:0")
fs, tune, chan, dhz, D, T = 1.0e6, 0.0, 1.0e5, 2.0e4, 4, 127
taps = lowpass_taps(T)
td = torch.from_numpy(taps).to(dev)
# accuracy: 256 K outputs of a real FM signal, n0 large so the phase wraps
n = 1 << 18
n0 = 123_456_789_013
x = fm_test_signal(n * D + T, n0=n0)
xd = torch.from_numpy(x).to(dev)
if a.mode == "fm":
    got = ops.fm_demod(xd, td, fs, tune, chan, dhz, D, n0, n).cpu().numpy()
    want = orc.fm_demod(x, taps, fs, tune, chan, dhz, D, n0, n)
    g = fs / (2 * np.pi * dhz)
    d = np.remainder(got.astype(np.float64) - want + np.pi * g, 2 * np.pi * g) - np.pi * g
    print(f"impl {os.environ.get('GSDR_NCO_IMPL', '0')}: max wrapped err / (pi g) = {np.max(np.abs(d)) / (np.pi * g):.3e}")
# timing at config 3
n_fm = (1 << 24) - 1
n_in = n_fm * D + T
gen = torch.Generator(device=dev).manual_seed(1)
xs = [(torch.rand(2 * n_in, device=dev, generator=gen) * 2 - 1).view(torch.complex64) for _ in range(3)]
y = torch.empty(n_fm, dtype=torch.float32, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
args = [(fs, tune, chan, dhz, D, 0, td.data_ptr(), T, xx.data_ptr(), y.data_ptr(), n_fm, 0, st) for xx in xs]
fn = abi.lib.gsdrFmDemod
if a.mode == "am":
    fn = abi.lib.gsdrAmDemod
    args = [(fs, tune, chan, D, 0, td.data_ptr(), T, xx.data_ptr(), y.data_ptr(), n_fm, 0, st) for xx in xs]
res = []
i = 0
for w in range(a.launches // a.window):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.window):
        fn(*args[i % 3])
        i += 1
    e.record()
    torch.cuda.synchronize()
    res.append(s.elapsed_time(e) / a.window * 1e3)
print(f"{a.mode} impl {os.environ.get('GSDR_NCO_IMPL', '0')}: us/launch per window " + " ".join(f"{r:.1f}" for r in res)
      + f" | steady {res[-1]:.1f} us = {(8 * n_in + 4 * n_fm) / res[-1] / 1e3:.0f} GB/s")
