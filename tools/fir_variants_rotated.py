#!/usr/bin/env python3
"""Headline-shape FIR tile variants (gsdrxFirFCVariant) timed side by side with inputs AND outputs rotating over 3
buffer sets (bench.py's timed region since round 6), and each also on one fixed output buffer (development tool):
    python tools/fir_variants_rotated.py [variant ...]      (default 0 8 10 11 14)
Interleaved over ROUNDS rounds in one process; min / median us per launch."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "5"))
REPS = int(os.environ.get("REPS", "60"))


def main():
    variants = [int(v) for v in sys.argv[1:]] or [0, 8, 10, 11, 14]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(5)
    D, T, NO = 4, 127, 1 << 24
    NI = (NO - 1) * D + T
    taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    xs = [(torch.rand(2 * NI, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(3)]
    ys = [torch.empty(NO, dtype=torch.complex64, device=dev) for _ in range(3)]
    fn = abi.lib.gsdrxFirFCVariant
    res = {}
    for _ in range(400):  # clock ramp
        assert fn(0, D, taps.data_ptr(), T, xs[0].data_ptr(), ys[0].data_ptr(), NO, 0, st) == 0
    for r in range(ROUNDS):
        for v in variants[r % len(variants):] + variants[:r % len(variants)]:
            for mode in ("rotated", "one_output"):
                for k in range(6):
                    assert fn(v, D, taps.data_ptr(), T, xs[k % 3].data_ptr(), ys[k % 3].data_ptr(), NO, 0, st) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for k in range(REPS):
                    y = ys[k % 3] if mode == "rotated" else ys[0]
                    fn(v, D, taps.data_ptr(), T, xs[k % 3].data_ptr(), y.data_ptr(), NO, 0, st)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((v, mode), []).append(e0.elapsed_time(e1) / REPS * 1e3)
    for v in variants:
        cols = []
        for mode in ("rotated", "one_output"):
            t = sorted(res[(v, mode)])
            cols.append(f"{mode} {t[0]:7.2f} / {t[len(t) // 2]:7.2f}")
        print(f"variant {v:3d}   " + "   ".join(cols) + "   us (min / median)", flush=True)


if __name__ == "__main__":
    main()
