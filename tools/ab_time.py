#!/usr/bin/env python3
"""A/B timing of builds of libgsdr.so in one process (development tool). Workloads at the bench
shapes: config 2 (gsdrFirFC, D = 4, T = 127, 2^24 outputs), config 3 (gsdrFmDemod), the AM chain and
the int8 FIR, each over 3 rotating input batches. Rounds alternate the builds; each measurement is a
clock settle (untimed launches) and then 100 launches inside one HIP event pair. Prints the median
per build and workload, and whether outputs equal the first build's bit for bit.

    python tools/ab_time.py [other_lib.so ...]     (the in-tree gsdr_amd/libgsdr.so is always first)
    AB_WORK=fir,fm,fm16  AB_ROUNDS=3   (fm16: gsdrxFmDemodMulti, 16 channels, time per launch;
                                       fir8 / fm8 / am8: the int8 I/Q entry points)
"""
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd.signals import lowpass_taps  # noqa: E402

D, T, N = 4, 127, 1 << 24
FS, TUNE, CHAN, DEV = 1.0e6, 0.0, 1.0e5, 2.0e4


def fm_channel(n, dev, seed, n0):
    import math
    idx = torch.arange(n0, n0 + n, dtype=torch.float64, device=dev)
    ph = 2 * math.pi * 0.1 * idx + 20.0 * torch.sin(2 * math.pi * 0.001 * idx)
    x = torch.polar(torch.ones_like(ph), ph).to(torch.complex64)
    g = torch.Generator(device=dev).manual_seed(seed)
    x += (torch.randn(2 * n, dtype=torch.float32, device=dev, generator=g) * 0.05).view(torch.complex64)
    return x


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(p) for p in sys.argv[1:]]
    work = os.environ.get("AB_WORK", "fir,fm,am,fir8").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    n_in = N * D + T
    g = torch.Generator(device=dev).manual_seed(7)
    xs = [fm_channel(n_in, dev, 100 + k, k * n_in) for k in range(3)]
    x8 = [torch.randint(-128, 128, (2 * n_in,), dtype=torch.int8, device=dev, generator=g) for _ in range(3)] \
        if "fir8" in work else []
    # config 3's signal quantised to int8 I/Q (the int8 chains)
    q8 = [torch.clamp(torch.round(torch.view_as_real(x).reshape(-1) * 100), -128, 127).to(torch.int8) for x in xs] \
        if ("fm8" in work or "am8" in work) else []
    yc = torch.empty(N, dtype=torch.complex64, device=dev)
    yf = torch.empty(N, dtype=torch.float32, device=dev)
    nch = 16
    ym = torch.empty(nch * (N - 1), dtype=torch.float32, device=dev) if "fm16" in work else yf
    chans = (ctypes.c_float * nch)(*[CHAN - 3.0e4 * k for k in range(nch)])
    devs = (ctypes.c_float * nch)(*([DEV] * nch))
    F, U32, SZ, P, I32 = ctypes.c_float, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32
    specs = {
        "fir": ("gsdrFirFC", [SZ, P, SZ, P, P, SZ, I32, P], yc,
                lambda x: (D, taps.data_ptr(), T, x.data_ptr(), yc.data_ptr(), N, 0, stream), xs),
        "fm": ("gsdrFmDemod", [F, F, F, F, U32, SZ, P, SZ, P, P, SZ, I32, P], yf,
               lambda x: (FS, TUNE, CHAN, DEV, D, 0, taps.data_ptr(), T, x.data_ptr(), yf.data_ptr(), N - 1, 0, stream),
               xs),
        "am": ("gsdrAmDemod", [F, F, F, U32, SZ, P, SZ, P, P, SZ, I32, P], yf,
               lambda x: (FS, TUNE, CHAN, D, 0, taps.data_ptr(), T, x.data_ptr(), yf.data_ptr(), N, 0, stream), xs),
        "fm16": ("gsdrxFmDemodMulti", [F, F, P, P, U32, U32, SZ, P, SZ, ctypes.c_int, P, P, SZ, I32, P], ym,
                 lambda x: (FS, TUNE, ctypes.cast(chans, P), ctypes.cast(devs, P), nch, D, 0, taps.data_ptr(), T, 0,
                            x.data_ptr(), ym.data_ptr(), N - 1, 0, stream), xs),
        "fir8": ("gsdrxFirFCInt8", [SZ, P, SZ, P, P, SZ, I32, P], yc,
                 lambda x: (D, taps.data_ptr(), T, x.data_ptr(), yc.data_ptr(), N, 0, stream), x8),
        "fm8": ("gsdrxFmDemodInt8", [F, F, F, F, U32, SZ, P, SZ, P, P, SZ, I32, P], yf,
                lambda x: (FS, TUNE, CHAN, DEV, D, 0, taps.data_ptr(), T, x.data_ptr(), yf.data_ptr(), N - 1, 0,
                           stream), q8),
        "am8": ("gsdrxAmDemodInt8", [F, F, F, U32, SZ, P, SZ, P, P, SZ, I32, P], yf,
                lambda x: (FS, TUNE, CHAN, D, 0, taps.data_ptr(), T, x.data_ptr(), yf.data_ptr(), N, 0, stream),
                q8),
    }
    handles = [ctypes.CDLL(p) for p in libs]
    res = {(li, w): [] for li in range(len(libs)) for w in work}
    first_out, same = {}, {}
    for r in range(rounds):
        for li, lib in enumerate(handles):
            for w in work:
                name, argt, y, mk, inputs = specs[w]
                fn = getattr(lib, name)
                fn.argtypes = argt
                args = [mk(x) for x in inputs]
                for i in range(150):
                    assert fn(*args[i % 3]) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(100):
                    fn(*args[i % 3])
                e1.record()
                torch.cuda.synchronize()
                res[(li, w)].append(e0.elapsed_time(e1) * 10.0)  # us per launch
                assert fn(*args[0]) == 0
                torch.cuda.synchronize()
                out = y.clone()
                if li == 0:
                    first_out[w] = out
                else:
                    same[(li, w)] = torch.equal(out.view(torch.uint8), first_out[w].view(torch.uint8))
    for li, p in enumerate(libs):
        cells = []
        for w in work:
            v = res[(li, w)]
            s = f"{w} {statistics.median(v):7.2f} us (min {min(v):.2f})"
            if li > 0:
                s += " =" if same[(li, w)] else " differs"
            cells.append(s)
        print(f"{os.path.relpath(p, ROOT):40s} " + " | ".join(cells), flush=True)


if __name__ == "__main__":
    main()
