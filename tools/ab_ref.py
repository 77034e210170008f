#!/usr/bin/env python3
"""Side-by-side timing of the working tree's libgsdr.so against an earlier build (development tool):
    python tools/ab_ref.py build/ref_50fdf7b/libgsdr.so
Each entry point on its bench shape, both libraries interleaved over ROUNDS rounds in one process on the same
buffers (HIP events around back-to-back launches; min over rounds), so box-to-box spread cancels. Inputs and outputs
rotate over 3 buffer sets, as bench.py's do, so no launch re-reads or re-writes a buffer the Infinity Cache holds."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd.signals import lowpass_taps  # noqa: E402

ROUNDS = int(os.environ.get("ROUNDS", "4"))
REPS = int(os.environ.get("REPS", "30"))
SETTLE = int(os.environ.get("SETTLE", "0"))  # untimed launches before each timed block
f, u32, i32, p, sz, u64 = ctypes.c_float, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
SIGS = {
    "gsdrFirFC": [sz, p, sz, p, p, sz, i32, p],
    "gsdrFirFF": [sz, p, sz, p, p, sz, i32, p],
    "gsdrFmDemod": [f, f, f, f, u32, sz, p, sz, p, p, sz, i32, p],
    "gsdrAmDemod": [f, f, f, u32, sz, p, sz, p, p, sz, i32, p],
    "gsdrxFmDemodInt8": [f, f, f, f, u32, sz, p, sz, p, p, sz, i32, p],
    "gsdrxAmDemodInt8": [f, f, f, u32, sz, p, sz, p, p, sz, i32, p],
    "gsdrxFirFCInt8": [sz, p, sz, p, p, sz, i32, p],
    "gsdrxQpsk256ModulateAwgn": [p, p, u32, u32, f, u64, u64, i32, p],
    "gsdrxQpsk256ModulateAwgnDemodulate": [p, p, p, u32, u32, f, u64, u64, i32, p],
    "gsdrQpsk256Demodulate": [p, p, u32, u32, i32, p],
    "gsdrQpsk256InitConstellation": [u32, f, i32, p],
    "gsdrIirFF": [p, p, sz, p, p, p, p, sz, i32, p],
    "gsdrIirCC": [p, p, sz, p, p, p, p, sz, i32, p],
}


def load(path):
    lib = ctypes.CDLL(path)
    for n, a in SIGS.items():
        if hasattr(lib, n):  # (an older build may lack an entry point: its cases are skipped)
            getattr(lib, n).argtypes = a
            getattr(lib, n).restype = ctypes.c_int
    return lib


def main():
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + sys.argv[1:]
    L = [load(x) for x in libs]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(7)
    D, T, NO = 4, 127, 1 << 24
    NI = (NO - 1) * D + T
    taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    K = 3
    xs = [(torch.rand(2 * NI, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(K)]
    x8s = [torch.randint(-100, 100, (2 * NI,), dtype=torch.int8, device=dev, generator=g) for _ in range(K)]
    ycs = [torch.empty(NO, dtype=torch.complex64, device=dev) for _ in range(K)]
    yfs = [torch.empty(NO, dtype=torch.float32, device=dev) for _ in range(K)]
    n5 = 1 << 24
    t1 = torch.rand(63, device=dev, generator=g)  # config 1: 2^20 real outputs, 63 taps, D = 1
    x1 = torch.rand((1 << 20) + 62, device=dev, generator=g)
    y1 = torch.empty(1 << 20, device=dev)
    symss = [torch.randint(0, 256, (n5,), dtype=torch.uint8, device=dev, generator=g) for _ in range(K)]
    rxs = [torch.empty(n5, dtype=torch.complex64, device=dev) for _ in range(K)]
    decs = [torch.empty(n5, dtype=torch.uint8, device=dev) for _ in range(K)]
    from scipy import signal as sps

    bb, aa = (torch.tensor(v, dtype=torch.float32, device=dev) for v in sps.butter(4, 0.1))
    bb8, aa8 = (torch.tensor(v, dtype=torch.float32, device=dev) for v in sps.butter(8, 0.2))
    xis = [torch.rand(n5, device=dev, generator=g) for _ in range(4)]
    yis = [torch.empty_like(x) for x in xis]
    xics = [torch.rand(2 * n5, device=dev, generator=g).view(torch.complex64) for _ in range(4)]
    yics = [torch.empty_like(x) for x in xics]
    for lib in L:
        assert lib.gsdrQpsk256InitConstellation(0, 1.0, 0, st) == 0
    cases = {
        "gsdrFirFF1": lambda lib, k: lib.gsdrFirFF(1, t1.data_ptr(), 63, x1.data_ptr(), y1.data_ptr(), 1 << 20, 0, st),
        "gsdrFirFC": lambda lib, k: lib.gsdrFirFC(D, taps.data_ptr(), T, xs[k % K].data_ptr(), ycs[k % K].data_ptr(), NO, 0, st),
        "gsdrFmDemod": lambda lib, k: lib.gsdrFmDemod(1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T, xs[k % K].data_ptr(),
                                                      yfs[k % K].data_ptr(), NO - 1, 0, st),
        "gsdrAmDemod": lambda lib, k: lib.gsdrAmDemod(1e6, 0.0, 1e5, D, 0, taps.data_ptr(), T, xs[k % K].data_ptr(),
                                                      yfs[k % K].data_ptr(), NO, 0, st),
        "gsdrxFirFCInt8": lambda lib, k: lib.gsdrxFirFCInt8(D, taps.data_ptr(), T, x8s[k % K].data_ptr(), ycs[k % K].data_ptr(),
                                                            NO, 0, st),
        "gsdrxFmDemodInt8": lambda lib, k: lib.gsdrxFmDemodInt8(1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T,
                                                                x8s[k % K].data_ptr(), yfs[k % K].data_ptr(), NO - 1, 0, st),
        "gsdrxAmDemodInt8": lambda lib, k: lib.gsdrxAmDemodInt8(1e6, 0.0, 1e5, D, 0, taps.data_ptr(), T,
                                                                x8s[k % K].data_ptr(), yfs[k % K].data_ptr(), NO - 1, 0, st),
        "gsdrxQpsk256ModulateAwgn": lambda lib, k: lib.gsdrxQpsk256ModulateAwgn(symss[k % K].data_ptr(), rxs[k % K].data_ptr(), n5, 0,
                                                                                0.02, 0x5EED0005, 0, 0, st),
        "gsdrQpsk256Demodulate": lambda lib, k: lib.gsdrQpsk256Demodulate(rxs[k % K].data_ptr(), decs[k % K].data_ptr(), n5, 0, 0, st),
        # config 5's round trip: modulate + AWGN, then demodulate what it wrote
        "config5_round_trip": lambda lib, k: (lib.gsdrxQpsk256ModulateAwgn(symss[k % K].data_ptr(), rxs[k % K].data_ptr(), n5, 0, 0.02,
                                                                           0x5EED0005, 0, 0, st),
                                              lib.gsdrQpsk256Demodulate(rxs[k % K].data_ptr(), decs[k % K].data_ptr(), n5, 0, 0, st))[1],
        "config5_fused": lambda lib, k: lib.gsdrxQpsk256ModulateAwgnDemodulate(
            symss[k % K].data_ptr(), rxs[k % K].data_ptr(), decs[k % K].data_ptr(), n5, 0, 0.02, 0x5EED0005, 0, 0, st),
        "gsdrIirFF": lambda lib, k: lib.gsdrIirFF(bb.data_ptr(), aa.data_ptr(), 5, None, None, xis[k % 4].data_ptr(),
                                                  yis[k % 4].data_ptr(), n5, 0, st),
        "gsdrIirCC": lambda lib, k: lib.gsdrIirCC(bb.data_ptr(), aa.data_ptr(), 5, None, None, xics[k % 4].data_ptr(),
                                                  yics[k % 4].data_ptr(), n5, 0, st),
        "gsdrIirFF9": lambda lib, k: lib.gsdrIirFF(bb8.data_ptr(), aa8.data_ptr(), 9, None, None, xis[k % 4].data_ptr(),
                                                   yis[k % 4].data_ptr(), n5, 0, st),
        "gsdrIirCC9": lambda lib, k: lib.gsdrIirCC(bb8.data_ptr(), aa8.data_ptr(), 9, None, None, xics[k % 4].data_ptr(),
                                                   yics[k % 4].data_ptr(), n5, 0, st),
    }
    only = os.environ.get("CASES")
    res = {}
    for r in range(ROUNDS):
        for name, fn in cases.items():
            if only and name not in only.split(","):
                continue
            for li in [(r + x) % len(L) for x in range(len(L))]:  # the order rotates round by round
                lib = L[li]
                if name == "config5_fused" and not hasattr(lib, "gsdrxQpsk256ModulateAwgnDemodulate"):
                    continue
                for k in range(5 + SETTLE):  # SETTLE: sustained-clock timing like bench.py's (default: short bursts)
                    assert fn(lib, k) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for k in range(REPS):
                    fn(lib, k)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, li), []).append(e0.elapsed_time(e1) / REPS * 1e3)
    names = [os.path.relpath(x, ROOT) for x in libs]
    print(f"{'entry point':26s} " + " ".join(f"{n[:24]:>24s}" for n in names) + "   (min / median us)")
    for name in cases:
        if (name, 0) not in res:
            continue
        cols = []
        for li in range(len(L)):
            if (name, li) not in res:
                cols.append("-")
                continue
            v = sorted(res[(name, li)])
            cols.append(f"{v[0]:11.2f} / {v[len(v) // 2]:9.2f}")
        print(f"{name:26s} " + " ".join(f"{c:>24s}" for c in cols), flush=True)


if __name__ == "__main__":
    main()
