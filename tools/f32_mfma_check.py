"""Development check of the float matrix-core FIR (gsdrxFirFCVariant 42-44, fir_f32_mfma.hpp): normwise
parity with the oracle on random, wide-dynamic-range, impulse-with-tiny-tail and non-finite inputs,
then config-2 timing interleaved with the packed-VALU default (variant 0), HIP events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps, uniform_iq  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def check(v, taps, x, D=4, name=""):
    dev = torch.device("cuda", 0)
    n = (x.size - taps.size) // D + 1
    y = ops.fir_variant(v, torch.from_numpy(taps).to(dev), torch.from_numpy(x).to(dev), D, n).cpu().numpy()
    ref = orc.fir(taps, x, D, n)
    s = orc.fir_bound_fc(taps, x, D, n)
    fin_ref = np.isfinite(ref.real) & np.isfinite(ref.imag)
    fin = np.isfinite(y.real) & np.isfinite(y.imag)
    mism = int(np.sum(fin != fin_ref))
    f = fin & fin_ref
    err = np.maximum(np.abs(y.real - ref.real), np.abs(y.imag - ref.imag))[f] / np.maximum(s[f], 1e-38)
    e = float(err.max()) if err.size else 0.0
    ok = mism == 0 and e <= 1e-5
    print(f"v{v} {name:12s} n={n} finite-mismatch={mism} max normwise err={e:.3e} {'OK' if ok else 'FAIL'}")
    return ok


def main():
    variants = [int(a) for a in sys.argv[1:]] or [42, 43, 44]
    if os.environ.get("TIME_ONLY"):
        return time_only(variants)
    rng = np.random.default_rng(7)
    T = 127
    taps = lowpass_taps(T)
    n = 200_000
    L = (n - 1) * 4 + T
    cases = {}
    cases["uniform"] = uniform_iq(L, seed=3)
    wide = uniform_iq(L, seed=4) * np.repeat(10.0 ** rng.uniform(-30, 30, L // 50 + 1), 50)[:L]
    cases["wide-range"] = wide.astype(np.complex64)
    imp = np.zeros(L, np.complex64)
    pos = rng.integers(0, L, 400)
    imp[pos] = 1.0 + 1.0j
    for d in range(1, 60):
        q = np.minimum(pos + d, L - 1)
        imp[q] += np.complex64(1e-12 * (0.9 ** d) * (1 - 0.5j))
    cases["impulse-tail"] = imp
    nf = uniform_iq(L, seed=5)
    nf[rng.integers(0, L, 20)] = np.inf
    nf[rng.integers(0, L, 20)] = np.nan
    nf[rng.integers(0, L, 20)] = complex(-np.inf, 1.0)
    cases["non-finite"] = nf
    cases["zeros"] = np.zeros(L, np.complex64)
    den = uniform_iq(L, seed=6) * np.float32(1e-39)
    cases["denormal"] = den.astype(np.complex64)
    ok = True
    for v in variants:
        for k, x in cases.items():
            ok &= check(v, taps, x, name=k)
        ok &= check(v, lowpass_taps(33), cases["uniform"][:100_003], name="T=33 odd n")
    print("PARITY", "OK" if ok else "FAIL")
    time_only(variants)


def time_only(variants):
    T = 127
    taps = lowpass_taps(T)
    dev = torch.device("cuda", 0)
    n, D = 1 << 24, 4
    L = (n - 1) * D + T
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.rand(2 * L, device=dev, generator=g).mul_(2).sub_(1).view(torch.complex64)
    td = torch.from_numpy(taps).to(dev)
    out = torch.empty(n, dtype=torch.complex64, device=dev)
    allv = [0] + variants
    for v in allv:
        for _ in range(300):
            ops.fir_variant(v, td, x, D, n, out=out)
    torch.cuda.synchronize()
    for rep in range(4):
        line = []
        for v in allv:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                ops.fir_variant(v, td, x, D, n, out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 200 * 1e3
            line.append(f"v{v} {us:7.2f} us ({(8 * L + 8 * n) / us / 1e3:6.0f} GB/s)")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
