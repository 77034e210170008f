#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz.

The reference (kernrj/gsdr) is CUDA-only and cannot be built or run in this image (no nvcc, no CUDA
runtime, and its build needs a CMake-generated gsdr_export.h), and its gtest suite holds no numeric
fixtures. The fixtures here are therefore an INDEPENDENT restatement of the reference's semantics in
numpy float64 (FIR, NCO, chains, discriminators) and exact integer / IEEE-float32 arithmetic (QPSK,
QPSK256), written from the reference source (cited per case) -- not from the C oracle -- so that the
oracle can be checked against something it does not share code with. Inputs are stored with the
expected outputs. Re-run with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from gsdr_amd.signals import fm_test_signal, lowpass_taps, random_bytes, uniform_iq  # noqa: E402


def save(name, **arrays):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)


def fir64(taps, x, D, N):
    """reference src/fir.cu:49-71 in float64: y[k] = sum_i x[kD+i] t[i]."""
    t = taps.astype(np.complex128 if np.iscomplexobj(taps) else np.float64)
    xx = x.astype(np.complex128 if np.iscomplexobj(x) else np.float64)
    T = t.size
    return np.array([np.dot(xx[k * D:k * D + T], t) for k in range(N)])


def bound64(taps, x, D, N):
    T = taps.size
    at, ax = np.abs(taps.astype(np.complex128)), np.abs(x.astype(np.complex128))
    return np.array([np.dot(ax[k * D:k * D + T], at) for k in range(N)])


def nco_inc(fs, tune, chan):
    df = np.float32(np.float32(tune) - np.float32(chan))
    scaled = (float(df) / float(np.float32(fs))) * 4294967296.0
    return int(np.int64(np.round(np.fmod(scaled, 4294967296.0)))) & 0xFFFFFFFF


def nco64(x, n0, inc):
    n = np.arange(x.size, dtype=np.uint64) + np.uint64(n0)
    p = ((n & np.uint64(0xFFFFFFFF)) * np.uint64(inc)) & np.uint64(0xFFFFFFFF)
    return x.astype(np.complex128) * np.exp(2j * np.pi * p.astype(np.float64) / 2.0 ** 32)


def main():
    # ---- FIR: 4 type combos x D in {1, 4} x T in {8, 63, 127} (fir.cu:26-171)
    for tt in ("FF", "FC", "CC", "CF"):
        for D in (1, 4):
            for T in (8, 63, 127):
                N = 257
                L = (N - 1) * D + T
                seed = 1000 + 10 * D + T
                rng = np.random.default_rng(seed)
                taps = lowpass_taps(T)
                if tt[0] == "C":
                    taps = (taps + 1j * rng.standard_normal(T).astype(np.float32) * 0.05).astype(np.complex64)
                x = uniform_iq(L, seed) if tt[1] == "C" else (rng.random(L, dtype=np.float32) * 2 - 1)
                save(f"fir_{tt}_D{D}_T{T}", taps=taps, x=x, D=D, N=N, y=fir64(taps, x, D, N),
                     s=bound64(taps, x, D, N))

    # ---- NCO + FM / AM chains (fm.cu:21-69, am.cu:21-50, re-specified in SURVEY.md App. A.3-A.4)
    fs, tune, chan, dev = 1.0e6, 0.0, 1.0e5, 2.0e4
    for n0 in (0, 123456789):
        D, T, N = 4, 127, 300
        x = fm_test_signal(N * D + T, fs=fs, noise=0.05, seed=7, n0=n0)
        taps = lowpass_taps(T, 0.1)
        inc = nco_inc(fs, tune, chan)
        z = nco64(x, n0, inc)
        y = fir64(taps, z, D, N + 1)
        g = float(np.float32(fs) / (np.float32(2.0) * np.float32(np.pi) * np.float32(dev)))
        fm = g * np.angle(y[1:] * np.conj(y[:-1]))
        am = 2.0 * np.clip(np.abs(y[:N]), 0.0, 1.0) - 1.0
        save(f"chain_n0_{n0}", x=x, taps=taps, fs=fs, tune=tune, chan=chan, dev=dev, D=D, N=N, n0=n0, inc=inc,
             y=y, fm=fm, am=am, g=g)

    # ---- quad demods and magnitude (quad_demod.cu:23-54, magnitude.cu:20-28)
    x = uniform_iq(1025, 11)
    xd = x.astype(np.complex128)
    save("quad", x=x, gain=0.5, fm=0.5 * np.angle(xd[1:] * np.conj(xd[:-1])),
         am=2.0 * np.clip(np.abs(xd), 0, 1) - 1.0, mag=np.abs(xd))

    # ---- QPSK (qpsk.cu:108-146, 221-268): integer-exact
    n = 1001
    bits = random_bytes((n + 3) // 4, 21)
    a = np.float32(0.75)
    s = np.array([(bits[k >> 2] >> (2 * (k & 3))) & 3 for k in range(n)], dtype=np.uint8)
    sym = np.where(s & 1, -a, a).astype(np.float32) + 1j * np.where(s & 2, -a, a).astype(np.float32)
    noisy = (sym + 0.3 * (np.random.default_rng(22).standard_normal(n) +
                          1j * np.random.default_rng(23).standard_normal(n))).astype(np.complex64)
    noisy[:4] = [0.0 + 0.0j, -0.0 + 0.0j, complex(0.0, -0.0), -1.0 + 0.0j]
    dec = ((noisy.real < 0) | np.isnan(noisy.real)).astype(np.uint8) | \
        (((noisy.imag < 0) | np.isnan(noisy.imag)).astype(np.uint8) << 1)
    prev = np.full((n + 3) // 4, 0xFF, dtype=np.uint8)
    packed = prev.copy()
    for k in range(n):
        sh = 2 * (k & 3)
        packed[k >> 2] = (int(packed[k >> 2]) & (~(3 << sh) & 0xFF)) | (int(dec[k]) << sh)
    save("qpsk", bits=bits, n=n, a=a, symbols=sym.astype(np.complex64), noisy=noisy, prev=prev, demod=packed)

    # ---- QPSK256 (qpsk256.cu:29-71 tables; 154-195 demod): float32 IEEE arithmetic in reference order
    amp = np.float32(1.0)
    i = np.arange(16, dtype=np.float32)
    lv = ((i - np.float32(7.5)) / np.float32(7.5)) * amp
    rect = (np.repeat(lv, 16) + 1j * np.tile(lv, 16)).astype(np.complex64)
    pts, radii = [1, 8, 16, 24, 32, 40, 48, 56], [0.0, 0.3, 0.6, 0.85, 1.1, 1.35, 1.6, 1.85]
    circ = []
    for c in range(8):
        r = np.float32(radii[c]) * amp
        for p in range(pts[c]):
            ang = np.float32(np.float32(np.float32(2.0) * np.float32(np.pi)) * np.float32(p)) / np.float32(pts[c]) \
                + np.float32(np.float32(c) * np.float32(0.5))
            circ.append(complex(r * np.float32(np.cos(np.float64(ang))), r * np.float32(np.sin(np.float64(ang)))))
    while len(circ) < 256:
        k = len(circ)
        ang = np.float32(np.float32(np.float32(2.0) * np.float32(np.pi)) * np.float32(k)) / np.float32(256.0)
        r = amp * np.float32(0.95)
        circ.append(complex(r * np.float32(np.cos(np.float64(ang))), r * np.float32(np.sin(np.float64(ang)))))
    circ = np.array(circ, dtype=np.complex64)
    syms = random_bytes(4096, 31)
    rng = np.random.default_rng(32)
    for name, tab, sig in (("rect", rect, 0.05), ("circ", circ, 0.01)):
        tx = tab[syms]
        rx = (tx + sig * (rng.standard_normal(syms.size) + 1j * rng.standard_normal(syms.size))).astype(np.complex64)
        rx[:3] = [complex(np.nan, 0.0), complex(np.inf, 1.0), complex(1e30, -1e30)]
        dx = rx.real[:, None].astype(np.float32) - tab.real[None, :].astype(np.float32)
        dy = rx.imag[:, None].astype(np.float32) - tab.imag[None, :].astype(np.float32)
        with np.errstate(invalid="ignore", over="ignore"):
            d = (dx * dx + dy * dy).astype(np.float32)
        d = np.where(np.isnan(d), np.float32(np.inf), d)
        best = np.argmin(d, axis=1).astype(np.uint8)
        allinf = np.all(np.isinf(d), axis=1)
        best[allinf] = 0  # strict '<' against +inf never fires
        save(f"qpsk256_{name}", table=tab, symbols=syms, tx=tx, rx=rx, demod=best)

    elementwise()


def elementwise():
    """reference src/add_const.cu:20-42, multiply.cu:20-27, magnitude.cu:30-36, conversion.cu:20-27,
    trig.cu:20-75 with the operator semantics of src/cuComplexOperatorOverloads.cuh:25-56. numpy float32
    arithmetic rounds each operation (no contraction), which is the build's contract for the exact maps;
    hypot and cos/sin come from float64 and are compared within a tolerance."""
    rng = np.random.default_rng(0xE1E)
    n = 1000
    f32 = np.float32
    x = rng.uniform(-10, 10, n).astype(f32)
    x[:6] = [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf]
    y = rng.uniform(-10, 10, n).astype(f32)
    xc = (rng.uniform(-10, 10, n) + 1j * rng.uniform(-10, 10, n)).astype(np.complex64)
    yc = (rng.uniform(-10, 10, n) + 1j * rng.uniform(-10, 10, n)).astype(np.complex64)
    cf, cc = f32(3.14), np.complex64(1.5 - 2.5j)
    xr, xi, yr, yi = xc.real, xc.imag, yc.real, yc.imag
    add_ff = (cf + x).astype(f32)
    add_cc = ((cc.real + xr) + 1j * (cc.imag + xi)).astype(np.complex64)
    add_cf = ((xr + cf) + 1j * xi).astype(np.complex64)            # real part only
    add_fc = ((cc.real + x) + 1j * np.full(n, cc.imag, f32)).astype(np.complex64)
    mul_cc = ((xr * yr - xi * yi) + 1j * (xr * yi + xi * yr)).astype(np.complex64)
    mul_ff = (x * y).astype(f32)
    mul_cf = ((xr * y) + 1j * (xi * y)).astype(np.complex64)
    m64 = np.hypot(xr.astype(np.float64), xi.astype(np.float64))
    a2m = (xc.astype(np.complex128) / m64 * (2.5 + m64)).astype(np.complex64)
    i8 = np.arange(-128, 128, dtype=np.int8)
    conv = np.maximum(f32(-1.0), i8.astype(f32) / f32(127.0)).astype(f32)
    phi0, phi1, nc = f32(-1.3), f32(40.0), 1000
    step = f32((phi1 - phi0) / np.float64(nc))  # float subtraction, double division (trig.cu:55)
    th = (np.arange(nc, dtype=np.float64) * np.float64(step) + np.float64(phi0)).astype(f32)
    cos_c = (np.cos(th.astype(np.float64)) + 1j * np.sin(th.astype(np.float64))).astype(np.complex64)
    save("elementwise", x=x, y=y, xc=xc, yc=yc, cf=np.array([cf]), cc=np.array([cc]), add_ff=add_ff,
         add_cc=add_cc, add_cf=add_cf, add_fc=add_fc, mul_cc=mul_cc, mul_ff=mul_ff, mul_cf=mul_cf,
         a2m_c=np.array([f32(2.5)]), a2m=a2m, abs=np.abs(x).astype(f32), i8=i8, conv=conv,
         phi=np.array([phi0, phi1]), cos_c=cos_c)


if __name__ == "__main__":
    main()
    print("golden fixtures written to", HERE)
