"""Shared parity metrics for the tests."""
from __future__ import annotations

import numpy as np

# north_star: float paths within 1e-5 relative, evaluated normwise (pointwise relative error is not
# attainable by any reordered fp32 sum: two correct orders differ by up to 2.9e-5 pointwise).
FLOAT_TOL = 1e-5


def bound(taps, x, D, N, k0=0, k1=None):
    """S_k = sum_i |t_i| |x_{kD+i}| in float64, for k in [k0, k1)."""
    k1 = N if k1 is None else k1
    T = taps.size
    at = np.abs(taps.astype(np.complex128))
    ax = np.abs(x.astype(np.complex128))
    # valid correlation then decimation, only over the needed span
    lo, hi = k0 * D, (k1 - 1) * D + T
    c = np.correlate(ax[lo:hi], at, mode="valid")
    return c[::D][: k1 - k0]


def normwise_err(got, want, s):
    """max_k |got_k - want_k| / S_k (S_k floored to avoid 0/0 on all-zero windows)."""
    got = np.asarray(got).astype(np.complex128)
    want = np.asarray(want).astype(np.complex128)
    s = np.maximum(np.asarray(s, dtype=np.float64), 1e-30)
    return float(np.max(np.abs(got - want) / s)) if got.size else 0.0


def wrapped_angle_err(got, want, g):
    """max |remainder(got - want, 2 pi g)| / (pi g): discriminator outputs are angles scaled by g."""
    d = np.remainder(np.asarray(got, np.float64) - np.asarray(want, np.float64) + np.pi * g, 2 * np.pi * g) - np.pi * g
    return float(np.max(np.abs(d)) / (np.pi * abs(g))) if d.size else 0.0
