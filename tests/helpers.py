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


def normwise_err_strict(got, want, s):
    """max_k |got_k - want_k| / S_k with no floor: an output whose window contributes nothing (S_k = 0)
    must match exactly (returns inf otherwise). For tap sets near the bottom of the float range and for
    sparse inputs, where S_k itself is tiny or zero."""
    got = np.asarray(got).astype(np.complex128)
    want = np.asarray(want).astype(np.complex128)
    s = np.asarray(s, dtype=np.float64)
    d = np.abs(got - want)
    if np.any(d[s == 0] != 0):
        return float("inf")
    pos = s > 0
    return float(np.max(d[pos] / s[pos])) if np.any(pos) else 0.0


def fm_conditioned_err(got, want, y_ref, s, g, eps=2e-6):
    """FM discriminator error relative to its conditioning: the wrapped angle error of output k divided by
    the angle the fp32 evaluation itself cannot resolve, with y the oracle's FIR outputs (N + 1) and S their
    normwise bounds:
      * a pair with a zero window (S_k = 0 or S_{k+1} = 0): the discriminator product is exactly zero and
        the reference's atan2f(+-0, +-0) value (0 or +-pi, from the signs) must come out: bar 1e-5 pi;
      * otherwise max(1e-5 pi, eps (S_k/|y_k| + S_{k+1}/|y_{k+1}|) + 8 * 2^-149 / (|y_k| |y_{k+1}|)) rad: a
        window that cancels to a small |y| makes any fp32 summation order's angle uncertain by ~eps S/|y|,
        and a product y_{k+1} conj(y_k) below fp32's normal range keeps only its subnormal absolute
        precision (2^-149 a component) in the reference as here.
    Returns the max ratio (<= 1 passes)."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    d = np.abs(np.remainder(got - want + np.pi * g, 2 * np.pi * g) - np.pi * g) / abs(g)
    ay = np.abs(np.asarray(y_ref).astype(np.complex128))
    s = np.asarray(s, np.float64)
    zero_pair = (s[:-1] == 0) | (s[1:] == 0)
    prod = ay[:-1] * ay[1:]
    with np.errstate(divide="ignore", invalid="ignore"):
        kappa = s / ay  # S > 0 with |y| = 0: unbounded
        allowed = eps * (kappa[:-1] + kappa[1:]) + 8.0 * 2.0 ** -149 / prod
    allowed = np.where(zero_pair, 1e-5 * np.pi, np.maximum(1e-5 * np.pi, np.nan_to_num(allowed, nan=np.inf)))
    return float(np.max(d / allowed)) if d.size else 0.0
