"""CPU: the IIR oracle (oracle_iir, float64 sequential recursion with history; include/gsdr/iir.h)
pinned against scipy.signal.lfilter with the initial state from scipy.signal.lfiltic -- an
independent implementation of the same difference equation -- and against closed-form known answers.
The reference's own kernel is not a recursive filter (state reset every 8 samples, src/iir.cu:121-127)
and its complex variant does not compile, so there are no reference outputs to pin to."""
import numpy as np
import pytest
from scipy import signal

from oracle import oracle as o


def design(kind, order):
    if kind == "butter":
        b, a = signal.butter(order, 0.1)
    else:  # cascade of real poles inside the unit circle: stable at any order
        rng = np.random.default_rng(order)
        poles = rng.uniform(-0.8, 0.8, order)
        a = np.poly(poles)
        b = rng.uniform(-0.5, 0.5, order + 1)
    return b.astype(np.float32), a.astype(np.float32)


@pytest.mark.parametrize("kind,order", [("butter", 1), ("butter", 2), ("butter", 4), ("butter", 6), ("poles", 12),
                                        ("poles", 31)])
@pytest.mark.parametrize("cplx", [False, True])
def test_oracle_matches_scipy_lfilter(kind, order, cplx):
    b, a = design(kind, order)
    rng = np.random.default_rng(order + cplx)
    n = 3000
    x = rng.standard_normal(n).astype(np.float32)
    if cplx:
        x = (x + 1j * rng.standard_normal(n)).astype(np.complex64)
    xh = (rng.standard_normal(order) * (1 + 1j if cplx else 1)).astype(x.dtype)
    yh = (rng.standard_normal(order) * (1 + 1j if cplx else 1)).astype(x.dtype)
    y, xh2, yh2 = o.iir(b, a, x, xh, yh)
    b64, a64 = b.astype(np.float64), a.astype(np.float64)
    zi = signal.lfiltic(b64, a64, yh.astype(np.complex128 if cplx else np.float64),
                        xh.astype(np.complex128 if cplx else np.float64))
    want, _ = signal.lfilter(b64, a64, x.astype(np.complex128 if cplx else np.float64), zi=zi)
    scale = max(1.0, float(np.max(np.abs(want))))
    assert np.max(np.abs(y - want)) / scale < 1e-6
    # returned history = last K-1 samples, newest first
    assert np.array_equal(xh2, x[::-1][:order])
    assert np.array_equal(yh2, y[::-1][:order])


def test_oracle_history_continues_the_recursion():
    b, a = design("butter", 4)
    x = np.random.default_rng(1).standard_normal(1000).astype(np.float32)
    whole, _, _ = o.iir(b, a, x)
    xh = np.zeros(4, np.float32)
    yh = np.zeros(4, np.float32)
    parts = []
    for lo, hi in ((0, 1), (1, 3), (3, 400), (400, 1000)):  # including chunks shorter than K-1
        y, xh, yh = o.iir(b, a, x[lo:hi], xh, yh)
        parts.append(y)
    assert np.max(np.abs(np.concatenate(parts) - whole)) < 1e-6


def test_ref_first_order_impulse_response():
    # the reference test's default design (tests/test_iir.cpp:125-126): b = {c, c}, a = {1, -(1-c)};
    # impulse response: y0 = c, y1 = c(2-c), y_n = (1-c) y_{n-1}
    c = np.float32(0.1)
    b = np.array([c, c], np.float32)
    a = np.array([1.0, -(1.0 - c)], np.float32)
    x = np.zeros(50, np.float32)
    x[0] = 1.0
    y, _, _ = o.iir(b, a, x)
    want = np.empty(50)
    want[0], want[1] = c, c * (2 - c)
    for k in range(2, 50):
        want[k] = (1 - c) * want[k - 1]
    assert np.allclose(y, want, rtol=1e-6, atol=1e-7)
