"""Deterministic synthetic inputs and filter design shared by tests, smoke() and bench.py.

All generators are numpy (host) so the CPU oracle and the GPU see the same bytes; nothing here
calls the library.
"""
from __future__ import annotations

import numpy as np

__all__ = ["lowpass_taps", "uniform_iq", "fm_test_signal", "random_bytes"]


def lowpass_taps(num_taps: int, cutoff: float = 0.1) -> np.ndarray:
    """Hamming-windowed sinc low-pass, cutoff in cycles/sample (fraction of fs), unit DC gain, float32."""
    n = np.arange(num_taps, dtype=np.float64) - (num_taps - 1) / 2.0
    h = 2.0 * cutoff * np.sinc(2.0 * cutoff * n)
    if num_taps > 1:
        h *= 0.54 - 0.46 * np.cos(2.0 * np.pi * np.arange(num_taps) / (num_taps - 1))
    h /= h.sum()
    return h.astype(np.float32)


def uniform_iq(n: int, seed: int = 0x5EED) -> np.ndarray:
    """I/Q i.i.d. uniform in [-1, 1), complex64."""
    rng = np.random.default_rng(seed)
    v = rng.random(2 * n, dtype=np.float32) * 2.0 - 1.0
    return v.view(np.complex64)


def fm_test_signal(n: int, fs: float = 1.0e6, carrier: float = 0.1, tone: float = 0.001, deviation: float = 0.02,
                   noise: float = 0.05, seed: int = 0x5EED, n0: int = 0) -> np.ndarray:
    """Constant-envelope FM: carrier offset `carrier`*fs, message tone `tone`*fs, peak deviation
    `deviation`*fs, amplitude 1, plus AWGN of std `noise` per axis."""
    idx = np.arange(n0, n0 + n, dtype=np.float64)
    beta = deviation / tone
    phase = 2.0 * np.pi * carrier * idx + beta * np.sin(2.0 * np.pi * tone * idx)
    x = np.exp(1j * phase)
    if noise > 0.0:
        rng = np.random.default_rng(seed)
        x = x + noise * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x.astype(np.complex64)


def random_bytes(n: int, seed: int = 0x5EED) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
