"""GPU parity: gsdrFmDemod / gsdrAmDemod (fused NCO + FIR + decimation + demod) vs the C oracle.

Reference: src/fm.cu:21-69, 181-218; src/am.cu:21-81; NCO re-specified in SURVEY.md App. A.3
(the reference's k_AdjustFrequency never returns its value, adjustFrequency.cu:56).
Bars: FM -- wrapped-angle error <= 1e-5 of full scale (pi * g) on a constant-envelope signal;
AM -- absolute error <= 1e-5 (outputs in [-1, 1]); the FIR stage itself is checked normwise via AM.
"""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, wrapped_angle_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu

FS, TUNE, CHAN, DEV = 1.0e6, 0.0, 1.0e5, 2.0e4


def fm_gain():
    return float(np.float32(FS) / (np.float32(2.0) * np.float32(np.pi) * np.float32(DEV)))


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


@pytest.mark.parametrize("n0", [0, 987654321, (1 << 32) + 5])
@pytest.mark.parametrize("T", [1, 31, 127])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 16, 20, 24, 32, 40, 50, 64])
def test_fm_demod_parity(cuda, D, T, n0):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    N = 2 * 4096 + 11
    x = fm_test_signal(N * D + T, fs=FS, noise=0.05, seed=D + T, n0=n0 % (1 << 20))
    taps = lowpass_taps(T, 0.1 if T > 1 else 0.5)
    out = ops.fm_demod(dev(x, cuda), dev(taps, cuda), FS, TUNE, CHAN, DEV, D, n0, N)
    torch.cuda.synchronize()
    ref = o.fm_demod(x, taps, FS, TUNE, CHAN, DEV, D, n0, N)
    assert wrapped_angle_err(out.cpu().numpy(), ref, fm_gain()) <= FLOAT_TOL


@pytest.mark.parametrize("n0", [0, (1 << 32) + 5])
@pytest.mark.parametrize("T", [1, 31, 127])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 16, 20, 24, 32, 40, 50, 64])
def test_am_demod_parity(cuda, D, T, n0):
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps, uniform_iq

    N = 2 * 4096 + 11
    x = (0.7 * uniform_iq((N - 1) * D + T, seed=D * T)).astype(np.complex64)
    taps = lowpass_taps(T, 0.1 if T > 1 else 0.5)
    out = ops.am_demod(dev(x, cuda), dev(taps, cuda), FS, TUNE, CHAN, D, n0, N)
    torch.cuda.synchronize()
    ref = o.am_demod(x, taps, FS, TUNE, CHAN, D, n0, N)
    assert float(np.max(np.abs(out.cpu().numpy() - ref))) <= FLOAT_TOL


def test_nco_against_golden_increment(cuda):
    from gsdr_amd import ops

    assert ops.nco_phase_increment(FS, TUNE, CHAN) == o.nco_inc(FS, TUNE, CHAN)


@pytest.mark.parametrize("D", [4, 1, 3, 5])
def test_fm_streaming_chunks_equal_monolithic(cuda, D):
    """Streaming contract (fm.h:26, firstSampleIndex fm.h:48): K chunked calls with numLowPassTaps of
    overlap reproduce one call bit for bit -- the NCO phase is a function of the absolute index and
    each FIR output is computed by the same arithmetic wherever its tile falls. Odd D puts chunks at
    8-byte-aligned addresses (shifted staging, odd-start NCO pairs)."""
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    T, N = 127, 30000
    x = dev(fm_test_signal(N * D + T, fs=FS, seed=3), cuda)
    taps = dev(lowpass_taps(T, 0.1), cuda)
    whole = ops.fm_demod(x, taps, FS, TUNE, CHAN, DEV, D, 1000, N)
    parts, m = [], 0
    for n in (7000, 1, 12345, N - 7000 - 1 - 12345):
        xs = x[m * D:(m + n) * D + T]
        parts.append(ops.fm_demod(xs, taps, FS, TUNE, CHAN, DEV, D, 1000 + m * D, n))
        m += n
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), whole)


def test_fm_pure_tone_known_answer(cuda):
    """A noiseless FM carrier at a constant offset f from the channel discriminates to the constant
    g * 2 pi f D'/fs where the discriminator sees decimated samples: arg step = 2 pi f D / fs."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    D, T, N = 4, 127, 5000
    f = 1.0e5 + 2000.0  # 2 kHz above the channel centre
    n = np.arange(N * D + T)
    x = np.exp(2j * np.pi * f / FS * n).astype(np.complex64)
    out = ops.fm_demod(dev(x, cuda), dev(lowpass_taps(T, 0.1), cuda), FS, TUNE, CHAN, DEV, D, 0, N)
    torch.cuda.synchronize()
    want = fm_gain() * 2 * np.pi * 2000.0 * D / FS
    assert np.max(np.abs(out.cpu().numpy() - want)) < 1e-4 * abs(want) + 1e-6


def test_fm_full_config(cuda):
    """BASELINE config 3: NCO + 127-tap FIR (D = 4) + FM over 67,108,987 samples; oracle spot checks."""
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    D, T, N = 4, 127, (1 << 24) - 1
    L = N * D + T
    x_np = fm_test_signal(L, fs=FS, noise=0.05, seed=0x5EED)
    taps = lowpass_taps(T, 0.1)
    x = dev(x_np, cuda)
    out = ops.fm_demod(x, dev(taps, cuda), FS, TUNE, CHAN, DEV, D, 0, N)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for m0 in (0, N // 3, N - 3000):
        m1 = m0 + 3000
        ref = o.fm_demod(x_np, taps, FS, TUNE, CHAN, DEV, D, 0, N, m0, m1)
        assert wrapped_angle_err(got[m0:m1], ref[m0:m1], fm_gain()) <= FLOAT_TOL
    assert np.all(np.isfinite(got))
