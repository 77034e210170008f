"""GPU: multi-channel chains (gsdrxFmDemodMulti / gsdrxAmDemodMulti).
Each channel must be bit-identical to the single-channel entry point with its own channel frequency
(and deviation), for float and int8 I/Q input, for channel counts that fill one launch, span two
(17 > 16) and for shapes that fall back to per-channel launches (odd decimation, very long filters);
one channel is also checked against the C oracle."""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, wrapped_angle_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu

FS, TUNE = 1.0e6, 0.0


def signal(n, n0, int8, seed=1):
    from gsdr_amd.signals import fm_test_signal

    # three FM carriers at -0.2, +0.1, +0.3 fs
    x = sum(fm_test_signal(n, carrier=c, noise=0.0, seed=seed + i, n0=n0) for i, c in enumerate((-0.2, 0.1, 0.3)))
    x = (x / 3 + 0.02 * (np.random.default_rng(seed).standard_normal(n) + 1j * np.random.default_rng(seed + 9)
                          .standard_normal(n))).astype(np.complex64)
    if int8:
        return np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
    return x


@pytest.mark.parametrize("D", [2, 3, 4, 8])
@pytest.mark.parametrize("C", [1, 4, 17])
@pytest.mark.parametrize("int8", [False, True])
def test_multi_equals_single(cuda, D, C, int8):
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    T, n0, N = 127, 77_777_777, 20_011
    x = torch.from_numpy(signal(N * D + T, n0, int8)).to(cuda)
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    chans = [float(v) for v in np.linspace(-0.35, 0.35, C) * FS]
    devs = [2.0e4 + 1000.0 * c for c in range(C)]
    fm = ops.fm_demod_multi(x, taps, FS, TUNE, chans, devs, D, n0, N)
    am = ops.am_demod_multi(x, taps, FS, TUNE, chans, D, n0, N)
    # int8: the single-channel gsdrx*Int8 defaults (at D = 4 the matrix-core chain, which the multi-channel
    # entry points then run per channel)
    for c in range(C):
        f1 = ops.fm_demod(x, taps, FS, TUNE, chans[c], devs[c], D, n0, N)
        a1 = ops.am_demod(x, taps, FS, TUNE, chans[c], D, n0, N)
        assert torch.equal(fm[c], f1), c
        assert torch.equal(am[c], a1), c


def test_multi_long_filter_falls_back(cuda):
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    T, D, N = 1201, 4, 5000
    x = torch.from_numpy(signal(N * D + T, 0, False)).to(cuda)
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    chans, devs = [-2.0e5, 1.0e5, 3.0e5], [2.0e4] * 3
    fm = ops.fm_demod_multi(x, taps, FS, TUNE, chans, devs, D, 0, N)
    for c in range(3):
        assert torch.equal(fm[c], ops.fm_demod(x, taps, FS, TUNE, chans[c], devs[c], D, 0, N))


def test_multi_channel_vs_oracle(cuda):
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    T, D, N, n0 = 127, 4, 30_000, 5
    xh = signal(N * D + T, n0, False)
    taps_h = lowpass_taps(T)
    x, taps = torch.from_numpy(xh).to(cuda), torch.from_numpy(taps_h).to(cuda)
    chans, devs = [-2.0e5, 1.0e5, 3.0e5], [2.0e4, 2.0e4, 2.0e4]
    fm = ops.fm_demod_multi(x, taps, FS, TUNE, chans, devs, D, n0, N).cpu().numpy()
    g = FS / (2 * np.pi * 2.0e4)
    for c in range(3):
        want = o.fm_demod(xh, taps_h, FS, TUNE, chans[c], devs[c], D, n0, N)
        assert wrapped_angle_err(fm[c], want, g) <= FLOAT_TOL


def test_multi_validation(cuda):
    from gsdr_amd import abi

    st = torch.cuda.current_stream(cuda).cuda_stream
    assert abi.lib.gsdrxFmDemodMulti(1e6, 0.0, None, None, 0, 4, 0, None, 0, 0, None, None, 10, cuda.index, st) == 0
    assert abi.lib.gsdrxFmDemodMulti(1e6, 0.0, None, None, 2, 4, 0, None, 0, 0, None, None, 10, cuda.index, st) != 0
