"""GPU parity on non-finite and signed-zero samples: every FIR / FM / AM kernel shape sums exactly the
T products the reference sums (fir.cu:29-31, 58-60: the tap loop stops at T-1), so an Inf or NaN
sample only reaches the outputs whose true window holds it.

The tiled cores round T up to whole tap chunks; an output that came out non-finite is recomputed
from the staged tile without the padding products (fir_engine.hpp, "Exact zero-padding semantics").
Bars: the NaN pattern, the Inf pattern and the sign of every infinite or zero output equal the
oracle's bit for bit; finite outputs meet the usual normwise bar. Streaming and multi-channel calls
stay bit-identical to one monolithic single-channel call on such inputs."""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, bound, normwise_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu

FS, TUNE, CHAN, DEV = 1.0e6, 0.0, 1.0e5, 2.0e4


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def poison(x, seed, runs_of_zero=True):
    """Sprinkle +-Inf and NaN components into a float view of x, plus runs of -0 / +0 samples."""
    f = x.view(np.float32)
    rng = np.random.default_rng(seed)
    n = f.size
    for val, k in ((np.inf, 3), (-np.inf, 3), (np.nan, 3)):
        f[rng.integers(0, n, k)] = val
    if runs_of_zero:
        for z in (-0.0, 0.0):
            s = int(rng.integers(0, max(1, n - 600)))
            f[s:s + 600] = z
    # a lone non-finite value in the very last sample (reached only by the last outputs' windows)
    f[-1] = np.inf
    return x


def make(tt, T, L, seed):
    rng = np.random.default_rng(seed)
    taps = (rng.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    if tt in ("CC", "CF"):
        taps = (taps + 1j * (rng.standard_normal(T) / np.sqrt(T))).astype(np.complex64)
    real_in = tt in ("FF", "CF")
    x = (rng.random(L * (1 if real_in else 2), dtype=np.float32) * 2 - 1)
    if not real_in:
        x = x.view(np.complex64)
    return taps, poison(x, seed)


def assert_same_specials(got, want):
    g = np.ascontiguousarray(got).view(np.float32)
    w = np.ascontiguousarray(want).view(np.float32)
    assert np.array_equal(np.isnan(g), np.isnan(w)), "NaN pattern"
    inf = np.isinf(w)
    assert np.array_equal(np.isinf(g), inf), "Inf pattern"
    assert np.array_equal(g[inf], w[inf]), "Inf signs"
    z = w == 0
    assert np.all(g[z] == 0) and np.array_equal(np.signbit(g[z]), np.signbit(w[z])), "zero signs"


def finite_rows(y):
    y = np.asarray(y)
    return np.isfinite(y.real) & np.isfinite(y.imag) if np.iscomplexobj(y) else np.isfinite(y)


@pytest.mark.parametrize("T", [5, 100, 127, 128])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 8, 9, 13, 16, 32, 50, 200])
@pytest.mark.parametrize("tt", ["FC", "FF", "CC", "CF"])
def test_fir_nonfinite_matches_oracle(cuda, tt, D, T):
    from gsdr_amd import ops

    N = 4096 + 517
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=D * 131 + T)
    y = ops.fir(dev(taps, cuda), dev(x, cuda), D, N).cpu().numpy()
    ref = o.fir(taps, x, D, N)
    assert_same_specials(y, ref)
    ok = finite_rows(ref)
    assert normwise_err(y[ok], ref[ok], bound(taps, x, D, N)[ok]) <= FLOAT_TOL


@pytest.mark.parametrize("variant", [0, 1, 3, 4, 5, 7, 8, 9, 10, 11, 13, 14, 24, 28])
def test_fir_variants_nonfinite(cuda, variant):
    from gsdr_amd import ops

    N, D, T = 20000 + 3, 4, 127
    taps, x = make("FC", T, (N - 1) * D + T, seed=variant)
    y = ops.fir_variant(variant, dev(taps, cuda), dev(x, cuda), D, N).cpu().numpy()
    ref = o.fir(taps, x, D, N)
    assert_same_specials(y, ref)
    ok = finite_rows(ref)
    if variant in (7, 13):  # ascending-order kernels: bit-identical to the oracle
        assert np.array_equal(y.view(np.uint64), ref.view(np.uint64))
    assert normwise_err(y[ok], ref[ok], bound(taps, x, D, N)[ok]) <= FLOAT_TOL


def test_fir_all_negative_zero_window(cuda):
    """Windows of -0 samples: every product is a signed zero and the sum starts from +0
    (zero<OUT_T>(), fir.cu:43, 66), so the output is +0 for every tap sign."""
    from gsdr_amd import ops

    N, D, T = 3000, 4, 127
    taps, _ = make("FC", T, 1, seed=3)
    x = np.zeros((N - 1) * D + T, np.complex64)
    x.view(np.float32)[:] = -0.0
    y = ops.fir(dev(taps, cuda), dev(x, cuda), D, N).cpu().numpy().view(np.float32)
    assert np.all(y == 0) and not np.any(np.signbit(y))


@pytest.mark.parametrize("T", [100, 127])
@pytest.mark.parametrize("D", [1, 3, 4, 8, 9, 16])
@pytest.mark.parametrize("mode", ["fm", "am"])
def test_chain_nonfinite_matches_oracle(cuda, mode, D, T):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    N, n0 = 4096 + 517, 987654321
    x = poison(fm_test_signal(N * D + T, noise=0.05, seed=D + T), seed=D * 7 + T, runs_of_zero=False)
    taps = lowpass_taps(T)
    if mode == "fm":
        y = ops.fm_demod(dev(x, cuda), dev(taps, cuda), FS, TUNE, CHAN, DEV, D, n0, N).cpu().numpy()
        ref = o.fm_demod(x, taps, FS, TUNE, CHAN, DEV, D, n0, N)
        g = float(np.float32(FS) / (np.float32(2.0) * np.float32(np.pi) * np.float32(DEV)))
        ok = np.isfinite(ref)
        d = np.remainder(y[ok].astype(np.float64) - ref[ok] + np.pi * g, 2 * np.pi * g) - np.pi * g
        assert float(np.max(np.abs(d))) / (np.pi * g) <= FLOAT_TOL
    else:
        y = ops.am_demod(dev(x, cuda), dev(taps, cuda), FS, TUNE, CHAN, D, n0, N).cpu().numpy()
        ref = o.am_demod(x, taps, FS, TUNE, CHAN, D, n0, N)
        ok = np.isfinite(ref)
        assert float(np.max(np.abs(y[ok] - ref[ok]))) <= FLOAT_TOL
    assert np.array_equal(np.isnan(y), np.isnan(ref))
    assert np.array_equal(np.isinf(y), np.isinf(ref))
    assert ok.sum() > N // 2  # the poisoned samples reach only their own windows


@pytest.mark.parametrize("D", [2, 4, 8])
def test_multi_channel_nonfinite_equals_single(cuda, D):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    N, T = 9000, 127
    x = dev(poison(fm_test_signal(N * D + T, seed=D), seed=D, runs_of_zero=False), cuda)
    taps = dev(lowpass_taps(T), cuda)
    chans, devs = [1.0e5, -2.5e5], [2.0e4, 3.0e4]
    multi = ops.fm_demod_multi(x, taps, FS, TUNE, chans, devs, D, 0, N)
    for c in range(2):
        single = ops.fm_demod(x, taps, FS, TUNE, chans[c], devs[c], D, 0, N)
        assert multi[c].cpu().numpy().tobytes() == single.cpu().numpy().tobytes()


@pytest.mark.parametrize("kind", ["fir", "fm", "am"])
@pytest.mark.parametrize("D", [1, 4, 9])
def test_stream_nonfinite_chunked_equals_monolithic(cuda, kind, D):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    T, n0, L = 127, 123456789, 60_000 + 3 * D
    x = dev(poison(fm_test_signal(L, noise=0.02, seed=D), seed=D + 1, runs_of_zero=False), cuda)
    taps = dev(lowpass_taps(T), cuda)
    if kind == "fir":
        want = ops.fir(taps, x, D)
    elif kind == "fm":
        want = ops.fm_demod(x, taps, FS, TUNE, CHAN, DEV, D, n0)
    else:
        want = ops.am_demod(x, taps, FS, TUNE, CHAN, D, n0)
    s = Stream(kind, taps, D, FS, TUNE, CHAN, DEV, first_sample_index=n0)
    parts, pos = [], 0
    rng = np.random.default_rng(D)
    while pos < L:
        m = min(L - pos, int(rng.choice([1, 5, T - 1, T + 7, 3000, 17000])))
        parts.append(s.process(x[pos:pos + m]).clone())
        pos += m
    s.close()
    got = torch.cat(parts)
    assert got.cpu().numpy().tobytes() == want.cpu().numpy().tobytes()
