"""GPU parity: the int8 I/Q front end fused into the filters (gsdrxFirFCInt8, gsdrxFmDemodInt8,
gsdrxAmDemodInt8).

Contract (gsdr_ext.h): identical to gsdrInt8ToNormFloat (reference src/conversion.cu:26) over the
2*L components followed by the float entry point. Where both paths run the same kernel (even
decimation -> polyphase kernel; odd decimation > 1 -> generic kernel) the results are compared bit for
bit; everything is also checked against the C oracle (conversion, then FIR/chain) with the
normwise FIR bound and the wrapped-angle discriminator tolerance."""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, bound, normwise_err, wrapped_angle_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def iq8(n_samples, seed):
    return np.random.default_rng(seed).integers(-128, 128, 2 * n_samples, dtype=np.int8)


def as_complex(f):  # float32 interleaved pairs -> complex64
    return f.view(np.complex64)


def taps_for(T, seed=1):
    from gsdr_amd.signals import lowpass_taps

    return lowpass_taps(T) if T > 1 else np.array([0.75], np.float32)


def test_conversion_exhaustive_through_the_fir(cuda):
    from gsdr_amd import ops

    # every int8 value in both I and Q of the even samples; D = 2, one unit tap -> y[k] = conv(x[2k])
    v = np.arange(-128, 128, dtype=np.int8)
    x = np.zeros(2 * 2 * 256, np.int8)
    x[0::4], x[1::4] = v, v[::-1]
    y = host(ops.fir(dev(np.array([1.0], np.float32), cuda), dev(x, cuda), 2))
    want = as_complex(o.int8_to_float(x))[0::2]
    assert y.tobytes() == want.tobytes()


@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 16, 20, 24, 32, 40, 50, 64])
@pytest.mark.parametrize("T", [1, 8, 63, 127, 200])
def test_fir_int8_parity(cuda, D, T):
    from gsdr_amd import ops

    n = 3001 + 17 * D
    L = (n - 1) * D + T
    x8 = iq8(L, seed=D * 1000 + T)
    taps = taps_for(T)
    y = host(ops.fir(dev(taps, cuda), dev(x8, cuda), D, n))
    xf = as_complex(o.int8_to_float(x8))
    want = o.fir(taps, xf, D, n)
    assert normwise_err(y, want, bound(taps, xf, D, n)) <= FLOAT_TOL
    yf = host(ops.fir(dev(taps, cuda), dev(xf, cuda), D, n))
    if D == 4 and T <= 196:  # matrix-core kernel (gsdr_ext.h): the normwise bar against the float path
        assert normwise_err(y, yf, bound(taps, xf, D, n)) <= FLOAT_TOL
    else:  # same kernel shape as the float entry point -> bit-identical
        assert y.tobytes() == yf.tobytes()


@pytest.mark.parametrize("offset_bytes", [1, 2, 6])
def test_fir_int8_unaligned(cuda, offset_bytes):
    from gsdr_amd import ops

    D, T, n = 4, 127, 5000
    L = (n - 1) * D + T
    raw = iq8(L + 8, seed=offset_bytes)
    xt = dev(raw, cuda)[offset_bytes:offset_bytes + 2 * L]
    taps = taps_for(T)
    y = host(ops.fir(dev(taps, cuda), xt, D, n))
    xf = as_complex(o.int8_to_float(raw[offset_bytes:offset_bytes + 2 * L]))
    assert normwise_err(y, o.fir(taps, xf, D, n), bound(taps, xf, D, n)) <= FLOAT_TOL


@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 16, 20, 24, 32, 40, 50, 64])
def test_fm_am_int8_chains(cuda, D):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal

    fs, tune, chan, dhz, T, n0 = 1.0e6, 0.0, 1.0e5, 2.0e4, 127, 987_654_321
    n = 20_000
    x = fm_test_signal(n * D + T, noise=0.02, n0=n0)
    x8 = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
    xf = as_complex(o.int8_to_float(x8))
    taps = taps_for(T)
    td = dev(taps, cuda)
    fm = host(ops.fm_demod(dev(x8, cuda), td, fs, tune, chan, dhz, D, n0, n))
    g = fs / (2 * np.pi * dhz)
    assert wrapped_angle_err(fm, o.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, n), g) <= FLOAT_TOL
    fm_f = host(ops.fm_demod(dev(xf, cuda), td, fs, tune, chan, dhz, D, n0, n))
    # D = 4 runs on the matrix cores (NCO folded into complex taps): the parity bar, not bit identity
    exact = D != 4
    if exact:
        assert fm.tobytes() == fm_f.tobytes()
    else:
        assert wrapped_angle_err(fm, fm_f, g) <= FLOAT_TOL
    am = host(ops.am_demod(dev(x8, cuda), td, fs, tune, chan, D, n0, n))
    am_f = host(ops.am_demod(dev(xf, cuda), td, fs, tune, chan, D, n0, n))
    if exact:
        assert am.tobytes() == am_f.tobytes()
    assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, n))) <= 2 * FLOAT_TOL


def test_fir_int8_full_config(cuda):
    """BASELINE configs[1] shape (2^24 outputs, D = 4, T = 127) from int8 I/Q through the default path
    (the matrix-core kernel) and through variant 0 (packed VALU): variant 0 bit-identical to the float
    path on the converted samples (itself checked against the oracle elsewhere), the default within the
    normwise bar of it (test_fir_int8_mfma_full_config)."""
    from gsdr_amd import ops

    n, D, T = 1 << 24, 4, 127
    L = (n - 1) * D + T
    g = torch.Generator(device=cuda).manual_seed(5)
    x8 = torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=cuda, generator=g)
    taps = dev(taps_for(T), cuda)
    y0 = ops.fir_variant(0, taps, x8, D, n)
    xf = ops.int8_to_norm_float(x8).view(torch.complex64)
    yf = ops.fir(taps, xf, D, n)
    y = ops.fir(taps, x8, D, n)
    y41 = ops.fir_variant(41, taps, x8, D, n)
    torch.cuda.synchronize()
    assert torch.equal(y0.view(torch.float32), yf.view(torch.float32))
    assert torch.equal(y.view(torch.float32), y41.view(torch.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("offset_bytes", [2, 6])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 8, 13])
def test_fir_int8_shifted_staging_bit_identical(cuda, D, offset_bytes):
    """Odd-sample (2-byte) offsets take stage_tile's shifted word loads: outputs equal the aligned call's."""
    import torch
    from gsdr_amd import ops

    T, n = 127, 60000
    L = (n - 1) * D + T
    raw = iq8(L + 8, seed=D)
    taps = dev(taps_for(T), cuda)
    buf = dev(raw, cuda)
    aligned = torch.empty(2 * L + 16, dtype=torch.int8, device=buf.device)[:2 * L]
    aligned.copy_(buf[offset_bytes:offset_bytes + 2 * L])
    y0 = host(ops.fir(taps, aligned, D, n))
    y1 = host(ops.fir(taps, buf[offset_bytes:offset_bytes + 2 * L], D, n))
    assert y1.tobytes() == y0.tobytes()


@pytest.mark.parametrize("mode", ["fm_demod", "am_demod"])
@pytest.mark.parametrize("offset_bytes", [2, 4, 6])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 8])
def test_chain_int8_misaligned_bit_identical(cuda, mode, D, offset_bytes):
    """FM / AM chains from int8 I/Q at 2-, 4- and 6-byte offsets (odd-sample offsets take the shifted
    staging, whose first pair starts one sample early and is mixed with the odd-index NCO phasor; FM at
    odd D also has the two-output tile overlap): bit-identical to the same samples at an aligned
    address, with the same firstSampleIndex."""
    from gsdr_amd import ops

    T, n, n0 = 127, 30000, 12345
    L = n * D + T
    raw = iq8(L + 8, seed=100 + D)
    taps = dev(taps_for(T), cuda)
    buf = dev(raw, cuda)
    aligned = torch.empty(2 * L + 16, dtype=torch.int8, device=buf.device)[:2 * L]
    aligned.copy_(buf[offset_bytes:offset_bytes + 2 * L])
    args = (1.0e6, 0.0, 1.0e5, 2.0e4) if mode == "fm_demod" else (1.0e6, 0.0, 1.0e5)
    fn = getattr(ops, mode)
    y0 = host(fn(aligned, taps, *args, D, n0, n))
    y1 = host(fn(buf[offset_bytes:offset_bytes + 2 * L], taps, *args, D, n0, n))
    assert y1.tobytes() == y0.tobytes()


# Matrix-core int8 FIR (gsdrxFirFCInt8Variant 40, k_fir_i8_mfma): exact fp16 samples, taps scaled by a
# power of two and split into two fp16 parts, fp32 accumulation in the matrix core's order -> the
# normwise bar against the oracle (not bit-identical to the ascending-order float path).
@pytest.mark.parametrize("variant", [40, 41])
@pytest.mark.parametrize("T", [1, 2, 8, 63, 127, 128, 196])
@pytest.mark.parametrize("N", [1, 2, 2047, 2048, 2049, 50000 + 3])
def test_fir_int8_mfma_parity(cuda, variant, T, N):
    from gsdr_amd import ops

    D = 4
    L = (N - 1) * D + T
    x8 = iq8(L, seed=T * 7 + N)
    rng = np.random.default_rng(T)
    taps = (rng.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    y = host(ops.fir_variant(variant, dev(taps, cuda), dev(x8, cuda), D, N))
    xf = as_complex(o.int8_to_float(x8))
    assert normwise_err(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("offset_bytes", [2, 6])
def test_fir_int8_mfma_unaligned(cuda, offset_bytes):
    """Input off 16-byte alignment takes the per-sample staging loads; same bar."""
    from gsdr_amd import ops

    D, T, N = 4, 127, 30000
    L = (N - 1) * D + T
    raw = iq8(L + 8, seed=offset_bytes)
    xt = dev(raw, cuda)[offset_bytes:offset_bytes + 2 * L]
    taps = taps_for(T)
    y = host(ops.fir_variant(41, dev(taps, cuda), xt, D, N))
    xf = as_complex(o.int8_to_float(raw[offset_bytes:offset_bytes + 2 * L]))
    assert normwise_err(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL


def test_fir_int8_mfma_tap_dynamic_range(cuda):
    """Taps spanning 1e-30 .. 1 (and signed zeros): the scaled two-part split keeps the normwise bar."""
    from gsdr_amd import ops

    D, T, N = 4, 127, 20000
    L = (N - 1) * D + T
    x8 = iq8(L, seed=3)
    rng = np.random.default_rng(4)
    taps = (rng.standard_normal(T) * 10.0 ** rng.uniform(-30, 0, T)).astype(np.float32)
    taps[::17] = -0.0
    y = host(ops.fir_variant(41, dev(taps, cuda), dev(x8, cuda), D, N))
    xf = as_complex(o.int8_to_float(x8))
    assert normwise_err(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL
    tiny = (taps * np.float32(1e-30)).astype(np.float32)  # max |t| near the float range's bottom
    y = host(ops.fir_variant(41, dev(tiny, cuda), dev(x8, cuda), D, N))
    assert normwise_err(y, o.fir(tiny, xf, D, N), bound(tiny, xf, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("bad", [np.inf, -np.inf, np.nan])
def test_fir_int8_mfma_nonfinite_taps(cuda, bad):
    """Taps that are not all finite take the exact ascending loop: bit-identical to the oracle."""
    from gsdr_amd import ops

    D, T, N = 4, 63, 5000
    L = (N - 1) * D + T
    x8 = iq8(L, seed=9)
    taps = taps_for(T).copy()
    taps[10] = bad
    y = host(ops.fir_variant(41, dev(taps, cuda), dev(x8, cuda), D, N))
    want = o.fir(taps, as_complex(o.int8_to_float(x8)), D, N)
    assert y.view(np.uint64).tobytes() == want.view(np.uint64).tobytes()


def test_fir_int8_mfma_full_config(cuda):
    """BASELINE configs[1] shape from int8 I/Q (2^24 outputs): against the float path on the converted
    samples (itself checked against the oracle), normwise."""
    from gsdr_amd import ops

    n, D, T = 1 << 24, 4, 127
    L = (n - 1) * D + T
    g = torch.Generator(device=cuda).manual_seed(5)
    x8 = torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=cuda, generator=g)
    taps = dev(taps_for(T), cuda)
    y = ops.fir(taps, x8, D, n)  # the default: matrix-core kernel
    xf = ops.int8_to_norm_float(x8).view(torch.complex64)
    yf = ops.fir(taps, xf, D, n)
    # normwise bound per output, S_k = sum_i |t_i| |x_{kD+i}| (helpers.bound), as a strided
    # cross-correlation on the device
    ax = xf.abs().double().view(1, 1, L)
    at = taps.abs().double().view(1, 1, T)
    bnd = torch.nn.functional.conv1d(ax, at, stride=D).view(-1)[:n]
    err = (y.to(torch.complex128) - yf.to(torch.complex128)).abs()
    assert float((err / bnd.clamp_min(1e-30)).max()) <= FLOAT_TOL


# Matrix-core int8 FM / AM chains (D = 4, k_chain_i8_mfma): NCO folded into complex taps, normwise parity
# with the oracle's chains at tile boundaries (FM tiles stride 1023 outputs, AM 1024), short and odd
# lengths, every supported tap count, large first-sample indices and tuning offsets.
@pytest.mark.parametrize("T", [1, 2, 33, 127, 132])
@pytest.mark.parametrize("N", [1, 2, 1022, 1023, 1024, 2046, 2047, 2048, 4095, 30_001])
def test_chain_int8_mfma_parity(cuda, T, N):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal

    D, n0 = 4, 4_000_000_123
    # the carrier (+0.1 fs) lands at 0 Hz: tune - chan = -1e5 (an out-of-band channel filters noise only,
    # whose angles are ill-conditioned for any summation order)
    fs, tune, chan, dhz = 1.0e6, 3.3e4, 1.33e5, 2.0e4
    x = fm_test_signal(N * D + T, noise=0.05, n0=n0)
    x8 = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
    xf = as_complex(o.int8_to_float(x8))
    taps = taps_for(T)
    td = dev(taps, cuda)
    g = fs / (2 * np.pi * dhz)
    fm = host(ops.fm_demod(dev(x8, cuda), td, fs, tune, chan, dhz, D, n0, N))
    assert wrapped_angle_err(fm, o.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, N), g) <= FLOAT_TOL
    am = host(ops.am_demod(dev(x8, cuda), td, fs, tune, chan, D, n0, N))
    assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, N))) <= 2 * FLOAT_TOL


@pytest.mark.parametrize("bad", [np.inf, -np.inf, np.nan])
def test_chain_int8_mfma_nonfinite_taps(cuda, bad):
    """Non-finite taps: the exact per-output chain, so the non-finite pattern is the oracle's."""
    from gsdr_amd import ops

    D, T, N, n0 = 4, 127, 5000, 7
    x8 = iq8(N * D + T, seed=9)
    xf = as_complex(o.int8_to_float(x8))
    taps = taps_for(T)
    taps[40] = bad
    td = dev(taps, cuda)
    am = host(ops.am_demod(dev(x8, cuda), td, 1.0e6, 0.0, 1.0e5, D, n0, N))
    ref = o.am_demod(xf, taps, 1.0e6, 0.0, 1.0e5, D, n0, N)
    assert np.array_equal(np.isnan(am), np.isnan(ref))
    fm = host(ops.fm_demod(dev(x8, cuda), td, 1.0e6, 0.0, 1.0e5, 2.0e4, D, n0, N))
    reff = o.fm_demod(xf, taps, 1.0e6, 0.0, 1.0e5, 2.0e4, D, n0, N)
    assert np.array_equal(np.isfinite(fm), np.isfinite(reff))


def test_chain_int8_mfma_config3_size(cuda):
    """Config 3's shape (2^24 outputs) from int8 I/Q: the matrix-core FM chain against the float chain on
    the converted samples over every output (the oracle itself is checked on windows elsewhere)."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    D, T, N, n0 = 4, 127, 1 << 24, 99
    L = N * D + T
    # config 3's signal (constant-envelope FM at +0.1 fs plus AWGN sigma 0.05), quantised to int8 I/Q
    idx = torch.arange(n0, n0 + L, dtype=torch.float64, device=cuda)
    ph = 2 * np.pi * 0.1 * idx + 20.0 * torch.sin(2 * np.pi * 0.001 * idx)
    del idx
    x = torch.view_as_real(torch.polar(torch.ones_like(ph), ph).to(torch.complex64)).reshape(-1)
    del ph
    g8 = torch.Generator(device=cuda).manual_seed(11)
    x += torch.randn(2 * L, dtype=torch.float32, device=cuda, generator=g8) * 0.05
    x8 = torch.clamp(torch.round(x * 100), -128, 127).to(torch.int8)
    del x
    xf = ops.int8_to_norm_float(x8).view(torch.complex64)
    td = torch.from_numpy(lowpass_taps(T)).to(cuda)
    fs, tune, chan, dhz = 1.0e6, 0.0, 1.0e5, 2.0e4
    g = fs / (2 * np.pi * dhz)
    fm8 = ops.fm_demod(x8, td, fs, tune, chan, dhz, D, n0, N)
    fmf = ops.fm_demod(xf, td, fs, tune, chan, dhz, D, n0, N)
    d = torch.remainder(fm8.double() - fmf.double() + np.pi * g, 2 * np.pi * g) - np.pi * g
    assert float(d.abs().max()) / (np.pi * g) <= FLOAT_TOL
    am8 = ops.am_demod(x8, td, fs, tune, chan, D, n0, N)
    amf = ops.am_demod(xf, td, fs, tune, chan, D, n0, N)
    assert float((am8 - amf).abs().max()) <= 2 * FLOAT_TOL
