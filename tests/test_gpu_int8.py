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

from helpers import FLOAT_TOL, bound, fm_conditioned_err, normwise_err, normwise_err_strict, wrapped_angle_err
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
    assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, n))) <= FLOAT_TOL


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


# Matrix-core int8 FIR (gsdrxFirFCInt8Variant 40 / 41, k_fir_i8_mfma): exact bf16 samples, taps scaled by a
# power of two and split exactly into three bf16 parts, fp32 accumulation in the matrix core's order -> the
# normwise bar against the oracle (not bit-identical to the ascending-order float path).
@pytest.mark.parametrize("variant", [40, 41, 42, 43, 44, 45, 46])
@pytest.mark.parametrize("T", [1, 2, 8, 63, 127, 128, 196])
@pytest.mark.parametrize("N", [1, 2, 2047, 2048, 2049, 50000 + 3])
def test_fir_int8_mfma_parity(cuda, variant, T, N):
    from gsdr_amd import ops

    if variant >= 42 and T > 132:
        pytest.skip("tile-size sweep variants cover T <= 132 (6 K steps)")

    D = 4
    L = (N - 1) * D + T
    x8 = iq8(L, seed=T * 7 + N)
    rng = np.random.default_rng(T)
    taps = (rng.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    y = host(ops.fir_variant(variant, dev(taps, cuda), dev(x8, cuda), D, N))
    xf = as_complex(o.int8_to_float(x8))
    assert normwise_err(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("N", [100_001, 2_000_003])
def test_fir_int8_mfma_tile_shapes_bit_identical(cuda, N):
    """512-output tiles with 3 or 4 workgroups a CU and one or two tiles in flight (variants 43-46, several
    rounds of tiles a workgroup at 2 M outputs) give the default's outputs bit for bit: an output's summation
    order depends only on its 16-output block."""
    from gsdr_amd import ops

    D, T = 4, 127
    x8 = dev(iq8((N - 1) * D + T, seed=N), cuda)
    taps = dev((np.random.default_rng(5).standard_normal(T) / np.sqrt(T)).astype(np.float32), cuda)
    want = ops.fir_variant(41, taps, x8, D, N).view(torch.float32)
    for variant in (42, 43, 44, 45, 46):
        assert torch.equal(ops.fir_variant(variant, taps, x8, D, N).view(torch.float32), want), variant


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


@pytest.mark.parametrize("scale", [1.0, 1e-30, 1e-36, 1e30])
def test_fir_int8_mfma_tap_dynamic_range(cuda, scale):
    """Taps spanning 30 decades (and signed zeros), scaled so that max |t| sits anywhere from the bottom of
    the float range (1e-36: outputs in the subnormal range) to 1e30: the exact three-part split and the
    two-step output scale keep the normwise bar, with no floor on S_k."""
    from gsdr_amd import ops

    D, T, N = 4, 127, 20000
    L = (N - 1) * D + T
    x8 = iq8(L, seed=3)
    rng = np.random.default_rng(4)
    taps = (rng.standard_normal(T) * 10.0 ** rng.uniform(-30, 0, T) * scale).astype(np.float32)
    taps[::17] = -0.0
    xf = as_complex(o.int8_to_float(x8))
    for variant in (40, 41):
        y = host(ops.fir_variant(variant, dev(taps, cuda), dev(x8, cuda), D, N))
        assert normwise_err_strict(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL


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
    assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, N))) <= FLOAT_TOL


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
    assert float((am8 - amf).abs().max()) <= FLOAT_TOL


# ------------------------------------------------------------------------------------------------
# Sparse inputs through the decimation-4 matrix-core defaults (gsdrxFirFCInt8, gsdrxFmDemodInt8,
# gsdrxAmDemodInt8). The reference's own known-answer case is an impulse through the FIR
# (tests/test_fir.cpp:191-206); on a sparse window one tap carries an output's whole normwise bound, so
# every tap, however small next to the largest (the ~1e-18 sinc zero crossings of lowpass_taps), must be
# exact. Impulses sit 131 samples apart (> T, odd): each output's window holds at most one, and over the
# train every tap position meets every phase mod 4 and every row of the 16-output summation blocks.
# ------------------------------------------------------------------------------------------------
def sparse_taps(kind, T=127):
    from gsdr_amd.signals import lowpass_taps

    if kind == "lowpass":
        return lowpass_taps(T, 0.1)  # 24 of 127 taps below 1e-17 of the largest
    rng = np.random.default_rng(21)
    return (rng.standard_normal(T) * 10.0 ** rng.uniform(-25, 0, T)).astype(np.float32)  # 25 decades


def impulse_train(L, spacing, seed, start=3):
    rng = np.random.default_rng(seed)
    x8 = np.zeros(2 * L, np.int8)
    pos = np.arange(start, L, spacing)
    v = rng.integers(-128, 128, (pos.size, 2)).astype(np.int8)
    v[v[:, 0] == 0, 0] = -128  # nonzero I, except where Q alone is kept below
    which = rng.integers(0, 3, pos.size)  # 0: I and Q, 1: I only, 2: Q only
    v[which == 1, 1] = 0
    v[which == 2, 0] = 0
    v[(which == 2) & (v[:, 1] == 0), 1] = 127
    x8[2 * pos], x8[2 * pos + 1] = v[:, 0], v[:, 1]
    return x8


def bursts(L, seed):
    """Bursts of 1-40 random samples between zero runs of 50-3000 samples."""
    rng = np.random.default_rng(seed)
    x8 = np.zeros(2 * L, np.int8)
    p = int(rng.integers(0, 200))
    while p < L:
        n = int(rng.integers(1, 41))
        x8[2 * p:2 * min(L, p + n)] = rng.integers(-128, 128, 2 * (min(L, p + n) - p)).astype(np.int8)
        p += n + int(rng.integers(50, 3001))
    return x8


@pytest.mark.parametrize("taps_kind", ["lowpass", "decades"])
@pytest.mark.parametrize("signal", ["impulses", "bursts"])
@pytest.mark.parametrize("variant", [-1, 40])
def test_fir_int8_mfma_sparse(cuda, taps_kind, signal, variant):
    from gsdr_amd import ops

    D, T, N = 4, 127, 30_000
    L = (N - 1) * D + T
    x8 = impulse_train(L, 131, seed=5) if signal == "impulses" else bursts(L, seed=6)
    taps = sparse_taps(taps_kind, T)
    td, xd = dev(taps, cuda), dev(x8, cuda)
    y = host(ops.fir(td, xd, D, N) if variant < 0 else ops.fir_variant(variant, td, xd, D, N))
    xf = as_complex(o.int8_to_float(x8))
    assert normwise_err_strict(y, o.fir(taps, xf, D, N), bound(taps, xf, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("taps_kind", ["lowpass", "decades"])
@pytest.mark.parametrize("signal", ["impulses", "bursts"])
def test_chain_int8_mfma_sparse(cuda, taps_kind, signal):
    """FM and AM chains on sparse int8 windows. AM: the absolute bar on the envelope. FM: single-impulse
    windows are well conditioned (|y| = S), and where one of the two FIR outputs of a discriminator pair
    is a zero window the reference's atan2f(+-0, +-0) value must come out exactly; bursts are held to the
    conditioned bar (helpers.fm_conditioned_err)."""
    from gsdr_amd import ops

    D, T, N, n0 = 4, 127, 30_000, 3_000_000_017
    fs, tune, chan, dhz = 1.0e6, 3.3e4, 1.33e5, 2.0e4
    L = N * D + T
    x8 = impulse_train(L, 137, seed=7) if signal == "impulses" else bursts(L, seed=8)
    taps = sparse_taps(taps_kind, T)
    td, xd = dev(taps, cuda), dev(x8, cuda)
    xf = as_complex(o.int8_to_float(x8))
    am = host(ops.am_demod(xd, td, fs, tune, chan, D, n0, N))
    assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, N))) <= FLOAT_TOL
    g = fs / (2 * np.pi * dhz)
    fm = host(ops.fm_demod(xd, td, fs, tune, chan, dhz, D, n0, N))
    want = o.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, N)
    y_ref = o.chain_fir(xf, taps, fs, tune, chan, D, n0, N + 1)
    assert fm_conditioned_err(fm, want, y_ref, bound(taps, xf, D, N + 1), g) <= 1.0
    if signal == "impulses" and taps_kind == "lowpass":  # no discriminator product below fp32's normal range
        assert wrapped_angle_err(fm, want, g) <= FLOAT_TOL


@pytest.mark.parametrize("what", ["zero_input", "zero_taps", "silent_gaps"])
def test_int8_mfma_zero_windows(cuda, what):
    """Silence and zero taps: FIR outputs exactly 0, AM exactly -1, FM the reference's atan2f(+-0, +-0)
    value bit for bit (the folded NCO's rotation must not be added to an exactly zero
    discriminator product); an FM signal with silent gaps holds the conditioned bar around the gaps."""
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps

    D, T, N, n0 = 4, 127, 20_000, 987_654_321
    fs, tune, chan, dhz = 1.0e6, 0.0, 1.0e5, 2.0e4
    L = N * D + T
    taps = lowpass_taps(T, 0.1)
    x = fm_test_signal(L, noise=0.02, n0=n0)
    x8 = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
    if what == "zero_input":
        x8[:] = 0
    elif what == "zero_taps":
        taps = np.zeros(T, np.float32)
    else:
        rng = np.random.default_rng(9)
        for p in rng.integers(0, L - 3000, 40):
            x8[2 * p:2 * (p + int(rng.integers(200, 3000)))] = 0
    td, xd = dev(taps, cuda), dev(x8, cuda)
    xf = as_complex(o.int8_to_float(x8))
    y = host(ops.fir(td, xd, D, N - 1))
    am = host(ops.am_demod(xd, td, fs, tune, chan, D, n0, N))
    fm = host(ops.fm_demod(xd, td, fs, tune, chan, dhz, D, n0, N))
    want_fm = o.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, N)
    g = fs / (2 * np.pi * dhz)
    if what != "silent_gaps":
        assert np.all(y.view(np.float32) == 0.0)
        assert np.all(am == -1.0)
        assert fm.tobytes() == want_fm.tobytes()
    else:
        assert normwise_err_strict(y, o.fir(taps, xf, D, N - 1), bound(taps, xf, D, N - 1)) <= FLOAT_TOL
        assert np.max(np.abs(am - o.am_demod(xf, taps, fs, tune, chan, D, n0, N))) <= FLOAT_TOL
        y_ref = o.chain_fir(xf, taps, fs, tune, chan, D, n0, N + 1)
        assert fm_conditioned_err(fm, want_fm, y_ref, bound(taps, xf, D, N + 1), g) <= 1.0


@pytest.mark.parametrize("kind", ["fir", "fm", "am"])
def test_int8_mfma_shift_invariant(cuda, kind):
    """The matrix-core kernels' summation blocks follow the absolute output index: a call over a sub-range
    (chains: with the matching firstSampleIndex; FIR: through the streaming object, whose launches pass the
    output index) reproduces the whole call's outputs bit for bit, at every offset mod 16 and at input and
    output pointers of every alignment."""
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    D, T, N, n0 = 4, 127, 9_000, 1_234_567
    fs, tune, chan, dhz = 1.0e6, 0.0, 1.0e5, 2.0e4
    L = N * D + T
    x = fm_test_signal(L, noise=0.02, n0=n0)
    x8 = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
    xd = dev(x8, cuda)
    td = dev(lowpass_taps(T, 0.1), cuda)
    if kind == "fir":
        whole = host(ops.fir(td, xd, D, N))
        # chunks in samples: every input-pointer alignment, output index mod 16 and seam/main split
        for chunk in (3, 5, 64, 37, 1001, 4093):
            s = Stream("fir", td, D, fs, tune, chan, dhz, first_sample_index=0, int8=True)
            parts, pos = [], 0
            while pos < L:
                m = min(chunk, L - pos)
                parts.append(s.process(xd[2 * pos:2 * (pos + m)]).clone())
                pos += m
            s.close()
            got = host(torch.cat(parts))[:N]
            assert got.tobytes() == whole.tobytes(), chunk
        return
    fn = ops.fm_demod if kind == "fm" else ops.am_demod
    args = (fs, tune, chan, dhz) if kind == "fm" else (fs, tune, chan)
    whole = host(fn(xd, td, *args, D, n0, N))
    for k0 in list(range(0, 17)) + [31, 1000, 1023, 4111]:
        n = N - k0 - 5
        out = torch.empty(n + 1, dtype=torch.float32, device=cuda)[1:]  # 4 bytes off 8-byte alignment
        src = xd[2 * D * k0:]
        if k0 % 3 == 1:  # input 2 bytes off 8-byte alignment: the per-sample staging loads
            buf = torch.empty(src.numel() + 2, dtype=torch.int8, device=cuda)[2:]
            buf.copy_(src)
            src = buf
        got = host(fn(src, td, *args, D, n0 + D * k0, n, out=out))
        assert got.tobytes() == whole[k0:k0 + n].tobytes(), k0


@pytest.mark.parametrize("kind", ["fir", "fm", "am"])
@pytest.mark.parametrize("case", ["inf_tap", "nan_tap", "impulses"])
def test_int8_stream_one_launch(cuda, kind, case):
    """int8 streams at decimation 4 run one matrix-core launch a call: the seam outputs read their samples
    before the chunk from the history buffer and the same launch writes the next history. Chunked ==
    monolithic bit for bit, for taps that are not finite (the exact per-output fallback, which reads the
    history as well) and for an impulse train, over chunk sizes from 1 sample up."""
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    D, T, n0 = 4, 127, 77_777_777
    fs, tune, chan, dhz = 1.0e6, 0.0, 1.0e5, 2.0e4
    L = 40_000 + 3
    taps = lowpass_taps(T, 0.1).copy()
    if case == "impulses":
        x8 = impulse_train(L, 131, seed=11)
    else:
        x = fm_test_signal(L, noise=0.02, n0=n0)
        x8 = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
        taps[40] = np.inf if case == "inf_tap" else np.nan
    xd, td = dev(x8, cuda), dev(taps, cuda)
    if kind == "fir":
        want = ops.fir(td, xd, D)
    elif kind == "fm":
        want = ops.fm_demod(xd, td, fs, tune, chan, dhz, D, n0)
    else:
        want = ops.am_demod(xd, td, fs, tune, chan, D, n0)
    s = Stream(kind, td, D, fs, tune, chan, dhz, first_sample_index=n0, int8=True)
    parts, pos = [], 0
    rng = np.random.default_rng(len(kind) + len(case))
    while pos < L:
        m = min(L - pos, int(rng.choice([1, 2, 3, 5, T - 1, T + 7, 333, 4096, 17001])))
        parts.append(s.process(xd[2 * pos:2 * (pos + m)]).clone())
        pos += m
    s.close()
    got = torch.cat(parts)
    torch.cuda.synchronize()
    assert got.numel() == want.numel()
    assert got.cpu().numpy().tobytes() == want.cpu().numpy().tobytes()


def test_fir_int8_mfma_tile_shapes_bit_identical(cuda):
    """Calls with fewer large tiles than two rounds of workgroup slots take 512-output tiles instead of
    2,048-output ones (fir_dispatch.hpp launch_i8_mfma_ns). The summation order is per 16-output block,
    aligned to the absolute output index, so the shapes agree bit for bit: config 2's int8 channel in one
    call (large tiles) against the same channel through the streaming object in 64 chunks (small tiles),
    and against the oracle's normwise bar."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps
    from gsdr_amd.stream import Stream

    D, T = 4, 127
    L = 67_108_987
    N = (L - T) // D + 1
    g = torch.Generator(device=cuda).manual_seed(64)
    xd = torch.randint(-128, 128, (2 * L,), dtype=torch.int8, device=cuda, generator=g)
    td = dev(lowpass_taps(T, 0.1), cuda)
    whole = ops.fir(td, xd, D, N)
    s = Stream("fir", td, D, 1.0, 0.0, 0.0, 1.0, first_sample_index=0, int8=True)
    cs = L // 64 + 1  # odd: chunk starts alternate between 2-byte and 4-byte alignment
    parts, pos = [], 0
    while pos < L:
        m = min(cs, L - pos)
        parts.append(s.process(xd[2 * pos:2 * (pos + m)]).clone())
        pos += m
    s.close()
    got = torch.cat(parts)[:N]
    assert torch.equal(got.view(torch.float32), whole.view(torch.float32))
    # a window of the whole call against the oracle (the bar the header states)
    k0, n = 12_345_677, 4096
    raw = xd[2 * k0 * D:2 * ((k0 + n - 1) * D + T)].cpu().numpy()
    xf = as_complex(o.int8_to_float(raw))
    taps = lowpass_taps(T, 0.1)
    assert normwise_err(host(whole[k0:k0 + n]), o.fir(taps, xf, D, n), bound(taps, xf, D, n)) <= FLOAT_TOL
