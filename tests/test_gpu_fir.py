"""GPU parity: gsdrFir{FC,FF,CC,CF} through the C ABI vs the C oracle (reference src/fir.cu:26-171).

Bar (north_star): normwise error max_k |y_gpu - y_cpu| / sum_i |t_i||x_{kD+i}| <= 1e-5.
Named after the reference's tests/test_fir.cpp cases where one corresponds.
"""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, bound, normwise_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu

TYPES = {"FC": (np.float32, np.complex64), "FF": (np.float32, np.float32),
         "CC": (np.complex64, np.complex64), "CF": (np.complex64, np.float32)}


def make(tt, T, L, seed):
    tdt, xdt = TYPES[tt]
    rng = np.random.default_rng(seed)
    taps = (rng.standard_normal(T) / np.sqrt(max(T, 1))).astype(np.float32)
    if tdt is np.complex64:
        taps = (taps + 1j * (rng.standard_normal(T) / np.sqrt(max(T, 1)))).astype(np.complex64)
    x = rng.random(L * (2 if xdt is np.complex64 else 1), dtype=np.float32) * 2 - 1
    if xdt is np.complex64:
        x = x.view(np.complex64)
    return taps, x


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def run_fir(cuda, taps, x, D, N, x_offset=0):
    from gsdr_amd import ops

    xt = dev(x, cuda)
    if x_offset:
        pad = torch.zeros(x_offset, dtype=xt.dtype, device=cuda)
        xt = torch.cat([pad, xt])[x_offset:]  # same values, pointer shifted off 16-byte alignment
    y = ops.fir(dev(taps, cuda), xt, D, N)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.mark.parametrize("T", [1, 8, 63, 127, 200])
@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 16, 20, 24, 32, 40, 50, 64, 100])
@pytest.mark.parametrize("tt", list(TYPES))
def test_fir_parity(cuda, tt, D, T):
    N = 2 * 4096 + 37  # several tiles plus a ragged tail
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=D * 1000 + T)
    y = run_fir(cuda, taps, x, D, N)
    ref = o.fir(taps, x, D, N)
    assert normwise_err(y, ref, bound(taps, x, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("N", [1, 2, 7, 255, 1024, 1025, 4097])
@pytest.mark.parametrize("tt", ["FC", "FF"])
def test_fir_ragged_sizes(cuda, tt, N):
    D, T = (4, 127) if tt == "FC" else (1, 63)
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=N)
    y = run_fir(cuda, taps, x, D, N)
    assert normwise_err(y, o.fir(taps, x, D, N), bound(taps, x, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("tt,D", [("FC", 4), ("FC", 1), ("FF", 1), ("CC", 2), ("CF", 4), ("FF", 8), ("FC", 3),
                                  ("FF", 5), ("CC", 6), ("CF", 7), ("FC", 10), ("FF", 12), ("CF", 16)])
def test_fir_unaligned_input(cuda, tt, D):
    """Caller passes input + 1 sample (streaming overlap): 8-/4-byte aligned only."""
    N, T = 3000, 63
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=77)
    y = run_fir(cuda, taps, x, D, N, x_offset=1)
    assert normwise_err(y, o.fir(taps, x, D, N), bound(taps, x, D, N)) <= FLOAT_TOL


def test_fir_impulse_response(cuda):
    """reference tests/test_fir.cpp:191-206, with the kernel's correlation semantics: impulse at
    x[T-1] returns the taps reversed, impulse at x[0] returns t[0] then zeros."""
    taps = np.array([0.1, 0.2, 0.3, 0.4, 0.3, 0.2, 0.1, 0.0], np.float32)
    n = 1000
    for pos, want in ((taps.size - 1, taps[::-1]), (0, taps[:1])):
        x = np.zeros(n + taps.size - 1, np.float32)
        x[pos] = 1.0
        y = run_fir(cuda, taps, x, 1, n)
        assert np.array_equal(y[:want.size], want) and np.all(y[want.size:] == 0)


def test_fir_zero_taps_and_zero_outputs(cuda):
    from gsdr_amd import abi, ops

    x = torch.ones(64, dtype=torch.complex64, device=cuda)
    out = torch.full((16,), 7.0 + 7.0j, dtype=torch.complex64, device=cuda)
    ops.fir(torch.zeros(0, dtype=torch.float32, device=cuda), x, 4, 16, out=out)
    torch.cuda.synchronize()
    assert torch.all(out == 0)
    # N == 0 is a no-op success, decimation 0 is rejected
    assert abi.lib.gsdrFirFC(4, x.data_ptr(), 1, x.data_ptr(), out.data_ptr(), 0, 0, None) == 0
    assert abi.lib.gsdrFirFC(0, x.data_ptr(), 1, x.data_ptr(), out.data_ptr(), 4, 0, None) != 0


def test_fir_restores_current_device(cuda):
    from gsdr_amd import ops

    torch.cuda.set_device(0)
    taps, x = make("FC", 15, 4 * 99 + 15, 3)
    ops.fir(dev(taps, cuda), dev(x, cuda), 4, 100)
    assert torch.cuda.current_device() == 0


# Tile shapes of gsdrxFirFCVariant (fir_dispatch.hpp launch_d4_complex). The per-output MAC order of
# the polyphase kernels depends only on (D, JC), so the JC = 16 shapes must equal variant 0 bit for
# bit; the generic kernel (7) and the matrix-core core (13) sum in ascending tap order, like the oracle.
VARIANTS_JC16 = [0, 1, 3, 8, 9, 10, 11, 14, 24, 25, 26, 28]
VARIANTS_OTHER_ORDER = [4, 5]  # JC = 32 / JC = 8: own MAC order, normwise bar
VARIANTS_ASCENDING = [7, 13]
INT8_VARIANTS = [0, 1, 3, 4, 5, 7, 24, 28]  # launch_d4_int8


@pytest.mark.parametrize("T", [127, 63, 200])
@pytest.mark.parametrize("variant", VARIANTS_JC16 + VARIANTS_OTHER_ORDER + VARIANTS_ASCENDING)
def test_fir_fc_d4_variants(cuda, variant, T):
    """Every exported tile shape of the headline kernel (gsdrxFirFCVariant) against the oracle."""
    from gsdr_amd import ops

    if variant == 13 and T > 132:
        pytest.skip("variant 13 holds at most 132 taps in registers (returns hipErrorInvalidValue)")
    N, D = 50000 + 3, 4
    taps, x = make("FC", T, (N - 1) * D + T, 99 + T)
    td, xd = dev(taps, cuda), dev(x, cuda)
    y = ops.fir_variant(variant, td, xd, D, N).cpu().numpy()
    ref = o.fir(taps, x, D, N)
    if variant in VARIANTS_ASCENDING:
        assert np.array_equal(y.view(np.uint64), ref.view(np.uint64))
    else:
        assert normwise_err(y, ref, bound(taps, x, D, N)) <= FLOAT_TOL
    if variant in VARIANTS_JC16:
        y0 = ops.fir_variant(0, td, xd, D, N).cpu().numpy()
        assert np.array_equal(y.view(np.uint64), y0.view(np.uint64))


def test_fir_fc_d4_variant_13_rejects_long_filters(cuda):
    from gsdr_amd import GsdrError, ops

    taps, x = make("FC", 133, 3 * 4 + 133, 5)
    with pytest.raises(GsdrError):
        ops.fir_variant(13, dev(taps, cuda), dev(x, cuda), 4, 4)


@pytest.mark.parametrize("variant", INT8_VARIANTS)
def test_fir_int8_d4_variants(cuda, variant):
    """gsdrxFirFCInt8Variant: each shape is bit-identical to gsdrxFirFCVariant of the same shape on the
    converted samples (the conversion exists only in LDS), and meets the bar against the oracle."""
    from gsdr_amd import ops

    N, D, T = 20000 + 5, 4, 127
    taps = make("FC", T, 1, 11)[0]
    rng = np.random.default_rng(variant)
    x8 = torch.from_numpy(rng.integers(-128, 128, 2 * ((N - 1) * D + T), dtype=np.int8)).to(cuda)
    td = dev(taps, cuda)
    y8 = ops.fir_variant(variant, td, x8, D, N)
    xf = ops.int8_to_norm_float(x8).view(torch.complex64)
    yf = ops.fir_variant(variant, td, xf, D, N)
    assert torch.equal(y8.view(torch.float32), yf.view(torch.float32))
    xh = xf.cpu().numpy()
    assert normwise_err(y8.cpu().numpy(), o.fir(taps, xh, D, N), bound(taps, xh, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("T", [1, 2, 3, 4, 5, 8, 63, 116, 117, 127, 128, 132])
@pytest.mark.parametrize("N", [1, 1023, 1024, 4097, 50000 + 3])
def test_fir_fc_d4_mfma_variant(cuda, T, N):
    """Matrix-core kernel (variant 13, k_fir_mfma_bc): f32 MFMA is an exact fmaf chain in ascending tap
    order, so its outputs equal the oracle's bit for bit (and the generic kernel's), ragged tails and
    every tap count up to its 132-tap register budget included."""
    from gsdr_amd import ops

    D = 4
    taps, x = make("FC", T, (N - 1) * D + T, 7 + T)
    y = ops.fir_variant(13, dev(taps, cuda), dev(x, cuda), D, N)
    torch.cuda.synchronize()
    ref = o.fir(taps, x, D, N)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("variant", [9, 10, 11, 14])
@pytest.mark.parametrize("N", [1024, 50000 + 3, 3 * 1024 + 1])
def test_fir_fc_d4_store_variants_bit_identical(cuda, variant, N):
    """Variants that change only the tile order or the store path (XCD order, LDS-transposed stores)
    keep the default's per-output MAC order: outputs equal variant 0 bit for bit, tails included."""
    from gsdr_amd import ops

    D, T = 4, 127
    taps, x = make("FC", T, (N - 1) * D + T, 5)
    tt, xt = dev(taps, cuda), dev(x, cuda)
    y0 = ops.fir_variant(0, tt, xt, D, N)
    y = ops.fir_variant(variant, tt, xt, D, N)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy().view(np.uint64), y0.cpu().numpy().view(np.uint64))


def test_fir_fc_d4_full_config(cuda):
    """BASELINE config 2: 127-tap FC, decimation 4, 2^24 outputs from 67,108,987 samples.
    Oracle spot checks on three windows; every output checked against an fp32 torch conv1d
    (cross-correlation with stride, the same operation) under the normwise bound."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    N, D, T = 1 << 24, 4, 127
    L = (N - 1) * D + T
    g = torch.Generator(device=cuda).manual_seed(0x5EED)
    x = (torch.rand(2 * L, device=cuda, generator=g) * 2 - 1).view(torch.complex64)
    taps_np = lowpass_taps(T, 0.1)
    taps = dev(taps_np, cuda)
    y = ops.fir(taps, x, D, N)
    torch.cuda.synchronize()
    # full-size property check vs torch fp32 conv1d
    xr = torch.view_as_real(x)
    w = taps.view(1, 1, T)
    f = torch.nn.functional.conv1d
    ref_re = f(xr[:, 0].reshape(1, 1, -1), w, stride=D).flatten()
    ref_im = f(xr[:, 1].reshape(1, 1, -1), w, stride=D).flatten()
    s = f(x.abs().reshape(1, 1, -1), taps.abs().view(1, 1, T), stride=D).flatten()
    err = torch.maximum((y.real - ref_re).abs(), (y.imag - ref_im).abs()) / s.clamp_min(1e-30)
    assert float(err.max()) <= FLOAT_TOL
    # oracle windows: head, middle, tail
    for k0 in (0, N // 2 - 1000, N - 4096):
        k1 = k0 + 4096
        xs = x[k0 * D:(k1 - 1) * D + T].cpu().numpy()
        ref = o.fir(taps_np, xs, D, k1 - k0)
        got = y[k0:k1].cpu().numpy()
        assert normwise_err(got, ref, bound(taps_np, xs, D, k1 - k0)) <= FLOAT_TOL


def test_fir_ff_config1(cuda):
    """BASELINE config 1 shape on the GPU: 63-tap real FIR, no decimation, 2^20 outputs."""
    from gsdr_amd.signals import lowpass_taps

    N, T = 1 << 20, 63
    rng = np.random.default_rng(1)
    x = (rng.random(N + T - 1, dtype=np.float32) * 2 - 1)
    taps = lowpass_taps(T, 0.1)
    y = run_fir(cuda, taps, x, 1, N)
    assert normwise_err(y, o.fir(taps, x, 1, N), bound(taps, x, 1, N)) <= FLOAT_TOL


def test_fir_linearity(cuda):
    """Size-independent property: fir(a x1 + b x2) = a fir(x1) + b fir(x2) within the bound."""
    from gsdr_amd import ops

    N, D, T = 200000, 4, 127
    taps, x1 = make("FC", T, (N - 1) * D + T, 5)
    _, x2 = make("FC", T, (N - 1) * D + T, 6)
    t, a, b = dev(taps, cuda), 0.75, -1.25
    lhs = ops.fir(t, dev((a * x1 + b * x2).astype(np.complex64), cuda), D, N)
    rhs = a * ops.fir(t, dev(x1, cuda), D, N) + b * ops.fir(t, dev(x2, cuda), D, N)
    s = bound(taps, np.abs(a * x1) + np.abs(b * x2), D, N)
    assert normwise_err(lhs.cpu().numpy(), rhs.cpu().numpy(), s) <= 2 * FLOAT_TOL


@pytest.mark.parametrize("tt", ["FC", "FF", "CC", "CF"])
@pytest.mark.parametrize("D,T", [(4, 1001), (4, 4001), (4, 6000), (2, 2500), (8, 3001), (1, 2048), (3, 1500),
                                 (9, 1500), (50, 4000), (32, 3000), (13, 9000)])
def test_fir_long_filters(cuda, tt, D, T):
    """Long filters: the polyphase tile grows with the tap span until it leaves the 64 KB LDS budget
    (near T = 4000 at D = 4), after which the generic kernel runs; both sides of that boundary. The
    runtime-decimation tile (D = 9, 13, 50) narrows to 128 or 64 outputs before giving up."""
    N = 3000 + D
    taps, x = make(tt, T, (N - 1) * D + T, T + D)
    y = run_fir(cuda, taps, x, D, N)
    ref = o.fir(taps, x, D, N)
    assert normwise_err(y, ref, bound(taps, x, D, N)) <= FLOAT_TOL


@pytest.mark.parametrize("tt,D", [("FC", 4), ("FC", 1), ("CC", 2), ("FC", 3), ("FC", 8), ("CC", 16), ("FC", 32)])
def test_fir_shifted_staging_bit_identical(cuda, tt, D):
    """A complex input 8 bytes off 16-byte alignment is staged with shifted 16-byte loads (stage_tile
    SH mode); the outputs must equal those of the same samples at an aligned address, bit for bit."""
    N, T = 3 * 4096 + 5, 127
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=91 + D)
    aligned = run_fir(cuda, taps, x, D, N)
    shifted = run_fir(cuda, taps, x, D, N, x_offset=1)
    assert aligned.tobytes() == shifted.tobytes()


@pytest.mark.parametrize("off", [1, 2, 3])
@pytest.mark.parametrize("tt,D", [("FF", 4), ("FF", 1), ("FF", 8), ("CF", 4), ("CF", 1), ("FF", 12), ("CF", 16),
                                  ("FF", 20)])
def test_fir_shifted_real_staging_bit_identical(cuda, tt, D, off):
    """Real input 1..3 floats off 16-byte alignment is staged with aligned 16-byte loads from `off`
    samples early, each quad split over two LDS granules (stage_tile's real SH mode); the outputs equal
    those of the same samples at an aligned address bit for bit, and the oracle's within the bar."""
    N, T = 3 * 4096 + 5, 127
    L = (N - 1) * D + T
    taps, x = make(tt, T, L, seed=17 * off + D)
    aligned = run_fir(cuda, taps, x, D, N)
    shifted = run_fir(cuda, taps, x, D, N, x_offset=off)
    assert aligned.tobytes() == shifted.tobytes()
    assert normwise_err(shifted, o.fir(taps, x, D, N), bound(taps, x, D, N)) <= FLOAT_TOL
