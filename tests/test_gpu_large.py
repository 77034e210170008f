"""GPU parity at the maximum sizes the ABI admits (counts are size_t for the FIR,
demodulator and element-wise entry points, uint32_t numSymbols for QPSK / QPSK256, qpsk.h:116-239,
qpsk256.h:125-215). Inputs of 2^31 .. 2^32 samples (17-34 GB, resident in HBM) put every 32-bit
sample index, byte offset and grid computation past its overflow point; outputs are checked against
the oracle on windows straddling each crossing and at the end, and the QPSK paths by a full
noise-free round trip compared on the device."""
import numpy as np
import pytest
import torch

from oracle import oracle as o
from helpers import FLOAT_TOL, normwise_err

pytestmark = pytest.mark.gpu

W = 2048  # outputs per checked window


@pytest.fixture(autouse=True)
def _release(cuda):
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def rand_iq(n, cuda, seed):
    g = torch.Generator(device=cuda).manual_seed(seed)
    return (torch.rand(2 * n, device=cuda, generator=g) * 2 - 1).view(torch.complex64)


def windows(n_out, crossings):
    """[k0, k1) windows: the start, the end, and W outputs either side of each crossing output index."""
    ws = [(0, W), (n_out - W, n_out)]
    for k in crossings:
        if W <= k <= n_out - W:
            ws.append((k - W, k + W))
    return ws


def test_fir_fc_d4_input_beyond_2_31_samples(cuda):
    """gsdrFirFC, D = 4, T = 127 over 2^31 + 147 input samples (17.2 GB): the input byte offset passes
    2^32 at output 2^27 and the sample index passes 2^31 at output 2^29."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    D, T = 4, 127
    n_out = (1 << 29) + 5
    n_in = (n_out - 1) * D + T
    x = rand_iq(n_in, cuda, 11)
    taps_np = lowpass_taps(T, 0.1)
    y = ops.fir(torch.from_numpy(taps_np).to(cuda), x, D, n_out)
    torch.cuda.synchronize()
    for k0, k1 in windows(n_out, [1 << 27, 1 << 29, (1 << 29) - (T // D)]):
        xs = x[k0 * D:(k1 - 1) * D + T].cpu().numpy()
        want = o.fir(taps_np, xs, D, k1 - k0)
        got = y[k0:k1].cpu().numpy()
        err = normwise_err(got, want, o.fir_bound_fc(taps_np, xs, D, k1 - k0))
        assert err <= FLOAT_TOL, (k0, err)


def test_fir_ff_d1_input_beyond_2_32_samples(cuda):
    """gsdrFirFF, D = 1 (the contiguous-window kernel), T = 63 over 2^32 + 70 real samples: the sample
    index passes 2^31 and 2^32 (config 1's shape at 4096x its length)."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    T = 63
    n_in = (1 << 32) + 70
    n_out = n_in - T + 1
    g = torch.Generator(device=cuda).manual_seed(12)
    x = torch.rand(n_in, device=cuda, generator=g) * 2 - 1
    taps_np = lowpass_taps(T, 0.1)
    y = ops.fir(torch.from_numpy(taps_np).to(cuda), x, 1, n_out)
    torch.cuda.synchronize()
    for k0, k1 in windows(n_out, [1 << 30, 1 << 31, 1 << 32]):
        xs = x[k0:k1 - 1 + T].cpu().numpy()
        want = o.fir(taps_np, xs, 1, k1 - k0)
        bound = np.convolve(np.abs(xs.astype(np.float64)), np.abs(taps_np[::-1].astype(np.float64)), "valid")
        err = normwise_err(y[k0:k1].cpu().numpy(), want, bound)
        assert err <= FLOAT_TOL, (k0, err)


def test_am_demod_beyond_2_31_samples_large_first_index(cuda):
    """gsdrAmDemod (NCO + FIR + envelope) over 2^31 + 123 samples with firstSampleIndex past 2^33: the
    absolute NCO index and the tile offsets both exceed 32 bits."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    D, T = 4, 127
    fs, tune, chan = 1.0e6, 0.0, 1.0e5
    n0 = (1 << 33) + 7
    n_out = (1 << 29) - 1
    n_in = (n_out - 1) * D + T
    x = rand_iq(n_in, cuda, 13) * 0.7
    taps_np = lowpass_taps(T, 0.1)
    y = ops.am_demod(x, torch.from_numpy(taps_np).to(cuda), fs, tune, chan, D, n0, n_out)
    torch.cuda.synchronize()
    for k0, k1 in windows(n_out, [1 << 27, 1 << 28]):
        xs = x[k0 * D:(k1 - 1) * D + T].cpu().numpy()
        want = o.am_demod(xs, taps_np, fs, tune, chan, D, n0 + k0 * D, k1 - k0)
        err = float(np.max(np.abs(y[k0:k1].cpu().numpy() - want)))
        assert err <= FLOAT_TOL, (k0, err)


def test_magnitude_beyond_2_31_elements(cuda):
    """gsdrMagnitude over 2^31 + 3 complex samples (17.2 GB in, 8.6 GB out)."""
    from gsdr_amd import ops

    n = (1 << 31) + 3
    x = rand_iq(n, cuda, 14)
    y = ops.magnitude(x)
    torch.cuda.synchronize()
    for k0, k1 in windows(n, [1 << 28, 1 << 30, 1 << 31]):
        ref = o.magnitude(x[k0:k1].cpu().numpy())
        got = y[k0:k1].cpu().numpy()
        assert np.max(np.abs(got - ref) / np.maximum(ref, 1e-30)) <= FLOAT_TOL, k0


def test_qpsk_round_trip_max_symbols(cuda):
    """gsdrQpskModulate / gsdrQpskDemodulate at numSymbols = 2^32 - 1 (the uint32_t maximum; 34 GB of
    symbols): every symbol is one of the four points of its bit pair (spot windows vs the oracle), the
    round trip returns every bit, and the final partial byte keeps its unused high pair."""
    from gsdr_amd import ops

    n = (1 << 32) - 1
    nb = (n + 3) // 4
    g = torch.Generator(device=cuda).manual_seed(15)
    bits = torch.randint(0, 256, (nb,), dtype=torch.uint8, device=cuda, generator=g)
    a = 0.8
    sym = ops.qpsk_modulate(bits, n, a)
    torch.cuda.synchronize()
    for s0 in (0, 1 << 29, 1 << 31, n - 4 * W + 1):
        s0 -= s0 % 4
        s1 = min(s0 + 4 * W, n)
        want = o.qpsk_mod(bits[s0 // 4:(s1 + 3) // 4].cpu().numpy(), s1 - s0, a)
        assert np.array_equal(sym[s0:s1].cpu().numpy(), want), s0
    back = torch.full((nb,), 0xFF, dtype=torch.uint8, device=cuda)
    ops.qpsk_demodulate(sym, n, out=back)
    torch.cuda.synchronize()
    assert torch.equal(back[:nb - 1], bits[:nb - 1])
    last = n % 4  # 3 symbols in the final byte: bits 0-5 from the data, bits 6-7 preserved
    mask = (1 << (2 * last)) - 1
    assert int(back[nb - 1]) & mask == int(bits[nb - 1]) & mask
    assert int(back[nb - 1]) & ~mask & 0xFF == 0xFF & ~mask


@pytest.mark.parametrize("ctype", [0, 1])
def test_qpsk256_round_trip_max_symbols(cuda, ctype):
    """gsdrQpsk256Modulate / gsdrQpsk256Demodulate at numSymbols = 2^32 - 1, both constellations: the
    modulated points equal the table entries of their bytes (spot windows) and the noise-free round
    trip returns every byte (compared on the device)."""
    from gsdr_amd import ops

    n = (1 << 32) - 1
    ops.qpsk256_init(ctype, 1.0)
    table = o.qpsk256_table(ctype, 1.0)
    g = torch.Generator(device=cuda).manual_seed(16 + ctype)
    syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=cuda, generator=g)
    pts = ops.qpsk256_modulate(syms, ctype)
    torch.cuda.synchronize()
    for s0 in (0, (1 << 31) - W, n - W):
        s1 = s0 + W
        assert np.array_equal(pts[s0:s1].cpu().numpy(), table[syms[s0:s1].cpu().numpy()]), s0
    back = ops.qpsk256_demodulate(pts, ctype)
    torch.cuda.synchronize()
    assert torch.equal(back, syms)


@pytest.mark.parametrize("cplx", [False, True])
def test_iir_beyond_2_31_samples(cuda, cplx):
    """gsdrIirFF over 2^31 + 5 real samples / gsdrIirCC over 2^30 + 5 complex ones (8.6 GB): 2^26 scan
    chunks, five scan levels. The 4th-order Butterworth's impulse response decays below 1e-30 within
    4096 samples, so the oracle restarted from zero state 4096 samples before a window reproduces the
    true recursion there."""
    from scipy import signal

    from gsdr_amd import ops

    b, a = (v.astype(np.float32) for v in signal.butter(4, 0.1))
    n = ((1 << 30) if cplx else (1 << 31)) + 5
    x = rand_iq(n, cuda, 17) if cplx else torch.rand(n, device=cuda, generator=torch.Generator(
        device=cuda).manual_seed(17)) * 2 - 1
    y = ops.iir(torch.from_numpy(b).to(cuda), torch.from_numpy(a).to(cuda), x)
    torch.cuda.synchronize()
    lead = 4096
    for k0, k1 in windows(n, [1 << 26, 1 << 29, 1 << 30, 1 << 31]):
        s = max(0, k0 - lead)
        want, _, _ = o.iir(b, a, x[s:k1].cpu().numpy())
        want = want[k0 - s:]
        got = y[k0:k1].cpu().numpy()
        e = float(np.max(np.abs(got - want))) / max(1.0, float(np.max(np.abs(want))))
        assert e <= 1e-6, (k0, e)


def periodic_fm_int8(n_in, cuda, seed):
    """Config 3's signal quantised to int8 I/Q (x 100) at any length: its clean part (carrier 0.1 fs, tone
    0.001 fs, deviation 0.02 fs) repeats every 1000 samples, so one period is tiled; the noise (uniform
    integers in [-5, 5] per component) is drawn chunk by chunk on the device."""
    idx = torch.arange(1000, dtype=torch.float64)
    ph = 2 * np.pi * 0.1 * idx + 20.0 * torch.sin(2 * np.pi * 0.001 * idx)
    period = torch.round(torch.view_as_real(torch.polar(torch.ones_like(ph), ph)).reshape(-1) * 100).to(torch.int16)
    period = period.to(cuda)
    x8 = torch.empty(2 * n_in, dtype=torch.int8, device=cuda)
    g = torch.Generator(device=cuda).manual_seed(seed)
    chunk = 2000 * (1 << 16)  # a multiple of the period's 2000 bytes
    for s in range(0, 2 * n_in, chunk):
        e = min(s + chunk, 2 * n_in)
        base = period.repeat(chunk // 2000)[:e - s]
        noise = torch.randint(-5, 6, (e - s,), dtype=torch.int16, device=cuda, generator=g)
        x8[s:e] = torch.clamp(base + noise, -128, 127).to(torch.int8)
    return x8


def test_int8_fir_and_fm_beyond_2_31_samples(cuda):
    """gsdrxFirFCInt8 and gsdrxFmDemodInt8 (D = 4, T = 127: the matrix-core kernels, whose output indexing is
    32-bit relative to each tile) over 2^31 + 143 int8 I/Q samples (4.3 GB in): windows at 2^30 and 2^31
    input samples and at the end, against the oracle on the converted samples (normwise for the FIR,
    wrapped angle for the FM chain, firstSampleIndex of each window = n0 + k0 D)."""
    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    from helpers import wrapped_angle_err

    D, T = 4, 127
    n_out = (1 << 29) + 5
    n_in = (n_out - 1) * D + T
    x8 = periodic_fm_int8(n_in, cuda, 21)
    taps_np = lowpass_taps(T, 0.1)
    td = torch.from_numpy(taps_np).to(cuda)
    y = ops.fir(td, x8, D, n_out)
    torch.cuda.synchronize()
    crossings = [1 << 28, 1 << 29, (1 << 29) - (T // D)]  # output k reads samples from 4k: 2^30, 2^31
    for k0, k1 in windows(n_out, crossings):
        xs = o.int8_to_float(x8[2 * k0 * D:2 * ((k1 - 1) * D + T)].cpu().numpy()).view(np.complex64)
        want = o.fir(taps_np, xs, D, k1 - k0)
        err = normwise_err(y[k0:k1].cpu().numpy(), want, o.fir_bound_fc(taps_np, xs, D, k1 - k0))
        assert err <= FLOAT_TOL, ("fir", k0, err)
    del y
    torch.cuda.empty_cache()
    fs, tune, chan, dhz, n0 = 1.0e6, 0.0, 1.0e5, 2.0e4, (1 << 32) + 11
    n_fm = (n_in - T) // D
    fm = ops.fm_demod(x8, td, fs, tune, chan, dhz, D, n0, n_fm)
    torch.cuda.synchronize()
    g = fs / (2 * np.pi * dhz)
    for k0, k1 in windows(n_fm, crossings):
        xs = o.int8_to_float(x8[2 * k0 * D:2 * (k1 * D + T)].cpu().numpy()).view(np.complex64)
        want = o.fm_demod(xs, taps_np, fs, tune, chan, dhz, D, n0 + k0 * D, k1 - k0)
        err = wrapped_angle_err(fm[k0:k1].cpu().numpy(), want, g)
        assert err <= FLOAT_TOL, ("fm", k0, err)
