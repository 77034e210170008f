"""GPU parity, bit-exact: QPSK (reference src/qpsk.cu) and QPSK256 (src/qpsk256.cu) through the C ABI
vs the C oracle. Named after the reference's tests/test_qpsk.cpp and tests/test_qpsk256.cpp cases."""
import numpy as np
import pytest
import torch

from oracle import oracle as o

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


NS = [1, 3, 4, 5, 15, 16, 17, 31, 33, 1001, 65536 + 3]


def noisy_qpsk(bits, n, a, seed):
    sym = o.qpsk_mod(bits, n, a)
    rng = np.random.default_rng(seed)
    rx = (sym + 0.4 * a * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    rx[: min(n, 3)] = [0.0, complex(-0.0, -0.0), complex(np.nan, 1.0)][: min(n, 3)]
    return sym, rx


@pytest.mark.parametrize("n", NS)
def test_qpsk_modulate_demodulate(cuda, n):
    from gsdr_amd import ops

    rng = np.random.default_rng(n)
    bits = rng.integers(0, 256, (n + 3) // 4, dtype=np.uint8)
    sym = ops.qpsk_modulate(dev(bits, cuda), n, 0.8)
    ref_sym, rx = noisy_qpsk(bits, n, 0.8, n)
    assert np.array_equal(sym.cpu().numpy(), ref_sym)
    # demod: bytes pre-filled with 0xff so the preserved high pairs of a final partial byte show
    prev = np.full((n + 3) // 4, 0xFF, dtype=np.uint8)
    got = dev(prev, cuda)
    ops.qpsk_demodulate(dev(rx, cuda), n, out=got)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), o.qpsk_demod(rx, n, initial=prev))


def test_qpsk_round_trip_and_points(cuda):
    """test_qpsk.cpp:87-170: ideal-channel round trip, four points, |.| = a sqrt 2."""
    from gsdr_amd import ops

    n = 100003
    bits = np.random.default_rng(1).integers(0, 256, (n + 3) // 4, dtype=np.uint8)
    for a in (0.5, 1.0, 2.0, 10.0):
        sym = ops.qpsk_modulate(dev(bits, cuda), n, a)
        back = ops.qpsk_demodulate(sym).cpu().numpy()
        s = sym.cpu().numpy()
        assert set(np.unique(s).tolist()) == {complex(a, a), complex(-a, a), complex(-a, -a), complex(a, -a)}
        last = n % 4
        full = n // 4
        assert np.array_equal(back[:full], bits[:full])
        if last:
            mask = (1 << (2 * last)) - 1
            assert (back[full] & mask) == (bits[full] & mask)


def test_qpsk_4x(cuda):
    from gsdr_amd import ops

    n = 4099
    rng = np.random.default_rng(2)
    bits = [rng.integers(0, 256, (n + 3) // 4, dtype=np.uint8) for _ in range(4)]
    outs = [torch.empty(n, dtype=torch.complex64, device=cuda) for _ in range(4)]
    ops.qpsk_modulate_4x([dev(b, cuda) for b in bits], outs, n, 1.5)
    rx = [noisy_qpsk(bits[i], n, 1.5, 10 + i)[1] for i in range(4)]
    got = [torch.zeros((n + 3) // 4, dtype=torch.uint8, device=cuda) for _ in range(4)]
    ops.qpsk_demodulate_4x([dev(r, cuda) for r in rx], got, n)
    torch.cuda.synchronize()
    for i in range(4):
        assert np.array_equal(outs[i].cpu().numpy(), o.qpsk_mod(bits[i], n, 1.5))
        assert np.array_equal(got[i].cpu().numpy(), o.qpsk_demod(rx[i], n))


@pytest.mark.parametrize("streams", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("n", [5, 1001, 4096])
def test_qpsk_templated(cuda, streams, n):
    """Consolidated layout (qpsk.cu:42, 56, 75, 87): bits at s*(n/4+1), symbols at s*n; unsupported
    stream counts fall back to stream 0 only (qpsk.cu:619-622)."""
    from gsdr_amd import ops

    S = 8
    stride = n // 4 + 1
    rng = np.random.default_rng(n + streams)
    bits = rng.integers(0, 256, S * stride, dtype=np.uint8)
    out = torch.zeros(S * n, dtype=torch.complex64, device=cuda)
    ops.qpsk_modulate_templated(dev(bits, cuda), out, n, 1.0, streams)
    active = streams if streams in (1, 2, 4, 8) else 1
    rx = np.concatenate([noisy_qpsk(bits[s * stride:(s + 1) * stride], n, 1.0, s)[1] for s in range(S)])
    got = torch.full((S * stride,), 0xAA, dtype=torch.uint8, device=cuda)
    ops.qpsk_demodulate_templated(dev(rx, cuda), got, n, streams)
    torch.cuda.synchronize()
    o_sym = out.cpu().numpy()
    g = got.cpu().numpy()
    for s in range(S):
        b = bits[s * stride:(s + 1) * stride]
        if s < active:
            assert np.array_equal(o_sym[s * n:(s + 1) * n], o.qpsk_mod(b, n, 1.0))
            want = o.qpsk_demod(rx[s * n:(s + 1) * n], n, initial=np.full(stride, 0xAA, np.uint8))
            assert np.array_equal(g[s * stride:(s + 1) * stride], want)
        else:
            assert np.all(o_sym[s * n:(s + 1) * n] == 0)
            assert np.all(g[s * stride:(s + 1) * stride] == 0xAA)


# ------------------------------------------------------------------------------------ QPSK256

@pytest.mark.parametrize("ctype", [0, 1])
@pytest.mark.parametrize("amp", [1.0, 0.5, 2.5])
def test_qpsk256_tables_and_modulate(cuda, ctype, amp):
    """test_qpsk256.cpp:128-170: 256 distinct points; the device table equals the oracle's bitwise."""
    from gsdr_amd import ops

    ops.qpsk256_init(ctype, amp)
    syms = np.arange(256, dtype=np.uint8)
    pts = ops.qpsk256_modulate(dev(syms, cuda), ctype).cpu().numpy()
    assert np.array_equal(pts, o.qpsk256_table(ctype, amp))
    assert len(set(pts.tolist())) == 256


@pytest.mark.parametrize("ctype,sigma", [(0, 0.02), (0, 0.08), (1, 0.01)])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 100003])
def test_qpsk256_demodulate_bit_exact(cuda, ctype, sigma, n):
    from gsdr_amd import ops

    amp = 1.0
    ops.qpsk256_init(ctype, amp)
    table = o.qpsk256_table(ctype, amp)
    rng = np.random.default_rng(n + ctype)
    syms = rng.integers(0, 256, n, dtype=np.uint8)
    rx = (table[syms] + sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    special = [complex(np.nan, 0), complex(np.inf, 1), complex(1e30, -1e30), complex(7.5, -7.5), 0j,
               complex(1.0 / 15.0, 1.0 / 15.0)]  # last: an exact midpoint between two grid levels
    rx[: min(n, len(special))] = special[: min(n, len(special))]
    got = ops.qpsk256_demodulate(dev(rx, cuda), ctype).cpu().numpy()
    assert np.array_equal(got, o.qpsk256_demod(table, rx))


def test_qpsk256_4x(cuda):
    from gsdr_amd import ops

    n, ctype = 5003, 0
    ops.qpsk256_init(ctype, 1.0)
    table = o.qpsk256_table(ctype, 1.0)
    rng = np.random.default_rng(44)
    syms = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)]
    outs = [torch.empty(n, dtype=torch.complex64, device=cuda) for _ in range(4)]
    ops.qpsk256_modulate_4x([dev(s, cuda) for s in syms], outs, n, ctype)
    back = [torch.empty(n, dtype=torch.uint8, device=cuda) for _ in range(4)]
    ops.qpsk256_demodulate_4x(outs, back, n, ctype)
    torch.cuda.synchronize()
    for i in range(4):
        assert np.array_equal(outs[i].cpu().numpy(), table[syms[i]])
        assert np.array_equal(back[i].cpu().numpy(), syms[i])


def _threads():
    import os

    return max(1, min(64, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("ctype,sigma", [(0, 0.02), (1, 0.01)])
def test_qpsk256_config5_round_trip(cuda, ctype, sigma):
    """BASELINE config 5 as specified: 2^24 symbols, modulate -> AWGN -> demod. The noisy buffer comes
    from gsdrxQpsk256ModulateAwgn (counter-based noise, gsdr_ext.h) and is bit-identical to the oracle's
    restatement over all 2^24 symbols; the GPU decisions equal the oracle's exhaustive argmin of the reference's cuCabsf
    rule (qpsk256.cu:171-181) over all 2^24 symbols. The symbol error rate against the transmitted bytes is a sanity figure."""
    from gsdr_amd import ops

    n, seed, first = 1 << 24, 0x5EED_0005, 3
    ops.qpsk256_init(ctype, 1.0)
    g = torch.Generator(device=cuda).manual_seed(0x5EED)
    syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=cuda, generator=g)
    rx = ops.qpsk256_modulate_awgn(syms, ctype, sigma, seed, first)
    got = ops.qpsk256_demodulate(rx, ctype)
    torch.cuda.synchronize()
    ser = float((got != syms).float().mean())
    assert 1e-5 < ser < 5e-2
    table = o.qpsk256_table(ctype, 1.0)
    syms_np = syms.cpu().numpy()
    rx_np = rx.cpu().numpy()
    want_rx = o.qpsk256_mod_awgn(table, syms_np, sigma, seed, first, nthreads=_threads())
    assert rx_np.tobytes() == want_rx.tobytes()
    assert np.array_equal(got.cpu().numpy(), o.qpsk256_demod(table, rx_np, nthreads=_threads()))


def test_qpsk256_awgn_tails_reach_beyond_five_sigma(cuda):
    """the channel's noise must keep the Gaussian's tails (the 21-bit construction had none past
    5.035 sigma). 2^24 symbols at sigma = 1 around point 0: the counts beyond 4.5 and 5.04 sigma over the
    2^25 components follow erfc within Poisson bounds (5 sigma), the largest |g| is past the old cut, and a
    tail-heavy slice is bit-identical to the oracle (which restates the extension)."""
    import math

    from gsdr_amd import ops

    n, seed = 1 << 24, 0xABCDEF
    ops.qpsk256_init(0, 1.0)
    syms = torch.zeros(n, dtype=torch.uint8, device=cuda)
    rx = ops.qpsk256_modulate_awgn(syms, 0, 1.0, seed, 0)
    p0 = torch.tensor(complex(o.qpsk256_table(0, 1.0)[0]), dtype=torch.complex64, device=cuda)
    g = torch.view_as_real(rx - p0).reshape(-1).abs()
    comps = 2 * n
    for t in (4.5, 5.04):
        want = comps * math.erfc(t / math.sqrt(2.0))
        got = int((g > t).sum())
        assert abs(got - want) <= 5 * math.sqrt(want) + 2, (t, got, want)
        assert got >= 4, (t, got)  # the 21-bit construction gave exactly 0 beyond 5.035
    assert float(g.max()) > 5.04
    # the symbols holding the largest components: the GPU's noisy values equal the oracle's bit for bit
    idx = torch.topk(g, 64).indices.div(2, rounding_mode="floor").unique().cpu().numpy()
    table = o.qpsk256_table(0, 1.0)
    rx_np = rx.cpu().numpy()
    for k in idx[:32]:
        want = o.qpsk256_mod_awgn(table, np.zeros(1, np.uint8), 1.0, seed, int(k))
        assert rx_np[k:k + 1].tobytes() == want.tobytes(), k


@pytest.mark.parametrize("n", [1, 2, 3, 5, 6, 7, 1535, 1537, 4607, 4608, 4609, 100_003])  # 6 a lane step, 4608 a workgroup
@pytest.mark.parametrize("first", [0, 1, 2, 2**32 - 1, 2**40 + 6, 2**33 + 3])  # first % 3: 0, 1, 2, 0, 1, 2
def test_qpsk256_awgn_sizes_and_offsets(cuda, n, first):
    """Every size, every residue of the first absolute index mod 3 (a Philox block serves three symbols,
    so blocks straddle the buffer's ends), indices past 2^32; a buffer split over two calls equals one
    call."""
    from gsdr_amd import ops

    ctype, sigma, seed = 1, 0.05, 0xFEEDFACE12345678
    ops.qpsk256_init(ctype, 0.9)
    table = o.qpsk256_table(ctype, 0.9)
    syms_np = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    syms = dev(syms_np, cuda)
    rx = ops.qpsk256_modulate_awgn(syms, ctype, sigma, seed, first).cpu().numpy()
    assert rx.tobytes() == o.qpsk256_mod_awgn(table, syms_np, sigma, seed, first).tobytes()
    if n > 2:
        h = n // 3
        a = ops.qpsk256_modulate_awgn(syms[:h].contiguous(), ctype, sigma, seed, first).cpu().numpy()
        b = ops.qpsk256_modulate_awgn(syms[h:].contiguous(), ctype, sigma, seed, first + h).cpu().numpy()
        assert np.concatenate([a, b]).tobytes() == rx.tobytes()


@pytest.mark.parametrize("in_off,out_off", [(0, 0), (1, 0), (0, 1), (1, 1), (2, 1)])
def test_qpsk256_awgn_pointer_alignment(cuda, in_off, out_off):
    """Odd input bytes and an output 8 bytes off 16-byte alignment take the per-lane path; aligned
    pointers the wave's LDS-transposed stores. Same bits either way, whole and ragged waves."""
    from gsdr_amd import ops

    ctype, sigma, seed, first = 0, 0.02, 0x5EED0005, 7
    ops.qpsk256_init(ctype, 1.0)
    table = o.qpsk256_table(ctype, 1.0)
    n = 3 * 4608 + 385
    syms_np = np.random.default_rng(in_off * 7 + out_off).integers(0, 256, n + 4, dtype=np.uint8)
    syms = dev(syms_np, cuda)[in_off:in_off + n]
    out = torch.empty(n + 1, dtype=torch.complex64, device=cuda)[out_off:out_off + n]
    ops.qpsk256_modulate_awgn(syms, ctype, sigma, seed, first, out=out)
    want = o.qpsk256_mod_awgn(table, syms_np[in_off:in_off + n], sigma, seed, first)
    assert out.cpu().numpy().tobytes() == want.tobytes()


def test_qpsk256_awgn_overflowing_sigma_matches_oracle(cuda):
    """sigma * g overflowing to +-inf: the tail test (a NaN in a lane's output sum, awgn.hpp) also fires on
    lanes whose infinities cancel in the sum; their exact pass must reproduce the same outputs."""
    from gsdr_amd import ops

    ctype, seed, first, n = 0, 0x5EED0005, 5, 3 * 4608 + 17
    ops.qpsk256_init(ctype, 1.0)
    table = o.qpsk256_table(ctype, 1.0)
    syms_np = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8)
    for sigma in (1e38, 3.4e38):
        rx = ops.qpsk256_modulate_awgn(dev(syms_np, cuda), ctype, sigma, seed, first).cpu().numpy()
        assert rx.tobytes() == o.qpsk256_mod_awgn(table, syms_np, sigma, seed, first).tobytes()
        assert np.isinf(rx.view(np.float32)).any()


def test_qpsk256_awgn_zero_sigma_is_modulate(cuda):
    from gsdr_amd import GsdrError, ops

    ops.qpsk256_init(0, 1.0)
    syms = torch.randint(0, 256, (10_001,), dtype=torch.uint8, device=cuda)
    a = ops.qpsk256_modulate_awgn(syms, 0, 0.0, 1)
    b = ops.qpsk256_modulate(syms, 0)
    assert torch.equal(a.view(torch.float32), b.view(torch.float32))
    for bad in (-1.0, float("nan"), float("inf")):
        with pytest.raises(GsdrError):
            ops.qpsk256_modulate_awgn(syms, 0, bad, 1)


@pytest.mark.parametrize("amp", [1.0, 0.37, -2.5])
def test_qpsk256_circular_cells_bit_exact_dense(cuda, amp):
    """The circular table's per-cell candidate lists (qpsk256.hip CircCells) reproduce the exhaustive
    argmin bit for bit: 5.4 M points uniform over a square larger than the grid (outside -> exhaustive);
    more 4096-symbol tiles than demodulation workgroups, so the grid-stride loop and the tail run."""
    from gsdr_amd import ops

    ops.qpsk256_init(1, amp)
    table = o.qpsk256_table(1, amp)
    rng = np.random.default_rng(int(abs(amp) * 100))
    n = (1 << 22) + 4096 * 300 + 7
    span = 2.2 * abs(amp)
    rx = (rng.uniform(-span, span, n) + 1j * rng.uniform(-span, span, n)).astype(np.complex64)
    got = ops.qpsk256_demodulate(dev(rx, cuda), 1).cpu().numpy()
    assert np.array_equal(got, o.qpsk256_demod(table, rx, nthreads=_threads()))


@pytest.mark.parametrize("amp", [1.0, 0.37])
def test_qpsk256_circular_near_ties(cuda, amp):
    """Points on and within a few ulp of the perpendicular bisector of every pair of neighbouring
    circular points (and of the ring-filler points): the list walk's near-tie re-ranking by cuCabsf
    must reproduce the reference's exhaustive cuCabsf argmin bit for bit."""
    from gsdr_amd import ops

    ops.qpsk256_init(1, amp)
    table = o.qpsk256_table(1, amp)
    p = table.astype(np.complex128)
    d = np.abs(p[:, None] - p[None, :])
    np.fill_diagonal(d, np.inf)
    pts = []
    for i in range(256):
        for j in np.argsort(d[i])[:4]:
            m = ((table[i] + table[j]) / np.float32(2)).astype(np.complex64)
            # walk along the bisector and across it by a few ulp
            u = (p[j] - p[i]) / abs(p[j] - p[i])
            for t in np.linspace(-0.4, 0.4, 9) * d[i, j]:
                c = m + np.complex64(1j * u * t)
                for k in range(-3, 4):
                    re = np.float32(c.real)
                    im = np.float32(c.imag)
                    for _ in range(abs(k)):
                        re = np.nextafter(re, np.float32(np.inf if k > 0 else -np.inf))
                        im = np.nextafter(im, np.float32(-np.inf if k > 0 else np.inf))
                    pts.append(complex(re, im))
    x = np.array(pts, dtype=np.complex64)
    got = ops.qpsk256_demodulate(dev(x, cuda), 1).cpu().numpy()
    want = o.qpsk256_demod(table, x, nthreads=_threads())
    assert np.array_equal(got, want)
    # the near-tie path is exercised: the squared-distance rule disagrees somewhere in this set
    assert np.count_nonzero(o.qpsk256_demod(table, x, "sq", nthreads=_threads()) != want) > 0


@pytest.mark.parametrize("ctype", [0, 1])
@pytest.mark.parametrize("in_off,out_off", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_qpsk256_blocks_and_alignment(cuda, ctype, in_off, out_off):
    """Several whole 4096-symbol blocks plus a ragged tail, with the input or output pointer offset
    by one element: the coalesced block path and the per-thread path must agree with the oracle."""
    from gsdr_amd import ops

    n = 3 * 4096 + 77
    ops.qpsk256_init(ctype, 1.0)
    table = o.qpsk256_table(ctype, 1.0)
    rng = np.random.default_rng(17 + ctype)
    syms = rng.integers(0, 256, n + 1, dtype=np.uint8)
    sym_t = dev(syms, cuda)[in_off:in_off + n]
    out = torch.empty(n + 1, dtype=torch.complex64, device=cuda)[out_off:out_off + n]
    ops.qpsk256_modulate(sym_t, ctype, out=out)
    assert np.array_equal(out.cpu().numpy(), o.qpsk256_mod(table, syms[in_off:in_off + n]))
    rx = (o.qpsk256_mod(table, syms[:n + 1]) + 0.01 * (rng.standard_normal(n + 1) + 1j * rng.standard_normal(n + 1)))
    rx = rx.astype(np.complex64)
    got = torch.empty(n + 1, dtype=torch.uint8, device=cuda)[out_off:out_off + n]
    ops.qpsk256_demodulate(dev(rx, cuda)[in_off:in_off + n], ctype, out=got)
    assert np.array_equal(got.cpu().numpy(), o.qpsk256_demod(table, rx[in_off:in_off + n]))


@pytest.mark.parametrize("out_off", [0, 1, 2])
def test_qpsk_blocks_and_alignment(cuda, out_off):
    """Whole 4096-symbol blocks plus a tail, output (modulate) / bit (demodulate) pointers offset."""
    from gsdr_amd import ops

    n = 5 * 4096 + 13
    nb = (n + 3) // 4
    rng = np.random.default_rng(out_off)
    bits = rng.integers(0, 256, nb, dtype=np.uint8)
    out = torch.empty(n + 2, dtype=torch.complex64, device=cuda)[out_off:out_off + n]
    ops.qpsk_modulate(dev(bits, cuda), n, 0.75, out=out)
    sym = o.qpsk_mod(bits, n, 0.75)
    assert np.array_equal(out.cpu().numpy(), sym)
    _, rx = noisy_qpsk(bits, n, 1.0, 3)
    got = torch.full((nb + 2,), 0x5A, dtype=torch.uint8, device=cuda)[out_off:out_off + nb]
    ops.qpsk_demodulate(dev(rx, cuda), n, out=got)
    assert np.array_equal(got.cpu().numpy(), o.qpsk_demod(rx, n, initial=np.full(nb, 0x5A, np.uint8)))


@pytest.mark.parametrize("amp", [1.0, 0.37, 3.0])
def test_qpsk256_rect_decision_boundaries(cuda, amp):
    """Points on and a few ulps around the midpoints between rectangular levels (where rounded
    distances tie and the first index must win), exact levels, and the grid edges: the per-axis
    fast path with its tie check must equal the exhaustive argmin bit for bit."""
    from gsdr_amd import ops

    ops.qpsk256_init(0, amp)
    table = o.qpsk256_table(0, amp)
    lv = np.unique(table.real.astype(np.float32))
    mids = ((lv[:-1] + lv[1:]) / np.float32(2)).astype(np.float32)
    axis = [lv, mids]
    for k in (1, 2, 3):
        axis.append(np.nextafter(mids, np.float32(np.inf)).astype(np.float32))
        axis.append(np.nextafter(mids, np.float32(-np.inf)).astype(np.float32))
        mids = np.nextafter(mids, np.float32(np.inf)).astype(np.float32)
    axis.append(np.array([lv[0] * 1.2, lv[-1] * 1.2, 0.0, -0.0], dtype=np.float32))
    ax = np.unique(np.concatenate(axis)).astype(np.float32)
    re, im = np.meshgrid(ax, ax)
    x = (re.ravel() + 1j * im.ravel()).astype(np.complex64)
    got = ops.qpsk256_demodulate(dev(x, cuda), 0).cpu().numpy()
    assert np.array_equal(got, o.qpsk256_demod(table, x))


@pytest.mark.parametrize("amp", [1.0, 0.37, -2.5])
def test_qpsk256_rect_quick_path_margin(cuda, amp):
    """The quick per-axis decision (qpsk256.hip demod_rect_quick) accepts a symbol only when its level coordinate u
    is more than 2^-10 of a level spacing from every midpoint: symbols on a dense grid across that margin on both
    sides of every midpoint, at the 4|a| edge and just beyond it, decide bit for bit as the exhaustive oracle."""
    from gsdr_amd import ops

    ops.qpsk256_init(0, amp)
    table = o.qpsk256_table(0, amp)
    lv = np.unique(table.real.astype(np.float32)).astype(np.float64)
    sp = (lv[-1] - lv[0]) / 15.0
    mids = (lv[:-1] + lv[1:]) / 2
    offs = np.concatenate([np.linspace(-3, 3, 61) * 2.0 ** -10, np.array([-0.02, 0.02, 0.3, -0.3])]) * sp
    ax = (mids[:, None] + offs[None, :]).ravel()
    edge = 4.0 * abs(amp)
    ax = np.concatenate([ax, [edge, -edge, np.nextafter(np.float32(edge), np.float32(np.inf)), -edge * 1.0001]])
    ax = np.unique(ax.astype(np.float32))
    re, im = np.meshgrid(ax, ax)
    x = (re.ravel() + 1j * im.ravel()).astype(np.complex64)
    got = ops.qpsk256_demodulate(dev(x, cuda), 0).cpu().numpy()
    assert np.array_equal(got, o.qpsk256_demod(table, x))


@pytest.mark.parametrize("n", [1, 5, 6, 7, 385, 4607, 4609, 3 * 4608 + 385, 100_003])
@pytest.mark.parametrize("first", [0, 1, 2, 2**33 + 3])
@pytest.mark.parametrize("ctype", [0, 1])
def test_qpsk256_fused_round_trip_equals_two_calls(cuda, n, first, ctype):
    """gsdrxQpsk256ModulateAwgnDemodulate writes exactly what gsdrxQpsk256ModulateAwgn followed by
    gsdrQpsk256Demodulate write: the same noisy symbols and the same decisions, bit for bit (rectangular: one fused
    kernel; circular: the two calls), at every size (partial waves and workgroups, n < 6) and residue of the first
    index mod 3; the decisions also equal the oracle's exhaustive cuCabsf argmin on the noisy symbols."""
    from gsdr_amd import ops

    sigma, seed = (0.05, 0x5EED0005) if ctype == 0 else (0.02, 0xFEED)
    ops.qpsk256_init(ctype, 1.0)
    syms_np = np.random.default_rng(n + first).integers(0, 256, n, dtype=np.uint8)
    syms = dev(syms_np, cuda)
    rx2 = ops.qpsk256_modulate_awgn(syms, ctype, sigma, seed, first)
    dec2 = ops.qpsk256_demodulate(rx2, ctype)
    rx1, dec1 = ops.qpsk256_modulate_awgn_demodulate(syms, ctype, sigma, seed, first)
    assert rx1.cpu().numpy().tobytes() == rx2.cpu().numpy().tobytes()
    assert torch.equal(dec1, dec2)
    table = o.qpsk256_table(ctype, 1.0)
    assert np.array_equal(dec1.cpu().numpy(), o.qpsk256_demod(table, rx1.cpu().numpy()))


@pytest.mark.parametrize("in_off,noisy_off,dec_off", [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)])
def test_qpsk256_fused_round_trip_pointer_alignment(cuda, in_off, noisy_off, dec_off):
    """Odd symbol bytes, noisy symbols 8 bytes off 16-byte alignment, odd decision bytes: the per-symbol path, same
    bits as the two calls."""
    from gsdr_amd import ops

    ops.qpsk256_init(0, 1.0)
    n = 2 * 4608 + 390
    syms_np = np.random.default_rng(in_off + 2 * noisy_off + 4 * dec_off).integers(0, 256, n + 4, dtype=np.uint8)
    syms = dev(syms_np, cuda)[in_off:in_off + n]
    noisy = torch.empty(n + 1, dtype=torch.complex64, device=cuda)[noisy_off:noisy_off + n]
    dec = torch.empty(n + 1, dtype=torch.uint8, device=cuda)[dec_off:dec_off + n]
    ops.qpsk256_modulate_awgn_demodulate(syms, 0, 0.03, 77, 11, noisy=noisy, out=dec)
    rx2 = ops.qpsk256_modulate_awgn(syms, 0, 0.03, 77, 11)
    assert noisy.cpu().numpy().tobytes() == rx2.cpu().numpy().tobytes()
    assert torch.equal(dec, ops.qpsk256_demodulate(rx2, 0))


def test_qpsk256_fused_config5_bit_exact(cuda):
    """BASELINE config 5 through the fused entry point: all 2^24 noisy symbols and decisions equal the oracle's
    (restated channel + exhaustive cuCabsf argmin), and the two-call results."""
    from gsdr_amd import ops

    n, seed, first, sigma = 1 << 24, 0x5EED_0005, 0, 0.02
    ops.qpsk256_init(0, 1.0)
    g = torch.Generator(device=cuda).manual_seed(0x5EED5)
    syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=cuda, generator=g)
    rx, dec = ops.qpsk256_modulate_awgn_demodulate(syms, 0, sigma, seed, first)
    assert torch.equal(dec, ops.qpsk256_demodulate(rx, 0))
    table = o.qpsk256_table(0, 1.0)
    syms_np, rx_np = syms.cpu().numpy(), rx.cpu().numpy()
    assert rx_np.tobytes() == o.qpsk256_mod_awgn(table, syms_np, sigma, seed, first, nthreads=_threads()).tobytes()
    assert np.array_equal(dec.cpu().numpy(), o.qpsk256_demod(table, rx_np, nthreads=_threads()))
    ser = float((dec != syms).float().mean())
    assert 1e-4 < ser < 1e-2
