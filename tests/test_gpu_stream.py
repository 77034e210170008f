"""GPU: the streaming object (include/gsdr/stream.h) -- chunked processing with random chunk sizes
(0, 1, shorter than the window, longer than many tiles) concatenates to exactly the outputs of one
monolithic call of the underlying entry point, bit for bit, for FIR / FM / AM, float and int8 I/Q,
with the NCO phase carried through the absolute sample index."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FS, TUNE, CHAN, DEV = 1.0e6, 0.0, 1.0e5, 2.0e4


def chunks(total, seed, W):
    rng = np.random.default_rng(seed)
    sizes = []
    while sum(sizes) < total:
        sizes.append(int(rng.choice([0, 1, 2, W - 1, W + 3, int(rng.integers(1, 3 * W)), int(rng.integers(1, 40000))])))
    sizes[-1] -= sum(sizes) - total
    return sizes


def monolithic(kind, x, taps, D, n0, int8):
    from gsdr_amd import ops

    # int8: the gsdrx*Int8 defaults, the decimation-4 matrix-core kernels included (their summation blocks
    # follow the absolute output index, so the stream's chunk launches reproduce the one call)
    if kind == "fir":
        return ops.fir(taps, x, D)
    if kind == "fm":
        return ops.fm_demod(x, taps, FS, TUNE, CHAN, DEV, D, n0)
    return ops.am_demod(x, taps, FS, TUNE, CHAN, D, n0)


@pytest.mark.parametrize("kind", ["fir", "fm", "am"])
@pytest.mark.parametrize("D", [1, 3, 4, 8])
@pytest.mark.parametrize("int8", [False, True])
def test_chunked_equals_monolithic(cuda, kind, D, int8):
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    T, n0 = 127, 4_000_000_123
    L = 150_000 + 7 * D
    x = fm_test_signal(L, noise=0.02, n0=n0)
    if int8:
        xh = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
        per = 2
    else:
        xh, per = x, 1
    xd = torch.from_numpy(xh).to(cuda)
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    want = monolithic(kind, xd, taps, D, n0, int8)
    s = Stream(kind, taps, D, FS, TUNE, CHAN, DEV, first_sample_index=n0, int8=int8)
    W = T + D if kind == "fm" else T
    parts, pos = [], 0
    for m in chunks(L, seed=D * 10 + len(kind) + int8, W=W):
        parts.append(s.process(xd[pos * per:(pos + m) * per]).clone())
        pos += m
    s.close()
    got = torch.cat(parts)
    torch.cuda.synchronize()
    assert got.numel() == want.numel()
    assert torch.equal(got.view(torch.float32), want.view(torch.float32))


@pytest.mark.parametrize("kind,D,T,L,nchunks", [
    ("fir", 4, 127, 20_000_000, 7),   # monolithic on 1,024-output tiles, the calls on 512-output tiles
    ("fm", 4, 127, 12_000_000, 5),
    ("fm", 4, 127, 20_000_000, 5),    # monolithic FM / AM above the R = 4 threshold too
    ("am", 4, 127, 20_000_000, 6),
    ("am", 9, 127, 400_000, 6),       # runtime-decimation kernel: the three-launch seam plan
    ("fir", 4, 300, 600_000, 4),      # longer filter, two tap chunks more
    ("fir", 2, 127, 600_000, 9),
])
def test_one_launch_calls_equal_monolithic(cuda, kind, D, T, L, nchunks):
    """Round 4: every float stream call on the tiled kernels is ONE launch (seam samples read from the
    history buffer, next history copied by the launch). Large calls whose tile shape differs from the
    monolithic call's (the per-output MAC order depends only on D and JC), a shape that keeps the seam plan
    (D = 9), and a long filter: concatenated outputs equal one call bit for bit."""
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    n0 = 77_777
    x = fm_test_signal(L, noise=0.02, n0=n0)
    xd = torch.from_numpy(x).to(cuda)
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    if L >= 20_000_000:
        # the monolithic call must run the 1,024-output (R = 4) tiles: launch_poly_d4 keeps R = 2 below
        # 3 * CUs * 4 tiles of 1,024 outputs
        cus = torch.cuda.get_device_properties(cuda).multi_processor_count
        assert -(-(L // D) // 1024) > 3 * cus * 4, (L, cus)
    want = monolithic(kind, xd, taps, D, n0, False)
    s = Stream(kind, taps, D, FS, TUNE, CHAN, DEV, first_sample_index=n0)
    rng = np.random.default_rng(L + D)
    cuts = np.sort(rng.choice(np.arange(1, L), nchunks - 1, replace=False))
    bounds = [0, *cuts.tolist(), L]
    got = torch.cat([s.process(xd[a:b]).clone() for a, b in zip(bounds[:-1], bounds[1:])])
    s.close()
    torch.cuda.synchronize()
    assert got.numel() == want.numel()
    assert torch.equal(got.view(torch.float32), want.view(torch.float32))


def test_tiny_chunks_and_skipping_decimation(cuda):
    """D > W: outputs skip samples; one-sample chunks throughout."""
    from gsdr_amd import ops
    from gsdr_amd.signals import uniform_iq
    from gsdr_amd.stream import Stream

    D, T = 16, 5
    x = torch.from_numpy(uniform_iq(2000, seed=3)).to(cuda)
    taps = torch.tensor([0.1, -0.2, 0.3, 0.25, 0.05], device=cuda)
    want = ops.fir(taps, x, D)
    s = Stream("fir", taps, D)
    got = torch.cat([s.process(x[i:i + 1]).clone() for i in range(x.numel())])
    assert torch.equal(got.view(torch.float32), want.view(torch.float32))


def test_create_validation(cuda):
    import ctypes

    from gsdr_amd import abi

    h = ctypes.c_void_p()
    taps = torch.ones(4, device=cuda)
    assert abi.lib.gsdrxStreamCreate(ctypes.byref(h), 0, 0, 0, taps.data_ptr(), 4, 1.0, 0.0, 0.0, 1.0, 0, 0) != 0
    assert abi.lib.gsdrxStreamCreate(ctypes.byref(h), 7, 0, 2, taps.data_ptr(), 4, 1.0, 0.0, 0.0, 1.0, 0, 0) != 0
    assert abi.lib.gsdrxStreamCreate(ctypes.byref(h), 0, 0, 2, None, 4, 1.0, 0.0, 0.0, 1.0, 0, 0) != 0
    assert abi.lib.gsdrxStreamDestroy(None) == 0


# Multi-channel streams (gsdrxStreamCreateMulti, SURVEY.md 8(f) rows 1 x 3): C channels of one RF input, one
# shared history; channel c must equal its own single-channel stream and one monolithic call, bit for bit.
MCH = [1.0e5, -2.5e5, 3.3e4, 0.0, -4.4e5, 1.7e5, 2.9e5, -1.1e5, 4.0e5, -3.0e5, 6.0e4, -6.0e4, 2.2e5, -2.2e5, 1.3e5,
       -1.3e5, 3.7e5, -3.7e5, 9.0e3]


@pytest.mark.parametrize("kind", ["fm", "am"])
@pytest.mark.parametrize("int8", [False, True])
@pytest.mark.parametrize("D,C", [(4, 3), (4, 17), (2, 5), (8, 2), (3, 4), (9, 3)])
def test_multi_stream_equals_single_streams(cuda, kind, int8, D, C):
    """D = 2 / 4 / 8 complex float: the grouped kernel (17 channels: two launches a call, the second without the
    history copy); int8 at D = 4: per-channel matrix-core chains; D = 3: per-channel tiled steps; D = 9: the
    shared seam plan (one gather, then each channel's two filter calls)."""
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    T, n0 = 127, 4_000_000_123
    L = 120_000 + 7 * D
    x = fm_test_signal(L, noise=0.02, n0=n0)
    if int8:
        xh = np.clip(np.round(np.stack([x.real, x.imag], 1).ravel() * 100), -128, 127).astype(np.int8)
        per = 2
    else:
        xh, per = x, 1
    xd = torch.from_numpy(xh).to(cuda)
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    chans = MCH[:C]
    devs = [DEV * (1 + 0.1 * c) for c in range(C)]
    ms = Stream(kind, taps, D, FS, TUNE, chans, devs, first_sample_index=n0, int8=int8)
    W = T + D if kind == "fm" else T
    parts, pos = [], 0
    sizes = chunks(L, seed=D * 100 + C + int8, W=W)
    for m in sizes:
        parts.append(ms.process(xd[pos * per:(pos + m) * per]).clone())
        pos += m
    ms.close()
    got = torch.cat(parts, dim=1)
    torch.cuda.synchronize()
    for c in range(C):
        s = Stream(kind, taps, D, FS, TUNE, chans[c], devs[c], first_sample_index=n0, int8=int8)
        single, pos = [], 0
        for m in sizes:
            single.append(s.process(xd[pos * per:(pos + m) * per]).clone())
            pos += m
        s.close()
        want = torch.cat(single)
        assert got.shape[1] == want.numel(), (c, got.shape, want.numel())
        assert torch.equal(got[c].view(torch.int32), want.view(torch.int32)), c
    # and the first and last channels against one monolithic call
    from gsdr_amd import ops

    for c in (0, C - 1):
        if kind == "fm":
            mono = ops.fm_demod(xd, taps, FS, TUNE, chans[c], devs[c], D, n0)
        else:
            mono = ops.am_demod(xd, taps, FS, TUNE, chans[c], D, n0)
        assert torch.equal(got[c].view(torch.int32), mono.view(torch.int32)), c


def test_multi_stream_output_stride_and_validation(cuda):
    """Channel c's outputs land at output + c * outputCapacity (a caller's fixed per-channel buffers), the rest of
    each row untouched; FIR kind, zero channels and a null deviation list for FM are refused."""
    import ctypes

    from gsdr_amd.abi import lib
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from gsdr_amd.stream import Stream

    T, D = 63, 4
    taps = torch.from_numpy(lowpass_taps(T)).to(cuda)
    x = torch.from_numpy(fm_test_signal(50_000, noise=0.02)).to(cuda)
    s = Stream("fm", taps, D, FS, TUNE, [1e5, -1e5, 2e5], [DEV] * 3)
    cap = 20_000
    out = torch.full((3, cap), 7.0, device=cuda)
    y = s.process(x, out=out)
    n = y.shape[1]
    assert n == (50_000 - T - D) // D + 1 and n < cap
    assert torch.all(out[:, n:] == 7.0)
    for c, f in enumerate([1e5, -1e5, 2e5]):
        from gsdr_amd import ops

        assert torch.equal(out[c, :n], ops.fm_demod(x, taps, FS, TUNE, f, DEV, D, 0, n))
    s.close()
    h = ctypes.c_void_p()
    f2 = (ctypes.c_float * 2)(1e5, 2e5)
    p = ctypes.cast(f2, ctypes.c_void_p)
    assert lib.gsdrxStreamCreateMulti(ctypes.byref(h), 0, 0, 4, taps.data_ptr(), T, FS, 0.0, p, p, 2, 0, 0) != 0
    assert lib.gsdrxStreamCreateMulti(ctypes.byref(h), 1, 0, 4, taps.data_ptr(), T, FS, 0.0, p, p, 0, 0, 0) != 0
    assert lib.gsdrxStreamCreateMulti(ctypes.byref(h), 1, 0, 4, taps.data_ptr(), T, FS, 0.0, p, None, 2, 0, 0) != 0
    assert lib.gsdrxStreamCreateMulti(ctypes.byref(h), 2, 0, 4, taps.data_ptr(), T, FS, 0.0, p, None, 2, 0, 0) == 0
    assert lib.gsdrxStreamDestroy(h) == 0
