"""GPU parity: the element-wise ABI (gsdrAddConst*, gsdrMultiply*, gsdrAddToMagnitude, gsdrAbs,
gsdrInt8ToNormFloat, gsdrCosine*) vs the C oracle. Exact maps are compared bit for bit (same
per-operation IEEE rounding on both sides); hypot / cos / sin go through device vs host libm and
are compared within a few ulp. Sizes follow the reference's tests/test_arithmetic.cpp:256-273."""
import numpy as np
import pytest
import torch

from oracle import oracle as o

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 4, 7, 8, 9, 31, 32, 33, 1023, 1024, 1025, (1 << 20) + 5]


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def same_bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def rand_f(n, seed):
    return np.random.default_rng(seed).uniform(-10, 10, n).astype(np.float32)


def rand_c(n, seed):
    r = np.random.default_rng(seed)
    return (r.uniform(-10, 10, n) + 1j * r.uniform(-10, 10, n)).astype(np.complex64)


@pytest.mark.parametrize("n", SIZES)
def test_add_const_bit_exact(cuda, n):
    from gsdr_amd import ops

    x, xc = rand_f(n, n), rand_c(n, n + 1)
    for inp, c in ((x, 3.14), (xc, 1.5 - 2.5j), (xc, -1.23), (x, 2.5 - 1.5j)):
        got = host(ops.add_const(dev(inp, cuda), c))
        assert same_bits(got, o.add_const(inp, c)), (inp.dtype, c)


@pytest.mark.parametrize("n", SIZES)
def test_multiply_bit_exact(cuda, n):
    from gsdr_amd import ops

    a, b, ac, bc = rand_f(n, n), rand_f(n, n + 1), rand_c(n, n + 2), rand_c(n, n + 3)
    for p, q in ((ac, bc), (a, b), (ac, b)):
        assert same_bits(host(ops.multiply(dev(p, cuda), dev(q, cuda))), o.multiply(p, q))


@pytest.mark.parametrize("n", SIZES)
def test_abs_int8_bit_exact(cuda, n):
    from gsdr_amd import ops

    x = rand_f(n, n)
    x[: min(n, 4)] = np.array([0.0, -0.0, -np.inf, np.nan], np.float32)[: min(n, 4)]
    assert same_bits(host(ops.abs_(dev(x, cuda))), o.abs_(x))
    i8 = np.random.default_rng(n).integers(-128, 128, n, dtype=np.int8)
    assert same_bits(host(ops.int8_to_norm_float(dev(i8, cuda))), o.int8_to_float(i8))


def test_int8_all_values(cuda):
    from gsdr_amd import ops

    i8 = np.arange(-128, 128, dtype=np.int8)
    got = host(ops.int8_to_norm_float(dev(i8, cuda)))
    assert same_bits(got, o.int8_to_float(i8))
    assert got[0] == -1.0 and got[1] == -1.0 and got[128] == 0.0 and got[255] == 1.0


@pytest.mark.parametrize("n", SIZES)
def test_add_to_magnitude(cuda, n):
    from gsdr_amd import ops

    x = rand_c(n, n)
    got = host(ops.add_to_magnitude(dev(x, cuda), 2.5))
    want = o.add_to_magnitude(x, 2.5)
    assert np.max(np.abs(got - want) / np.abs(want)) < 1e-6


def test_add_to_magnitude_zero_is_nan(cuda):
    from gsdr_amd import ops

    got = host(ops.add_to_magnitude(dev(np.zeros(3, np.complex64), cuda), 1.0))
    assert np.all(np.isnan(got.real)) and np.all(np.isnan(got.imag))  # 0 / |0| as the reference


@pytest.mark.parametrize("n", [1, 5, 1023, 1025, 65536, (1 << 20) + 5])
@pytest.mark.parametrize("rng", [(0.0, 2 * np.pi), (-np.pi, np.pi), (-1.3, 40.0), (100.0, -2000.0)])
def test_cosine(cuda, n, rng):
    from gsdr_amd import ops

    for cplx in (True, False):
        got = host(ops.cosine(rng[0], rng[1], n, complex_out=cplx, device=cuda))
        want = o.cosine(rng[0], rng[1], n, cplx)
        assert np.max(np.abs(got - want)) < 1e-6, cplx


def test_unaligned_pointers(cuda):
    from gsdr_amd import ops

    n = 4099
    x = rand_c(n + 1, 7)
    xt = dev(x, cuda)[1:]  # 8-byte aligned, not 16
    y = rand_f(n + 1, 8)
    yt = dev(y, cuda)[1:]
    out = torch.empty(n + 1, dtype=torch.complex64, device=cuda)[1:]
    ops.multiply(xt, yt, out=out)
    assert same_bits(host(out), o.multiply(x[1:], y[1:]))
    outf = torch.empty(n + 3, dtype=torch.float32, device=cuda)[3:]
    ops.add_const(yt, 1.25, out=outf)
    assert same_bits(host(outf), o.add_const(y[1:], 1.25))


def test_exactly_n_written_and_zero_length(cuda):
    from gsdr_amd import abi, ops

    n = 1000
    out = torch.full((n + 16,), 7.0, dtype=torch.float32, device=cuda)
    ops.abs_(dev(rand_f(n, 1), cuda), out=out[:n])
    assert np.all(host(out)[n:] == 7.0)  # the reference also wrote out[n]
    st = torch.cuda.current_stream(cuda).cuda_stream
    assert abi.lib.gsdrAbs(None, None, 0, cuda.index, st) == 0
    assert abi.lib.gsdrCosineF(0.0, 1.0, None, 0, cuda.index, st) == 0
    assert abi.lib.gsdrAbs(None, out.data_ptr(), 4, cuda.index, st) != 0
