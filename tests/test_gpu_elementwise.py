"""GPU parity: gsdrQuadFmDemod / gsdrQuadAmDemod / gsdrMagnitude vs the C oracle
(reference src/quad_demod.cu:23-74, src/magnitude.cu:20-45; tests/test_quad_demod.cpp)."""
import numpy as np
import pytest
import torch

from helpers import FLOAT_TOL, wrapped_angle_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu


def dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


SIZES = [1, 2, 3, 4, 5, 1023, 1024, 1025, (1 << 20) + 3]


@pytest.mark.parametrize("n", SIZES)
def test_quad_fm_parity(cuda, n):
    from gsdr_amd import ops
    from gsdr_amd.signals import fm_test_signal

    x = fm_test_signal(n + 1, noise=0.02, seed=n)
    out = ops.quad_fm_demod(dev(x, cuda), 1.7)
    torch.cuda.synchronize()
    assert wrapped_angle_err(out.cpu().numpy(), o.quad_fm(x, 1.7), 1.7) <= FLOAT_TOL


@pytest.mark.parametrize("n", SIZES)
def test_quad_am_and_magnitude_parity(cuda, n):
    from gsdr_amd import ops
    from gsdr_amd.signals import uniform_iq

    x = uniform_iq(n, seed=n)
    xt = dev(x, cuda)
    am = ops.quad_am_demod(xt)
    mag = ops.magnitude(xt)
    torch.cuda.synchronize()
    assert np.max(np.abs(am.cpu().numpy() - o.quad_am(x))) <= FLOAT_TOL
    ref = o.magnitude(x)
    assert np.max(np.abs(mag.cpu().numpy() - ref) / np.maximum(ref, 1e-30)) <= FLOAT_TOL


def test_quad_unaligned_pointers(cuda):
    from gsdr_amd import ops
    from gsdr_amd.signals import uniform_iq

    x = uniform_iq(5001, seed=4)
    xt = dev(x, cuda)
    out = torch.empty(5003, dtype=torch.float32, device=cuda)
    ops.quad_fm_demod(xt[1:], 1.0, out=out[1:5000])
    ops.quad_am_demod(xt[1:], out=out[1:5001])
    torch.cuda.synchronize()
    assert np.max(np.abs(out[1:5001].cpu().numpy() - o.quad_am(x[1:]))) <= FLOAT_TOL


def test_quad_zero_input(cuda):
    """reference tests/test_quad_demod.cpp:248-263: zero input -> zero output (atan2(0, 0) = 0)."""
    from gsdr_amd import ops

    out = ops.quad_fm_demod(torch.zeros(4097, dtype=torch.complex64, device=cuda), 1.0)
    torch.cuda.synchronize()
    assert torch.all(out == 0)


def test_quad_constant_frequency(cuda):
    """reference tests/test_quad_demod.cpp:99-115 input (0.1 cycles/sample tone); correct answer is
    the constant 2 pi 0.1 (the test's '< 0.1' expectation is wrong)."""
    from gsdr_amd import ops

    x = np.exp(2j * np.pi * 0.1 * np.arange(65537)).astype(np.complex64)
    out = ops.quad_fm_demod(dev(x, cuda), 1.0)
    torch.cuda.synchronize()
    assert np.max(np.abs(out.cpu().numpy() - 2 * np.pi * 0.1)) < 1e-5


def test_am_saturation_and_nan(cuda):
    """2 * saturate(|x|) - 1 with saturate(NaN) = 0 (quad_demod.cu:47-48)."""
    from gsdr_amd import ops

    x = np.array([0, 0.5, 1.0, 3.0 + 4.0j, complex(np.nan, 0), complex(np.inf, 0)], dtype=np.complex64)
    out = ops.quad_am_demod(dev(x, cuda)).cpu().numpy()
    assert np.array_equal(out, o.quad_am(x)) and np.array_equal(out[:4], [-1.0, 0.0, 1.0, 1.0])
    assert out[4] == -1.0 and out[5] == 1.0
