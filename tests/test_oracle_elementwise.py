"""CPU: the element-wise oracle (oracle/gsdr_oracle.c) against the independent numpy fixture
tests/golden/elementwise.npz, and the reference's own known answers
(tests/test_arithmetic.cpp, tests/test_conversion.cpp, tests/test_trig.cpp in kernrj/gsdr)."""
import os

import numpy as np
import pytest

from oracle import oracle as o

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "elementwise.npz"))


def same_bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def test_add_const_golden_bit_exact():
    cf, cc = float(G["cf"][0]), complex(G["cc"][0])
    assert same_bits(o.add_const(G["x"], cf), G["add_ff"])
    assert same_bits(o.add_const(G["xc"], cc), G["add_cc"])
    assert same_bits(o.add_const(G["xc"], cf), G["add_cf"])
    assert same_bits(o.add_const(G["x"], cc), G["add_fc"])


def test_multiply_golden_bit_exact():
    assert same_bits(o.multiply(G["xc"], G["yc"]), G["mul_cc"])
    assert same_bits(o.multiply(G["x"], G["y"]), G["mul_ff"])
    assert same_bits(o.multiply(G["xc"], G["y"]), G["mul_cf"])


def test_abs_and_int8_golden_bit_exact():
    assert same_bits(o.abs_(G["x"]), G["abs"])
    assert same_bits(o.int8_to_float(G["i8"]), G["conv"])


def test_add_to_magnitude_golden():
    got = o.add_to_magnitude(G["xc"], float(G["a2m_c"][0]))
    want = G["a2m"]
    assert np.max(np.abs(got - want) / np.abs(want)) < 4e-7


def test_cosine_golden():
    phi0, phi1 = (float(v) for v in G["phi"])
    want = G["cos_c"]
    got = o.cosine(phi0, phi1, want.size, True)
    assert np.max(np.abs(got - want)) < 5e-7
    assert same_bits(o.cosine(phi0, phi1, want.size, False), got.real.copy())


# ---- the reference's known answers ----------------------------------------------------------

def test_ref_int8_edge_cases():
    # tests/test_conversion.cpp:63-77 and :108-124
    out = o.int8_to_float(np.array([-128, -127, -1, 0, 1, 126, 127], np.int8))
    assert out[0] == -1.0 and out[1] == -1.0 and out[3] == 0.0 and out[6] == 1.0
    assert abs(out[5] - 1.0) < 1e-2 and out[5] == np.float32(126) / np.float32(127)
    out = o.int8_to_float(np.array([0, 1, -1, 64, -64, 127, -128], np.int8))
    assert out[0] == 0.0 and out[6] == -1.0
    assert np.allclose(out[1:6], np.array([1, -1, 64, -64, 127]) / 127.0, atol=1e-6)


def test_ref_abs_special_values():
    # tests/test_arithmetic.cpp:289-305
    out = o.abs_(np.array([0.0, 1.0, -1.0, np.inf, -np.inf, np.nan], np.float32))
    assert list(out[:5]) == [0.0, 1.0, 1.0, np.inf, np.inf] and np.isnan(out[5])


def test_ref_zero_input_and_large_numbers():
    # tests/test_arithmetic.cpp:234-253 and :275-287
    z = np.zeros(1000, np.float32)
    assert np.all(o.add_const(z, 5.0) == 5.0)
    assert np.all(o.multiply(z, np.ones(1000, np.float32)) == 0.0)
    big = np.full(1000, 1e6, np.float32)
    assert np.allclose(o.multiply(big, big), 1e12, atol=1e6)


def test_ref_add_to_magnitude_keeps_phase():
    # tests/test_arithmetic.cpp:208-232
    rng = np.random.default_rng(3)
    x = (rng.uniform(-1, 1, 1000) + 1j * rng.uniform(-1, 1, 1000)).astype(np.complex64)
    out = o.add_to_magnitude(x, 2.5)
    assert np.allclose(np.abs(out), np.abs(x) + 2.5, atol=1e-5)
    assert np.allclose(np.angle(out), np.angle(x), atol=1e-5)


def test_ref_add_const_cf_adds_to_real_part_only():
    # the reference's operator+(cuComplex, float) (src/cuComplexOperatorOverloads.cuh:50-52) touches
    # the real part only; its tests/test_arithmetic.cpp:100 expects both parts -- this build returns
    # what the reference computes.
    out = o.add_const(np.array([1 + 2j], np.complex64), -1.23)
    assert out[0] == np.complex64(complex(np.float32(1) + np.float32(-1.23), 2))
    out = o.add_const(np.array([1.0], np.float32), 2.5 - 1.5j)
    assert out[0] == np.complex64(3.5 - 1.5j)


@pytest.mark.parametrize("complex_out", [True, False])
def test_ref_cosine_ramp(complex_out):
    # tests/test_trig.cpp: a full period over n samples starts at cos(phi0)
    out = o.cosine(0.0, 2 * np.pi, 1024, complex_out)
    k = np.arange(1024)
    want = np.exp(1j * 2 * np.pi * k / 1024)
    if not complex_out:
        want = want.real
    assert np.max(np.abs(out - want)) < 2e-6
