"""CPU: the oracle's config-5 channel model and the reference's QPSK256 decision rule.

* Philox4x32-10 against the published known-answer vectors of the Random123 distribution
  (Salmon et al., SC'11; kat_vectors, philox4x32 with 10 rounds).
* The Box-Muller normals (own ln / sin / cos polynomials, no libm) against a float64 evaluation of
  the same formula from the same Philox words, and their distribution (moments, Kolmogorov-Smirnov).
* cuCabsf (CUDA cuComplex.h, with nvcc's default fmaf contraction) against float64 hypot, and the
  cuCabsf argmin rule (qpsk256.cu:171-181) against the squared-distance rule on random points."""
import math

import numpy as np
import pytest

from oracle import oracle as o

KAT = [
    ([0x00000000] * 4, [0x00000000] * 2, [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(ctr, key, want):
    assert [int(v) for v in o.philox4x32_10(ctr, key)] == want


def _ref_normals(seed, k):
    blk, slot = divmod(k, 3)  # three symbols per Philox block, 39 bits each (gsdr_amd/csrc/awgn.hpp)
    w = [int(v) for v in o.philox4x32_10([blk & 0xffffffff, blk >> 32, 0, 0], [seed & 0xffffffff, seed >> 32])]
    a, b = [(w[0] >> 9, w[3] & 0xffff), (w[1] >> 9, w[3] >> 16),
            (w[2] >> 9, ((w[0] & 0x1ff) << 7) | (w[1] & 0x7f))][slot]
    u1 = (a + 0.5) * 2.0 ** -23
    u2 = b * 2.0 ** -16
    r = math.sqrt(-2.0 * math.log(u1))
    return r * math.cos(2 * math.pi * u2), r * math.sin(2 * math.pi * u2)


def test_awgn_normals_match_float64_box_muller():
    seed = 0x1234_5678_9ABC_DEF0
    worst = 0.0
    for k in list(range(2000)) + [2**32 - 1, 2**32, 2**40 + 3, 2**63 + 7]:
        g = o.awgn_normals(seed, k)
        want = _ref_normals(seed, k)
        for a, b in zip(g, want):
            worst = max(worst, abs(a - b) / max(1.0, abs(b)))
    assert worst < 2e-6, worst


def test_awgn_distribution():
    from scipy import stats

    table = o.qpsk256_table(0, 1.0)
    n = 400_000
    sym = np.zeros(n, np.uint8)
    x = o.qpsk256_mod_awgn(table, sym, 1.0, seed=99, first_symbol=12345, nthreads=4) - table[0]
    for v in (x.real.astype(np.float64), x.imag.astype(np.float64)):
        assert abs(v.mean()) < 0.01 and abs(v.var() - 1.0) < 0.01
        assert abs(stats.kurtosis(v)) < 0.05 and abs(stats.skew(v)) < 0.02
        assert stats.kstest(v, "norm").pvalue > 1e-3
    # I and Q independent
    assert abs(np.corrcoef(x.real, x.imag)[0, 1]) < 0.01


def test_awgn_is_a_function_of_the_absolute_symbol_index():
    table = o.qpsk256_table(1, 0.8)
    sym = np.random.default_rng(1).integers(0, 256, 1001, dtype=np.uint8)
    whole = o.qpsk256_mod_awgn(table, sym, 0.05, seed=7, first_symbol=999)
    part = o.qpsk256_mod_awgn(table, sym[333:], 0.05, seed=7, first_symbol=999 + 333)
    assert whole[333:].tobytes() == part.tobytes()
    mt = o.qpsk256_mod_awgn(table, sym, 0.05, seed=7, first_symbol=999, nthreads=3)
    assert mt.tobytes() == whole.tobytes()


def test_cucabsf_against_float64():
    rng = np.random.default_rng(5)
    v = rng.standard_normal((20000, 2)).astype(np.float32) * np.float32(3.0)
    for re, im in v:
        want = math.hypot(float(re), float(im))
        got = o.cuCabsf(float(re), float(im))
        assert abs(got - want) <= 3 * np.spacing(np.float32(want))
    assert o.cuCabsf(0.0, 0.0) == 0.0
    assert o.cuCabsf(float("inf"), 1.0) == float("inf") and o.cuCabsf(-3.0, float("inf")) == float("inf")
    assert math.isnan(o.cuCabsf(float("nan"), 1.0))


@pytest.mark.parametrize("ctype,amp", [(0, 1.0), (1, 1.0), (1, 0.37)])
def test_cuabs_rule_close_to_squared_distance(ctype, amp):
    """The two rules pick the same point except at near-ties; both are the first index of their
    minimum, strict <."""
    table = o.qpsk256_table(ctype, amp)
    rng = np.random.default_rng(ctype)
    x = (rng.uniform(-1.2, 1.2, (50000, 2)) * amp).astype(np.float32).view(np.complex64).ravel()
    a = o.qpsk256_demod(table, x, "sq", nthreads=4)
    b = o.qpsk256_demod(table, x, "cuabs", nthreads=4)
    assert np.array_equal(b, o.qpsk256_demod(table, x, "cuabs"))
    assert np.count_nonzero(a != b) <= 5
