"""ctypes binding of the C oracle (oracle/gsdr_oracle.c) for numpy arrays -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker or as the timed CPU baseline. Complex arrays are numpy complex64 (interleaved
float pairs, the hipFloatComplex layout).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

# GSDR_ORACLE_LIB: another build of the same C source (bench.py's cpu_baseline builds one tuned for the
# host it runs on); the default is the in-tree build.
LIB_PATH = os.environ.get("GSDR_ORACLE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "build",
                                                             "liboracle.so")
if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} missing: run `make oracle/build/liboracle.so`")
_lib = ctypes.CDLL(LIB_PATH)

_p, _sz, _u32, _u64, _f, _int = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64,
                                 ctypes.c_float, ctypes.c_int)
_SIG = {
    "oracle_fir_ff": [_sz, _p, _sz, _p, _p, _sz, _sz],
    "oracle_fir_fc": [_sz, _p, _sz, _p, _p, _sz, _sz],
    "oracle_fir_cc": [_sz, _p, _sz, _p, _p, _sz, _sz],
    "oracle_fir_cf": [_sz, _p, _sz, _p, _p, _sz, _sz],
    "oracle_fir_fc_mt": [_sz, _p, _sz, _p, _p, _sz, _int],
    "oracle_fir_bound_fc": [_sz, _p, _sz, _p, _p, _sz, _sz],
    "oracle_nco_mix": [_p, _p, _u64, _u32, _sz, _sz],
    "oracle_fm_demod": [_f, _f, _f, _f, _u32, _u64, _p, _sz, _p, _p, _sz, _sz],
    "oracle_am_demod": [_f, _f, _f, _u32, _u64, _p, _sz, _p, _p, _sz, _sz],
    "oracle_chain_fir": [_f, _f, _f, _u32, _u64, _p, _sz, _p, _p, _sz, _sz],
    "oracle_quad_fm": [_p, _p, _f, _sz],
    "oracle_quad_am": [_p, _p, _sz],
    "oracle_magnitude": [_p, _p, _sz],
    "oracle_qpsk_mod": [_p, _p, _u32, _f],
    "oracle_qpsk_demod": [_p, _p, _u32],
    "oracle_qpsk256_table": [_u32, _f, _p],
    "oracle_qpsk256_mod": [_p, _p, _p, _u32],
    "oracle_qpsk256_demod": [_p, _p, _p, _u32],
    "oracle_qpsk256_demod_hypot": [_p, _p, _p, _u32],
    "oracle_qpsk256_demod_cuabs": [_p, _p, _p, _u32],
    "oracle_philox4x32_10": [_p, _p, _p],
    "oracle_awgn_normals": [_u64, _u64, _p, _p],
    "oracle_qpsk256_mod_awgn": [_p, _p, _p, _u32, _f, _u64, _u64],
    "oracle_fir_ff_mt": [_sz, _p, _sz, _p, _p, _sz, _int],
    "oracle_fm_demod_mt": [_f, _f, _f, _f, _u32, _u64, _p, _sz, _p, _p, _sz, _sz, _int],
    "oracle_qpsk256_demod_mt": [_int, _p, _p, _p, _u32, _int],
    "oracle_qpsk256_mod_awgn_mt": [_p, _p, _p, _u32, _f, _u64, _u64, _int],
    "oracle_add_const": [_int, _p, _f, _f, _p, _sz],
    "oracle_multiply": [_int, _p, _p, _p, _sz],
    "oracle_add_to_magnitude": [_p, _f, _p, _sz],
    "oracle_abs": [_p, _p, _sz],
    "oracle_int8_to_float": [_p, _p, _sz],
    "oracle_cosine": [_int, _f, _f, _p, _sz],
    "oracle_iir": [_int, _p, _p, _sz, _p, _p, _p, _p, _sz],
    "oracle_iir_f32": [_int, _p, _p, _sz, _p, _p, _p, _p, _sz],
}
for _name, _args in _SIG.items():
    getattr(_lib, _name).argtypes = _args
    getattr(_lib, _name).restype = None
_lib.oracle_nco_inc.argtypes = [_f, _f, _f]
_lib.oracle_cuCabsf.argtypes = [_f, _f]
_lib.oracle_cuCabsf.restype = _f
_lib.oracle_awgn_normal21.argtypes = [_u32]
_lib.oracle_awgn_normal21.restype = _f
_lib.oracle_awgn_tail_normal.argtypes = [_u32, _u32]
_lib.oracle_awgn_tail_normal.restype = _f
_lib.oracle_nco_inc.restype = _u32


def _c(a, dtype):
    a = np.ascontiguousarray(a, dtype=dtype)
    return a


def _ptr(a):
    return a.ctypes.data


_FIR = {
    (np.float32, np.float32): ("oracle_fir_ff", np.float32),
    (np.float32, np.complex64): ("oracle_fir_fc", np.complex64),
    (np.complex64, np.complex64): ("oracle_fir_cc", np.complex64),
    (np.complex64, np.float32): ("oracle_fir_cf", np.complex64),
}


def fir(taps, x, decimation=1, num_outputs=None, k0=0, k1=None):
    """y[k] for k in [k0, k1) (other entries zero). Dtypes pick FF/FC/CC/CF like the C ABI."""
    taps = np.ascontiguousarray(taps)
    x = np.ascontiguousarray(x)
    name, odt = _FIR[(taps.dtype.type, x.dtype.type)]
    T = taps.size
    if num_outputs is None:
        num_outputs = (x.size - T) // decimation + 1
    k1 = num_outputs if k1 is None else k1
    assert x.size >= (k1 - 1) * decimation + T if k1 > 0 else True
    y = np.zeros(num_outputs, dtype=odt)
    getattr(_lib, name)(decimation, _ptr(taps), T, _ptr(x), _ptr(y), k0, k1)
    return y


def fir_fc_mt(taps, x, decimation, num_outputs, nthreads):
    taps = _c(taps, np.float32)
    x = _c(x, np.complex64)
    y = np.empty(num_outputs, dtype=np.complex64)
    _lib.oracle_fir_fc_mt(decimation, _ptr(taps), taps.size, _ptr(x), _ptr(y), num_outputs, nthreads)
    return y


def fir_bound_fc(taps, x, decimation, num_outputs, k0=0, k1=None):
    taps = _c(taps, np.float32)
    x = _c(x, np.complex64)
    k1 = num_outputs if k1 is None else k1
    s = np.zeros(num_outputs, dtype=np.float32)
    _lib.oracle_fir_bound_fc(decimation, _ptr(taps), taps.size, _ptr(x), _ptr(s), k0, k1)
    return s


def nco_inc(fs, tune, chan):
    return int(_lib.oracle_nco_inc(fs, tune, chan))


def nco_mix(x, n0, inc):
    x = _c(x, np.complex64)
    z = np.empty_like(x)
    _lib.oracle_nco_mix(_ptr(x), _ptr(z), n0, inc, 0, x.size)
    return z


def fm_demod(x, taps, fs, tune, chan, dev, decimation, first_sample_index=0, num_outputs=None, m0=0, m1=None):
    x = _c(x, np.complex64)
    taps = _c(taps, np.float32)
    if num_outputs is None:
        num_outputs = (x.size - taps.size) // decimation
    m1 = num_outputs if m1 is None else m1
    out = np.zeros(num_outputs, dtype=np.float32)
    _lib.oracle_fm_demod(fs, tune, chan, dev, decimation, first_sample_index, _ptr(taps), taps.size, _ptr(x),
                         _ptr(out), m0, m1)
    return out


def am_demod(x, taps, fs, tune, chan, decimation, first_sample_index=0, num_outputs=None, m0=0, m1=None):
    x = _c(x, np.complex64)
    taps = _c(taps, np.float32)
    if num_outputs is None:
        num_outputs = (x.size - taps.size) // decimation + 1
    m1 = num_outputs if m1 is None else m1
    out = np.zeros(num_outputs, dtype=np.float32)
    _lib.oracle_am_demod(fs, tune, chan, decimation, first_sample_index, _ptr(taps), taps.size, _ptr(x),
                         _ptr(out), m0, m1)
    return out


def chain_fir(x, taps, fs, tune, chan, decimation, first_sample_index, num_outputs, m0=0, m1=None):
    x = _c(x, np.complex64)
    taps = _c(taps, np.float32)
    m1 = num_outputs if m1 is None else m1
    y = np.zeros(num_outputs, dtype=np.complex64)
    _lib.oracle_chain_fir(fs, tune, chan, decimation, first_sample_index, _ptr(taps), taps.size, _ptr(x), _ptr(y),
                          m0, m1)
    return y


def quad_fm(x, gain, n=None):
    x = _c(x, np.complex64)
    n = x.size - 1 if n is None else n
    out = np.empty(n, dtype=np.float32)
    _lib.oracle_quad_fm(_ptr(x), _ptr(out), gain, n)
    return out


def quad_am(x):
    x = _c(x, np.complex64)
    out = np.empty(x.size, dtype=np.float32)
    _lib.oracle_quad_am(_ptr(x), _ptr(out), x.size)
    return out


def magnitude(x):
    x = _c(x, np.complex64)
    out = np.empty(x.size, dtype=np.float32)
    _lib.oracle_magnitude(_ptr(x), _ptr(out), x.size)
    return out


def qpsk_mod(bits, n, a):
    bits = _c(bits, np.uint8)
    assert bits.size >= (n + 3) // 4
    out = np.empty(n, dtype=np.complex64)
    _lib.oracle_qpsk_mod(_ptr(bits), _ptr(out), n, a)
    return out


def qpsk_demod(x, n=None, initial=None):
    x = _c(x, np.complex64)
    n = x.size if n is None else n
    bits = np.zeros((n + 3) // 4, dtype=np.uint8) if initial is None else np.array(initial, dtype=np.uint8)
    _lib.oracle_qpsk_demod(_ptr(x), _ptr(bits), n)
    return bits


def qpsk256_table(ctype, amplitude):
    t = np.empty(256, dtype=np.complex64)
    _lib.oracle_qpsk256_table(ctype, amplitude, _ptr(t))
    return t


def qpsk256_mod(table, symbols):
    table = _c(table, np.complex64)
    symbols = _c(symbols, np.uint8)
    out = np.empty(symbols.size, dtype=np.complex64)
    _lib.oracle_qpsk256_mod(_ptr(table), _ptr(symbols), _ptr(out), symbols.size)
    return out


def qpsk256_demod(table, x, rule="cuabs", nthreads=1):
    """rule: "cuabs" the reference's cuCabsf rule (qpsk256.cu:171-181; the library's contract), "sq" the
    squared distance (cross-check), "hypot" libm hypotf in place of cuCabsf."""
    table = _c(table, np.complex64)
    x = _c(x, np.complex64)
    out = np.empty(x.size, dtype=np.uint8)
    if nthreads > 1 and rule in ("sq", "cuabs"):
        _lib.oracle_qpsk256_demod_mt(1 if rule == "cuabs" else 0, _ptr(table), _ptr(x), _ptr(out), x.size, nthreads)
        return out
    fn = {"sq": _lib.oracle_qpsk256_demod, "hypot": _lib.oracle_qpsk256_demod_hypot,
          "cuabs": _lib.oracle_qpsk256_demod_cuabs}[rule]
    fn(_ptr(table), _ptr(x), _ptr(out), x.size)
    return out


def cuCabsf(re, im):
    return float(_lib.oracle_cuCabsf(re, im))


def philox4x32_10(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.empty(4, dtype=np.uint32)
    _lib.oracle_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def awgn_normal21(bits):
    """One standard normal from 21 random bits (the AWGN construction, gsdr_amd/csrc/awgn.hpp)."""
    return float(_lib.oracle_awgn_normal21(bits))


def awgn_tail_normal(bits, ext):
    """The tail extension of a component whose 20-bit a is below 32: 18 more bits `ext` (awgn.hpp)."""
    return float(_lib.oracle_awgn_tail_normal(bits, ext))


def awgn_normals(seed, symbol_index):
    g0, g1 = ctypes.c_float(), ctypes.c_float()
    _lib.oracle_awgn_normals(seed, symbol_index, ctypes.byref(g0), ctypes.byref(g1))
    return g0.value, g1.value


def qpsk256_mod_awgn(table, symbols, sigma, seed, first_symbol=0, nthreads=1):
    """gsdrxQpsk256ModulateAwgn's contract: table[s] + sigma * counter-based Gaussian pair."""
    table = _c(table, np.complex64)
    symbols = _c(symbols, np.uint8)
    out = np.empty(symbols.size, dtype=np.complex64)
    if nthreads > 1:
        _lib.oracle_qpsk256_mod_awgn_mt(_ptr(table), _ptr(symbols), _ptr(out), symbols.size, sigma, seed, first_symbol,
                                        nthreads)
    else:
        _lib.oracle_qpsk256_mod_awgn(_ptr(table), _ptr(symbols), _ptr(out), symbols.size, sigma, seed, first_symbol)
    return out


def fir_ff_mt(taps, x, decimation, num_outputs, nthreads):
    taps = _c(taps, np.float32)
    x = _c(x, np.float32)
    y = np.empty(num_outputs, dtype=np.float32)
    _lib.oracle_fir_ff_mt(decimation, _ptr(taps), taps.size, _ptr(x), _ptr(y), num_outputs, nthreads)
    return y


def fm_demod_mt(x, taps, fs, tune, chan, dev, decimation, first_sample_index, num_outputs, nthreads, m0=0, m1=None):
    x = _c(x, np.complex64)
    taps = _c(taps, np.float32)
    m1 = num_outputs if m1 is None else m1
    out = np.zeros(num_outputs, dtype=np.float32)
    _lib.oracle_fm_demod_mt(fs, tune, chan, dev, decimation, first_sample_index, _ptr(taps), taps.size, _ptr(x),
                            _ptr(out), m0, m1, nthreads)
    return out


def add_const(x, c):
    """gsdrAddConst{FF,CC,CF,FC} by x's dtype and whether c is complex."""
    is_c = isinstance(c, complex)
    cplx_in = np.iscomplexobj(x)
    x = _c(x, np.complex64 if cplx_in else np.float32)
    variant = {(False, False): 0, (True, True): 1, (True, False): 2, (False, True): 3}[(cplx_in, is_c)]
    out = np.empty(x.size, np.complex64 if (cplx_in or is_c) else np.float32)
    cr, ci = (c.real, c.imag) if is_c else (float(c), 0.0)
    _lib.oracle_add_const(variant, _ptr(x), cr, ci, _ptr(out), x.size)
    return out


def multiply(a, b):
    ca, cb = np.iscomplexobj(a), np.iscomplexobj(b)
    variant = {(True, True): 0, (False, False): 1, (True, False): 2}[(ca, cb)]
    a = _c(a, np.complex64 if ca else np.float32)
    b = _c(b, np.complex64 if cb else np.float32)
    out = np.empty(a.size, np.complex64 if ca else np.float32)
    _lib.oracle_multiply(variant, _ptr(a), _ptr(b), _ptr(out), a.size)
    return out


def add_to_magnitude(x, c):
    x = _c(x, np.complex64)
    out = np.empty(x.size, np.complex64)
    _lib.oracle_add_to_magnitude(_ptr(x), float(c), _ptr(out), x.size)
    return out


def abs_(x):
    x = _c(x, np.float32)
    out = np.empty(x.size, np.float32)
    _lib.oracle_abs(_ptr(x), _ptr(out), x.size)
    return out


def int8_to_float(x):
    x = _c(x, np.int8)
    out = np.empty(x.size, np.float32)
    _lib.oracle_int8_to_float(_ptr(x), _ptr(out), x.size)
    return out


def cosine(phi_begin, phi_end, n, complex_out=True):
    out = np.empty(n, np.complex64 if complex_out else np.float32)
    _lib.oracle_cosine(1 if complex_out else 0, float(phi_begin), float(phi_end), _ptr(out), n)
    return out


def iir(b, a, x, x_hist=None, y_hist=None):
    """IIR in double (include/gsdr/iir.h semantics). Returns (y, new_x_hist, new_y_hist); histories are
    arrays of K-1 samples (x[-1-i], y[-1-i]) or None."""
    b = _c(b, np.float32)
    a = _c(a, np.float32)
    K = b.size
    cplx = np.iscomplexobj(x)
    dt = np.complex64 if cplx else np.float32
    x = _c(x, dt)
    y = np.empty(x.size, dt)
    xh = None if x_hist is None else _c(np.array(x_hist, dt).copy(), dt)
    yh = None if y_hist is None else _c(np.array(y_hist, dt).copy(), dt)
    _lib.oracle_iir(1 if cplx else 0, _ptr(b), _ptr(a), K, None if xh is None else _ptr(xh),
                    None if yh is None else _ptr(yh), _ptr(x), _ptr(y), x.size)
    return y, xh, yh


def iir_f32(b, a, x, x_hist=None, y_hist=None):
    """The IIR as a sequential float32 loop (error scale of any fp32 implementation)."""
    b = _c(b, np.float32)
    a = _c(a, np.float32)
    cplx = np.iscomplexobj(x)
    dt = np.complex64 if cplx else np.float32
    x = _c(x, dt)
    y = np.empty(x.size, dt)
    xh = None if x_hist is None else _c(x_hist, dt)
    yh = None if y_hist is None else _c(y_hist, dt)
    _lib.oracle_iir_f32(1 if cplx else 0, _ptr(b), _ptr(a), b.size, None if xh is None else _ptr(xh),
                        None if yh is None else _ptr(yh), _ptr(x), _ptr(y), x.size)
    return y
