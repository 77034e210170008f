"""torch-tensor conveniences over the C ABI (gsdr_amd.abi).

Each function checks shapes/dtypes, allocates the output if none is given, and calls the matching
`gsdr*` entry point on the tensor's device and on torch's current stream for that device, raising
GsdrError on a non-zero hipError_t. Complex tensors are torch.complex64 (interleaved float pairs,
the hipFloatComplex layout).
"""
from __future__ import annotations

import torch

from .abi import Complex, check, lib

__all__ = [
    "fir", "fir_variant", "fm_demod", "am_demod", "quad_fm_demod", "quad_am_demod", "magnitude",
    "qpsk_modulate", "qpsk_demodulate", "qpsk_modulate_4x", "qpsk_demodulate_4x",
    "qpsk_modulate_templated", "qpsk_demodulate_templated",
    "qpsk256_init", "qpsk256_modulate", "qpsk256_modulate_awgn", "qpsk256_demodulate", "qpsk256_modulate_4x", "qpsk256_demodulate_4x",
    "nco_phase_increment", "stream_of",
    "fm_demod_multi", "am_demod_multi", "iir", "add_const", "multiply", "add_to_magnitude", "abs_", "cosine", "int8_to_norm_float",
]


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _dev(t: torch.Tensor) -> int:
    if t.device.type != "cuda":
        raise ValueError("gsdr_amd operates on device tensors (got %s)" % t.device)
    return t.device.index


def _ptr(t):
    return None if t is None else t.data_ptr()


def _require(t: torch.Tensor, dtype, name: str, min_len: int = 0):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.numel() < min_len:
        raise ValueError(f"{name}: need at least {min_len} elements, got {t.numel()}")


_FIR = {
    (torch.float32, torch.complex64): ("gsdrFirFC", torch.complex64),
    (torch.float32, torch.float32): ("gsdrFirFF", torch.float32),
    (torch.complex64, torch.complex64): ("gsdrFirCC", torch.complex64),
    (torch.complex64, torch.float32): ("gsdrFirCF", torch.complex64),
    (torch.float32, torch.int8): ("gsdrxFirFCInt8", torch.complex64),  # interleaved int8 I/Q
}


def _nsamp(x):
    """samples in x: int8 tensors hold interleaved I/Q pairs (gsdr_ext.h)."""
    if x.dtype == torch.int8:
        if x.numel() % 2:
            raise ValueError("int8 I/Q input needs an even number of elements")
        return x.numel() // 2
    return x.numel()


def _require_samples(x, dtype, name, min_samples):
    _require(x, dtype, name, min_samples * (2 if dtype == torch.int8 else 1))


def _fir_prepare(taps, x, decimation, num_outputs, out):
    key = (taps.dtype, x.dtype)
    if key not in _FIR:
        raise TypeError(f"unsupported tap/input dtypes {key}")
    name, odt = _FIR[key]
    T = taps.numel()
    L = _nsamp(x)
    if num_outputs is None:
        num_outputs = (L - T) // decimation + 1 if L >= T else 0
    if num_outputs > 0:
        _require_samples(x, x.dtype, "input", (num_outputs - 1) * decimation + T)
    if out is None:
        out = torch.empty(num_outputs, dtype=odt, device=x.device)
    _require(out, odt, "output", num_outputs)
    return name, num_outputs, out


def fir(taps: torch.Tensor, x: torch.Tensor, decimation: int = 1, num_outputs: int | None = None,
        out: torch.Tensor | None = None) -> torch.Tensor:
    """y[k] = sum_i x[k*decimation + i] * taps[i] (gsdrFirFC/FF/CC/CF by dtype)."""
    name, n, out = _fir_prepare(taps, x, decimation, num_outputs, out)
    check(name, getattr(lib, name)(decimation, _ptr(taps), taps.numel(), _ptr(x), _ptr(out), n, _dev(x),
                                   stream_of(x)))
    return out


def fir_variant(variant: int, taps: torch.Tensor, x: torch.Tensor, decimation: int = 4,
                num_outputs: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """gsdrFirFC (complex64 input) or gsdrxFirFCInt8 (int8 I/Q input) with an explicit tile shape
    (tuning; see gsdr_ext.h)."""
    name, n, out = _fir_prepare(taps, x, decimation, num_outputs, out)
    if name not in ("gsdrFirFC", "gsdrxFirFCInt8"):
        raise TypeError("fir_variant takes real taps on complex64 or int8 I/Q input")
    entry = "gsdrxFirFCVariant" if name == "gsdrFirFC" else "gsdrxFirFCInt8Variant"
    check(entry, getattr(lib, entry)(variant, decimation, _ptr(taps), taps.numel(), _ptr(x), _ptr(out), n, _dev(x),
                                     stream_of(x)))
    return out


def fm_demod(x, taps, rf_sample_rate, tuning_frequency, channel_frequency, frequency_deviation, decimation,
             first_sample_index=0, num_outputs=None, out=None):
    """gsdrFmDemod: NCO shift + low-pass FIR + decimation + FM discriminator (fm.h); int8 I/Q input
    selects gsdrxFmDemodInt8."""
    if x.dtype not in (torch.complex64, torch.int8):
        raise TypeError(f"input: expected complex64 or int8 I/Q, got {x.dtype}")
    _require(x, x.dtype, "input")
    _require(taps, torch.float32, "taps")
    T = taps.numel()
    if num_outputs is None:
        num_outputs = max(0, (_nsamp(x) - T) // decimation)
    if num_outputs > 0:
        _require_samples(x, x.dtype, "input", num_outputs * decimation + T)
    if out is None:
        out = torch.empty(num_outputs, dtype=torch.float32, device=x.device)
    _require(out, torch.float32, "output", num_outputs)
    name = "gsdrxFmDemodInt8" if x.dtype == torch.int8 else "gsdrFmDemod"
    check(name, getattr(lib, name)(rf_sample_rate, tuning_frequency, channel_frequency, frequency_deviation,
                                         decimation, first_sample_index, _ptr(taps), T, _ptr(x), _ptr(out),
                                         num_outputs, _dev(x), stream_of(x)))
    return out


def am_demod(x, taps, rf_sample_rate, tuning_frequency, channel_frequency, decimation, first_sample_index=0,
             num_outputs=None, out=None):
    """gsdrAmDemod: NCO shift + low-pass FIR + decimation + envelope (am.h); int8 I/Q input selects
    gsdrxAmDemodInt8."""
    if x.dtype not in (torch.complex64, torch.int8):
        raise TypeError(f"input: expected complex64 or int8 I/Q, got {x.dtype}")
    _require(x, x.dtype, "input")
    _require(taps, torch.float32, "taps")
    T = taps.numel()
    L = _nsamp(x)
    if num_outputs is None:
        num_outputs = (L - T) // decimation + 1 if L >= T else 0
    if num_outputs > 0:
        _require_samples(x, x.dtype, "input", (num_outputs - 1) * decimation + T)
    if out is None:
        out = torch.empty(num_outputs, dtype=torch.float32, device=x.device)
    _require(out, torch.float32, "output", num_outputs)
    name = "gsdrxAmDemodInt8" if x.dtype == torch.int8 else "gsdrAmDemod"
    check(name, getattr(lib, name)(rf_sample_rate, tuning_frequency, channel_frequency, decimation,
                                         first_sample_index, _ptr(taps), T, _ptr(x), _ptr(out), num_outputs,
                                         _dev(x), stream_of(x)))
    return out


def _multi(name, x, taps, fs, tune, chans, devs, decimation, first_sample_index, num_outputs, fm):
    import ctypes

    if x.dtype not in (torch.complex64, torch.int8):
        raise TypeError(f"input: expected complex64 or int8 I/Q, got {x.dtype}")
    _require(x, x.dtype, "input")
    _require(taps, torch.float32, "taps")
    T, L = taps.numel(), _nsamp(x)
    if num_outputs is None:
        num_outputs = max(0, (L - T) // decimation) if fm else ((L - T) // decimation + 1 if L >= T else 0)
    need = num_outputs * decimation + T if fm else (num_outputs - 1) * decimation + T
    if num_outputs > 0:
        _require_samples(x, x.dtype, "input", need)
    C = len(chans)
    out = torch.empty((C, num_outputs), dtype=torch.float32, device=x.device)
    fa = (ctypes.c_float * max(C, 1))(*chans)
    args = [fs, tune, fa]
    if fm:
        args.append((ctypes.c_float * max(C, 1))(*devs))
    args += [C, decimation, first_sample_index, _ptr(taps), T, 1 if x.dtype == torch.int8 else 0, _ptr(x), _ptr(out),
             num_outputs, _dev(x), stream_of(x)]
    check(name, getattr(lib, name)(*args))
    return out


def fm_demod_multi(x, taps, rf_sample_rate, tuning_frequency, channel_frequencies, frequency_deviations,
                   decimation, first_sample_index=0, num_outputs=None):
    """gsdrxFmDemodMulti: out[c] = gsdrFmDemod with channel_frequencies[c], frequency_deviations[c]."""
    return _multi("gsdrxFmDemodMulti", x, taps, rf_sample_rate, tuning_frequency, channel_frequencies,
                  frequency_deviations, decimation, first_sample_index, num_outputs, True)


def am_demod_multi(x, taps, rf_sample_rate, tuning_frequency, channel_frequencies, decimation,
                   first_sample_index=0, num_outputs=None):
    """gsdrxAmDemodMulti: out[c] = gsdrAmDemod with channel_frequencies[c]."""
    return _multi("gsdrxAmDemodMulti", x, taps, rf_sample_rate, tuning_frequency, channel_frequencies, None,
                  decimation, first_sample_index, num_outputs, False)


def quad_fm_demod(x, gain, num_outputs=None, out=None):
    _require(x, torch.complex64, "input")
    n = max(0, x.numel() - 1) if num_outputs is None else num_outputs
    if n > 0:
        _require(x, torch.complex64, "input", n + 1)
    out = torch.empty(n, dtype=torch.float32, device=x.device) if out is None else out
    _require(out, torch.float32, "output", n)
    check("gsdrQuadFmDemod", lib.gsdrQuadFmDemod(_ptr(x), _ptr(out), gain, n, _dev(x), stream_of(x)))
    return out


def quad_am_demod(x, num_outputs=None, out=None):
    _require(x, torch.complex64, "input")
    n = x.numel() if num_outputs is None else num_outputs
    _require(x, torch.complex64, "input", n)
    out = torch.empty(n, dtype=torch.float32, device=x.device) if out is None else out
    _require(out, torch.float32, "output", n)
    check("gsdrQuadAmDemod", lib.gsdrQuadAmDemod(_ptr(x), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def magnitude(x, out=None):
    _require(x, torch.complex64, "input")
    n = x.numel()
    out = torch.empty(n, dtype=torch.float32, device=x.device) if out is None else out
    _require(out, torch.float32, "output", n)
    check("gsdrMagnitude", lib.gsdrMagnitude(_ptr(x), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def iir(b, a, x, x_hist=None, y_hist=None, out=None):
    """gsdrIirFF / gsdrIirCC (iir.h): y[n] = sum b[i] x[n-i] - sum_{i>=1} a[i] y[n-i]. x_hist / y_hist
    (K-1 samples, device tensors of x's dtype, or None) hold the state before x and are updated in
    place with the state after it."""
    _require(b, torch.float32, "bCoeffs")
    _require(a, torch.float32, "aCoeffs", b.numel())
    if x.dtype not in (torch.float32, torch.complex64):
        raise TypeError(f"input: expected float32 or complex64, got {x.dtype}")
    _require(x, x.dtype, "input")
    K, n = b.numel(), x.numel()
    for h, nm in ((x_hist, "inputHistory"), (y_hist, "outputHistory")):
        if h is not None:
            _require(h, x.dtype, nm, K - 1)
    out = torch.empty_like(x) if out is None else out
    _require(out, x.dtype, "output", n)
    name = "gsdrIirCC" if x.dtype == torch.complex64 else "gsdrIirFF"
    check(name, getattr(lib, name)(_ptr(b), _ptr(a), K, _ptr(x_hist), _ptr(y_hist), _ptr(x), _ptr(out), n,
                                   _dev(x), stream_of(x)))
    return out


_ADD = {
    (torch.float32, False): ("gsdrAddConstFF", torch.float32),
    (torch.complex64, True): ("gsdrAddConstCC", torch.complex64),
    (torch.complex64, False): ("gsdrAddConstCF", torch.complex64),
    (torch.float32, True): ("gsdrAddConstFC", torch.complex64),
}


def add_const(x, c, out=None):
    """gsdrAddConst{FF,CC,CF,FC}: the variant follows x's dtype and whether c is complex."""
    is_c = isinstance(c, complex)
    if (x.dtype, is_c) not in _ADD:
        raise TypeError(f"unsupported input dtype {x.dtype}")
    name, odt = _ADD[(x.dtype, is_c)]
    _require(x, x.dtype, "input")
    n = x.numel()
    out = torch.empty(n, dtype=odt, device=x.device) if out is None else out
    _require(out, odt, "output", n)
    cval = Complex(c.real, c.imag) if is_c else float(c)
    check(name, getattr(lib, name)(_ptr(x), cval, _ptr(out), n, _dev(x), stream_of(x)))
    return out


_MUL = {
    (torch.complex64, torch.complex64): ("gsdrMultiplyCC", torch.complex64),
    (torch.float32, torch.float32): ("gsdrMultiplyFF", torch.float32),
    (torch.complex64, torch.float32): ("gsdrMultiplyCF", torch.complex64),
}


def multiply(a, b, out=None):
    key = (a.dtype, b.dtype)
    if key not in _MUL:
        raise TypeError(f"unsupported dtypes {key}")
    name, odt = _MUL[key]
    n = a.numel()
    _require(a, a.dtype, "in1")
    _require(b, b.dtype, "in2", n)
    out = torch.empty(n, dtype=odt, device=a.device) if out is None else out
    _require(out, odt, "out", n)
    check(name, getattr(lib, name)(_ptr(a), _ptr(b), _ptr(out), n, _dev(a), stream_of(a)))
    return out


def add_to_magnitude(x, c, out=None):
    _require(x, torch.complex64, "input")
    n = x.numel()
    out = torch.empty(n, dtype=torch.complex64, device=x.device) if out is None else out
    _require(out, torch.complex64, "output", n)
    check("gsdrAddToMagnitude", lib.gsdrAddToMagnitude(_ptr(x), float(c), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def abs_(x, out=None):
    _require(x, torch.float32, "in")
    n = x.numel()
    out = torch.empty(n, dtype=torch.float32, device=x.device) if out is None else out
    _require(out, torch.float32, "out", n)
    check("gsdrAbs", lib.gsdrAbs(_ptr(x), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def cosine(phi_begin, phi_end, n, complex_out=True, device=None, out=None):
    """gsdrCosineC / gsdrCosineF: a phase ramp from phi_begin towards phi_end over n samples."""
    odt = torch.complex64 if complex_out else torch.float32
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    out = torch.empty(n, dtype=odt, device=device) if out is None else out
    _require(out, odt, "output", n)
    name = "gsdrCosineC" if complex_out else "gsdrCosineF"
    check(name, getattr(lib, name)(float(phi_begin), float(phi_end), _ptr(out), n, _dev(out), stream_of(out)))
    return out


def int8_to_norm_float(x, out=None):
    _require(x, torch.int8, "input")
    n = x.numel()
    out = torch.empty(n, dtype=torch.float32, device=x.device) if out is None else out
    _require(out, torch.float32, "output", n)
    check("gsdrInt8ToNormFloat", lib.gsdrInt8ToNormFloat(_ptr(x), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def qpsk_modulate(bits, num_symbols, amplitude=1.0, out=None):
    _require(bits, torch.uint8, "inputBits", (num_symbols + 3) // 4)
    out = torch.empty(num_symbols, dtype=torch.complex64, device=bits.device) if out is None else out
    _require(out, torch.complex64, "output", num_symbols)
    check("gsdrQpskModulate", lib.gsdrQpskModulate(_ptr(bits), _ptr(out), num_symbols, amplitude, _dev(bits),
                                                   stream_of(bits)))
    return out


def qpsk_demodulate(x, num_symbols=None, out=None):
    _require(x, torch.complex64, "input")
    n = x.numel() if num_symbols is None else num_symbols
    out = torch.zeros((n + 3) // 4, dtype=torch.uint8, device=x.device) if out is None else out
    _require(out, torch.uint8, "outputBits", (n + 3) // 4)
    check("gsdrQpskDemodulate", lib.gsdrQpskDemodulate(_ptr(x), _ptr(out), n, _dev(x), stream_of(x)))
    return out


def qpsk_modulate_4x(bits4, outs4, num_symbols, amplitude=1.0):
    check("gsdrQpskModulate4x", lib.gsdrQpskModulate4x(*[_ptr(b) for b in bits4], *[_ptr(o) for o in outs4],
                                                       num_symbols, amplitude, _dev(outs4[0]),
                                                       stream_of(outs4[0])))


def qpsk_demodulate_4x(ins4, bits4, num_symbols):
    check("gsdrQpskDemodulate4x", lib.gsdrQpskDemodulate4x(*[_ptr(i) for i in ins4], *[_ptr(b) for b in bits4],
                                                           num_symbols, _dev(ins4[0]), stream_of(ins4[0])))


def qpsk_modulate_templated(bits, out, num_symbols, amplitude, num_streams):
    check("gsdrQpskModulateTemplated", lib.gsdrQpskModulateTemplated(_ptr(bits), _ptr(out), num_symbols, amplitude,
                                                                     num_streams, _dev(out), stream_of(out)))


def qpsk_demodulate_templated(x, bits, num_symbols, num_streams):
    check("gsdrQpskDemodulateTemplated", lib.gsdrQpskDemodulateTemplated(_ptr(x), _ptr(bits), num_symbols,
                                                                         num_streams, _dev(x), stream_of(x)))


def qpsk256_init(constellation_type, amplitude, device=None):
    dev = torch.cuda.current_device() if device is None else device
    stream = torch.cuda.current_stream(dev).cuda_stream
    check("gsdrQpsk256InitConstellation", lib.gsdrQpsk256InitConstellation(constellation_type, amplitude, dev,
                                                                           stream))


def qpsk256_modulate(symbols, constellation_type, amplitude=1.0, out=None):
    _require(symbols, torch.uint8, "inputBytes")
    n = symbols.numel()
    out = torch.empty(n, dtype=torch.complex64, device=symbols.device) if out is None else out
    _require(out, torch.complex64, "output", n)
    check("gsdrQpsk256Modulate", lib.gsdrQpsk256Modulate(_ptr(symbols), _ptr(out), n, amplitude, constellation_type,
                                                         _dev(symbols), stream_of(symbols)))
    return out


def qpsk256_modulate_awgn(symbols, constellation_type, sigma, seed, first_symbol_index=0, out=None):
    """gsdrxQpsk256ModulateAwgn: table[s] + sigma * counter-based Gaussian noise of (seed, absolute index)."""
    _require(symbols, torch.uint8, "inputBytes")
    n = symbols.numel()
    out = torch.empty(n, dtype=torch.complex64, device=symbols.device) if out is None else out
    _require(out, torch.complex64, "output", n)
    check("gsdrxQpsk256ModulateAwgn", lib.gsdrxQpsk256ModulateAwgn(_ptr(symbols), _ptr(out), n, constellation_type,
                                                                   sigma, seed, first_symbol_index, _dev(symbols),
                                                                   stream_of(symbols)))
    return out


def qpsk256_modulate_awgn_demodulate(symbols, constellation_type, sigma, seed, first_symbol_index=0, noisy=None,
                                     out=None):
    """gsdrxQpsk256ModulateAwgnDemodulate: (noisy symbols, decisions) -- exactly gsdrxQpsk256ModulateAwgn then
    gsdrQpsk256Demodulate, one pass for the rectangular table."""
    _require(symbols, torch.uint8, "inputBytes")
    n = symbols.numel()
    noisy = torch.empty(n, dtype=torch.complex64, device=symbols.device) if noisy is None else noisy
    out = torch.empty(n, dtype=torch.uint8, device=symbols.device) if out is None else out
    _require(noisy, torch.complex64, "noisySymbols", n)
    _require(out, torch.uint8, "outputBytes", n)
    check("gsdrxQpsk256ModulateAwgnDemodulate",
          lib.gsdrxQpsk256ModulateAwgnDemodulate(_ptr(symbols), _ptr(noisy), _ptr(out), n, constellation_type, sigma,
                                                 seed, first_symbol_index, _dev(symbols), stream_of(symbols)))
    return noisy, out


def qpsk256_demodulate(x, constellation_type, out=None):
    _require(x, torch.complex64, "input")
    n = x.numel()
    out = torch.empty(n, dtype=torch.uint8, device=x.device) if out is None else out
    _require(out, torch.uint8, "outputBytes", n)
    check("gsdrQpsk256Demodulate", lib.gsdrQpsk256Demodulate(_ptr(x), _ptr(out), n, constellation_type, _dev(x),
                                                             stream_of(x)))
    return out


def qpsk256_modulate_4x(ins4, outs4, num_symbols, constellation_type, amplitude=1.0):
    check("gsdrQpsk256Modulate4x", lib.gsdrQpsk256Modulate4x(*[_ptr(i) for i in ins4], *[_ptr(o) for o in outs4],
                                                             num_symbols, amplitude, constellation_type,
                                                             _dev(outs4[0]), stream_of(outs4[0])))


def qpsk256_demodulate_4x(ins4, outs4, num_symbols, constellation_type):
    check("gsdrQpsk256Demodulate4x", lib.gsdrQpsk256Demodulate4x(*[_ptr(i) for i in ins4], *[_ptr(o) for o in outs4],
                                                                 num_symbols, constellation_type, _dev(ins4[0]),
                                                                 stream_of(ins4[0])))


def nco_phase_increment(rf_sample_rate, tuning_frequency, channel_frequency) -> int:
    return int(lib.gsdrNcoPhaseIncrement(rf_sample_rate, tuning_frequency, channel_frequency))
