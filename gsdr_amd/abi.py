"""ctypes view of libgsdr.so's C ABI (include/gsdr/*.h), one Python callable per exported symbol.

This is the drop-in boundary as an FFI would bind it: pointers are plain integers (device
addresses), sizes are integers, every call returns the hipError_t code. `gsdr_amd.ops` wraps these for
torch tensors. The shared library is the only implementation: if it is missing, importing this
module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

__all__ = ["lib", "LIB_PATH", "SIGNATURES", "GsdrError", "Complex", "check"]

# GSDR_LIB selects another build of the same ABI (the tools/ scripts load the tuning-probe build,
# build/probes/libgsdr_probes.so); the default is the in-tree product library.
LIB_PATH = os.environ.get("GSDR_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgsdr.so")

_p = ctypes.c_void_p
_sz = ctypes.c_size_t
_u32 = ctypes.c_uint32
_i32 = ctypes.c_int32
_int = ctypes.c_int
_f = ctypes.c_float
_u64 = ctypes.c_uint64
_err = ctypes.c_int  # hipError_t


class Complex(ctypes.Structure):
    """hipFloatComplex passed by value (two floats, 8-byte aligned)."""

    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float)]


_c = Complex

# name -> (restype, argtypes), in the order of include/gsdr/*.h
SIGNATURES = {
    # fir.h
    "gsdrFirFC": (_err, [_sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrFirFF": (_err, [_sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrFirCC": (_err, [_sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrFirCF": (_err, [_sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    # fm.h / am.h
    "gsdrFmDemod": (_err, [_f, _f, _f, _f, _u32, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrAmDemod": (_err, [_f, _f, _f, _u32, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    # quad_demod.h / arithmetic.h
    "gsdrQuadFmDemod": (_err, [_p, _p, _f, _sz, _i32, _p]),
    "gsdrQuadAmDemod": (_err, [_p, _p, _sz, _i32, _p]),
    "gsdrMagnitude": (_err, [_p, _p, _sz, _i32, _p]),
    "gsdrAddConstFF": (_err, [_p, _f, _p, _sz, _i32, _p]),
    "gsdrAddConstCC": (_err, [_p, _c, _p, _sz, _i32, _p]),
    "gsdrAddConstCF": (_err, [_p, _f, _p, _sz, _i32, _p]),
    "gsdrAddConstFC": (_err, [_p, _c, _p, _sz, _i32, _p]),
    "gsdrMultiplyCC": (_err, [_p, _p, _p, _sz, _i32, _p]),
    "gsdrMultiplyFF": (_err, [_p, _p, _p, _sz, _i32, _p]),
    "gsdrMultiplyCF": (_err, [_p, _p, _p, _sz, _i32, _p]),
    "gsdrAddToMagnitude": (_err, [_p, _f, _p, _sz, _i32, _p]),
    "gsdrAbs": (_err, [_p, _p, _sz, _i32, _p]),
    # iir.h
    "gsdrIirFF": (_err, [_p, _p, _sz, _p, _p, _p, _p, _sz, _i32, _p]),
    "gsdrIirCC": (_err, [_p, _p, _sz, _p, _p, _p, _p, _sz, _i32, _p]),
    "gsdrIirFFCustom": (_err, [_p, _p, _sz, _p, _p, _p, _p, _sz, _sz, _i32, _p]),
    "gsdrIirCCCustom": (_err, [_p, _p, _sz, _p, _p, _p, _p, _sz, _sz, _i32, _p]),
    # trig.h / conversion.h
    "gsdrCosineC": (_err, [_f, _f, _p, _sz, _i32, _p]),
    "gsdrCosineF": (_err, [_f, _f, _p, _sz, _i32, _p]),
    "gsdrInt8ToNormFloat": (_err, [_p, _p, _sz, _i32, _p]),
    # qpsk.h
    "gsdrQpskModulate": (_err, [_p, _p, _u32, _f, _i32, _p]),
    "gsdrQpskModulate4x": (_err, [_p, _p, _p, _p, _p, _p, _p, _p, _u32, _f, _i32, _p]),
    "gsdrQpskDemodulate": (_err, [_p, _p, _u32, _i32, _p]),
    "gsdrQpskDemodulate4x": (_err, [_p, _p, _p, _p, _p, _p, _p, _p, _u32, _i32, _p]),
    "gsdrQpskModulateTemplated": (_err, [_p, _p, _u32, _f, _int, _i32, _p]),
    "gsdrQpskDemodulateTemplated": (_err, [_p, _p, _u32, _int, _i32, _p]),
    # qpsk256.h
    "gsdrQpsk256Modulate": (_err, [_p, _p, _u32, _f, _u32, _i32, _p]),
    "gsdrxQpsk256ModulateAwgn": (_err, [_p, _p, _u32, _u32, _f, _u64, _u64, _i32, _p]),
    "gsdrxQpsk256ModulateAwgnDemodulate": (_err, [_p, _p, _p, _u32, _u32, _f, _u64, _u64, _i32, _p]),
    "gsdrQpsk256Demodulate": (_err, [_p, _p, _u32, _u32, _i32, _p]),
    "gsdrQpsk256Modulate4x": (_err, [_p, _p, _p, _p, _p, _p, _p, _p, _u32, _f, _u32, _i32, _p]),
    "gsdrQpsk256Demodulate4x": (_err, [_p, _p, _p, _p, _p, _p, _p, _p, _u32, _u32, _i32, _p]),
    "gsdrQpsk256InitConstellation": (_err, [_u32, _f, _i32, _p]),
    # gsdr_ext.h
    "gsdrVersion": (ctypes.c_char_p, []),
    "gsdrNcoPhaseIncrement": (_u32, [_f, _f, _f]),
    "gsdrxFirFCVariant": (_err, [_int, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrxFirFCInt8": (_err, [_sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrxFirFCInt8Variant": (_err, [_int, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrxFmDemodInt8": (_err, [_f, _f, _f, _f, _u32, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
    "gsdrxFmDemodMulti": (_err, [_f, _f, _p, _p, _u32, _u32, _sz, _p, _sz, _int, _p, _p, _sz, _i32, _p]),
    "gsdrxAmDemodMulti": (_err, [_f, _f, _p, _u32, _u32, _sz, _p, _sz, _int, _p, _p, _sz, _i32, _p]),
    # stream.h
    "gsdrxStreamCreate": (_err, [ctypes.POINTER(_p), _int, _int, _u32, _p, _sz, _f, _f, _f, _f, _sz, _i32]),
    "gsdrxStreamCreateMulti": (_err, [ctypes.POINTER(_p), _int, _int, _u32, _p, _sz, _f, _f, _p, _p, _u32, _sz, _i32]),
    "gsdrxStreamOutputsFor": (_sz, [_p, _sz]),
    "gsdrxStreamProcess": (_err, [_p, _p, _sz, _p, _sz, ctypes.POINTER(_sz), _p]),
    "gsdrxStreamDestroy": (_err, [_p]),
    "gsdrxStreamPlan": (None, [_u32, _sz, ctypes.c_uint64, ctypes.c_uint64, _sz, ctypes.POINTER(ctypes.c_uint64)]),
    "gsdrxAmDemodInt8": (_err, [_f, _f, _f, _u32, _sz, _p, _sz, _p, _p, _sz, _i32, _p]),
}


class GsdrError(RuntimeError):
    """A gsdr entry point returned a non-zero hipError_t."""

    def __init__(self, name: str, code: int):
        super().__init__(f"{name} failed with hipError_t {code}")
        self.name = name
        self.code = code


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
            "gsdr_amd has no CPU fallback")
    handle = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    return handle


lib = _load()


def check(name: str, code: int) -> None:
    if code != 0:
        raise GsdrError(name, code)
