"""CPU: the C-ABI library loads, exports exactly what include/gsdr/*.h declares, and its host-only
logic (argument validation that returns before any device work, the NCO increment) behaves as
specified. No compute call is made here."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDRS = sorted(glob.glob(os.path.join(ROOT, "include", "gsdr", "*.h")))

HIP_SUCCESS = 0
HIP_ERROR_INVALID_VALUE = 1


def declared_symbols():
    names = {}
    for h in HDRS:
        text = open(h).read()
        for m in re.finditer(r"GSDR_PUBLIC\s+[\w\s\*]+?\b(gsdr\w+)\s*\(([^;]*?)\)\s*GSDR_NO_EXCEPT", text, re.S):
            args = m.group(2).strip()
            nargs = 0 if args in ("", "void") else args.count(",") + 1
            names[m.group(1)] = nargs
    return names


@pytest.fixture(scope="module")
def abi():
    from gsdr_amd import abi

    return abi


def test_headers_declare_the_reference_surface():
    names = declared_symbols()
    # the reference's hot-path C ABI
    ref = ["gsdrFirFC", "gsdrFirFF", "gsdrFirCC", "gsdrFirCF", "gsdrFmDemod", "gsdrAmDemod", "gsdrQuadFmDemod",
           "gsdrQuadAmDemod", "gsdrMagnitude", "gsdrQpskModulate", "gsdrQpskModulate4x", "gsdrQpskDemodulate",
           "gsdrQpskDemodulate4x", "gsdrQpskModulateTemplated", "gsdrQpskDemodulateTemplated",
           "gsdrQpsk256Modulate", "gsdrQpsk256Demodulate", "gsdrQpsk256Modulate4x", "gsdrQpsk256Demodulate4x",
           "gsdrQpsk256InitConstellation",
           # element-wise surface: arithmetic.h:26-95, trig.h, conversion.h
           "gsdrAddConstFF", "gsdrAddConstCC", "gsdrAddConstCF", "gsdrAddConstFC", "gsdrMultiplyCC", "gsdrMultiplyFF",
           "gsdrMultiplyCF", "gsdrAddToMagnitude", "gsdrAbs", "gsdrCosineC", "gsdrCosineF", "gsdrInt8ToNormFloat"]
    for n in ref:
        assert n in names, n
    # argument counts of the reference headers (fir.h:30-68, fm.h:42-55, am.h:25-37, ...)
    assert names["gsdrFirFC"] == 8 and names["gsdrFmDemod"] == 13 and names["gsdrAmDemod"] == 12
    assert names["gsdrQpskModulate4x"] == 12 and names["gsdrQpsk256Demodulate4x"] == 12


def test_library_exports_every_declared_symbol(abi):
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    declared = declared_symbols()
    assert set(declared) <= exported, set(declared) - exported
    # nothing but the C ABI leaks out of the library
    assert {e for e in exported if not e.startswith("gsdr")} == set()
    for name, nargs in declared.items():
        assert name in abi.SIGNATURES, name
        assert len(abi.SIGNATURES[name][1]) == nargs, name
        getattr(abi.lib, name)


def test_version(abi):
    assert abi.lib.gsdrVersion().decode().startswith("gsdr-mi355x")


def test_nco_increment_matches_oracle(abi):
    from oracle import oracle as o

    cases = [(1e6, 0.0, 1e5), (1e6, 1e5, 0.0), (2.4e6, 101.1e6, 100.9e6), (48000.0, 0.0, 0.0),
             (1e6, 0.0, 5e5), (1e6, 0.0, -5e5), (1e6, 3e6, 0.0), (3.0, 1.0, 0.0), (1e6, 0.0, 0.25)]
    for fs, tune, chan in cases:
        assert abi.lib.gsdrNcoPhaseIncrement(fs, tune, chan) == o.nco_inc(fs, tune, chan), (fs, tune, chan)
    assert abi.lib.gsdrNcoPhaseIncrement(1e6, 0.0, 1e5) == (2 ** 32 - 429496730)


def test_host_argument_validation_without_device_work(abi):
    lib = abi.lib
    null = None
    # numOutputs == 0: success, nothing launched (the reference launches a 0-block grid)
    assert lib.gsdrFirFC(4, null, 127, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrFirFF(1, null, 63, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrFmDemod(1e6, 0.0, 1e5, 2e4, 4, 0, null, 127, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrQpskModulate(null, null, 0, 1.0, 0, null) == HIP_SUCCESS
    assert lib.gsdrQpsk256Demodulate(null, null, 0, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrQuadFmDemod(null, null, 1.0, 0, 0, null) == HIP_SUCCESS
    # decimation == 0 or missing output: hipErrorInvalidValue, before any device call
    assert lib.gsdrFirFC(0, null, 127, null, null, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrFirCC(4, null, 127, null, null, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrFmDemod(1e6, 0.0, 1e5, 2e4, 0, 0, null, 127, null, null, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrAmDemod(1e6, 0.0, 1e5, 0, 0, null, 127, null, null, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    dummy = ctypes.c_void_p(16)
    assert lib.gsdrFmDemod(0.0, 0.0, 1e5, 2e4, 4, 0, dummy, 127, dummy, dummy, 16, 0, null) == \
        HIP_ERROR_INVALID_VALUE


def test_extension_validation_without_device_work(abi):
    """The gsdrx extensions and the IIR / element-wise entry points reject bad arguments (or accept
    empty work) before touching a device, as the core entry points do."""
    lib = abi.lib
    null = None
    dummy = ctypes.c_void_p(16)
    # int8 front end
    assert lib.gsdrxFirFCInt8(4, null, 127, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrxFirFCInt8(0, dummy, 127, dummy, dummy, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxFmDemodInt8(1e6, 0.0, 1e5, 2e4, 0, 0, dummy, 127, dummy, dummy, 16, 0, null) == \
        HIP_ERROR_INVALID_VALUE
    # multi-channel: no channels / no outputs succeed; missing channel arrays or bad format fail
    assert lib.gsdrxFmDemodMulti(1e6, 0.0, null, null, 0, 4, 0, dummy, 127, 0, dummy, dummy, 16, 0, null) == \
        HIP_SUCCESS
    assert lib.gsdrxFmDemodMulti(1e6, 0.0, null, null, 3, 4, 0, dummy, 127, 0, dummy, dummy, 16, 0, null) == \
        HIP_ERROR_INVALID_VALUE
    chans = (ctypes.c_float * 2)(1e5, 2e5)
    assert lib.gsdrxAmDemodMulti(1e6, 0.0, chans, 2, 4, 0, dummy, 127, 7, dummy, dummy, 16, 0, null) == \
        HIP_ERROR_INVALID_VALUE
    # IIR: the reference's coefficient-count limits, empty input, Custom samplesPerThread limits
    for K in (0, 1, 33):
        assert lib.gsdrIirFF(dummy, dummy, K, null, null, dummy, dummy, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrIirCC(dummy, dummy, 5, null, null, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrIirFFCustom(dummy, dummy, 5, null, null, dummy, dummy, 16, 0, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrIirCCCustom(dummy, dummy, 5, null, null, dummy, dummy, 16, 33, 0, null) == HIP_ERROR_INVALID_VALUE
    # element-wise: empty work succeeds, missing operands fail
    assert lib.gsdrMultiplyCC(null, null, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrMultiplyFF(dummy, null, dummy, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrCosineC(0.0, 1.0, null, 0, 0, null) == HIP_SUCCESS
    assert lib.gsdrInt8ToNormFloat(null, dummy, 16, 0, null) == HIP_ERROR_INVALID_VALUE
    # streaming object: creation argument checks, null handle, zero-length process
    h = ctypes.c_void_p()
    assert lib.gsdrxStreamCreate(null, 0, 0, 4, dummy, 127, 1.0, 0.0, 0.0, 1.0, 0, 0) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxStreamCreate(ctypes.byref(h), 0, 0, 0, dummy, 127, 1.0, 0.0, 0.0, 1.0, 0, 0) == \
        HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxStreamCreate(ctypes.byref(h), 3, 0, 4, dummy, 127, 1.0, 0.0, 0.0, 1.0, 0, 0) == \
        HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxStreamCreate(ctypes.byref(h), 0, 2, 4, dummy, 127, 1.0, 0.0, 0.0, 1.0, 0, 0) == \
        HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxStreamProcess(null, dummy, 16, dummy, 16, null, null) == HIP_ERROR_INVALID_VALUE
    assert lib.gsdrxStreamOutputsFor(null, 100) == 0
    assert lib.gsdrxStreamDestroy(null) == HIP_SUCCESS


def test_ops_module_imports(abi):
    from gsdr_amd import ops

    assert callable(ops.fir) and callable(ops.fm_demod)
