"""gsdr_amd: MI355X-native GSDR DSP primitives.

The product is the C-ABI shared library `libgsdr.so` (include/gsdr/*.h, kernels in gsdr_amd/csrc).
`gsdr_amd.abi` binds it with ctypes exactly as an external FFI would; `gsdr_amd.ops` offers
torch-tensor conveniences on top. torch is imported first so that the process has a single HIP
runtime (torch's libamdhip64.so.7 satisfies libgsdr.so's dependency by SONAME).
"""
import torch  # noqa: F401  (must precede loading libgsdr.so)

from . import abi  # noqa: E402
from .abi import GsdrError, lib  # noqa: E402,F401

__version__ = abi.lib.gsdrVersion().decode()
