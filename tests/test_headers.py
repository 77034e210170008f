"""CPU: the drop-in boundary as a native caller sees it (reference include/gsdr/gsdr.h:18-31).

Every include/gsdr/*.h compiles on its own as C11 and as C++17 (the reference's callers are C++ that
include <gsdr/gsdr.h>); a caller using the reference's helper names (SAFE_CUDA_RET, CHECK_CUDA_RET,
getCurrentCudaDevice -- reference include/gsdr/cuda_util.h:32-97) compiles and links against
libgsdr.so; examples/fm_receiver.cpp builds with hipcc against the library. Running the example is
a GPU test (tests/test_gpu_example.py)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
HDRS = sorted(os.path.basename(h) for h in glob.glob(os.path.join(INC, "gsdr", "*.h")))
ROCM_INC = "/opt/rocm/include"
FLAGS = ["-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I" + INC, "-I" + ROCM_INC]

pytestmark = pytest.mark.skipif(not os.path.isdir(ROCM_INC), reason="needs the ROCm headers")


def _compile(tmp_path, src, lang, extra=()):
    ext = "c" if lang == "c" else "cpp"
    f = tmp_path / f"t.{ext}"
    f.write_text(src)
    cc = ["gcc", "-std=c11"] if lang == "c" else ["g++", "-std=c++17"]
    r = subprocess.run(cc + FLAGS + ["-c", str(f), "-o", str(tmp_path / "t.o")] + list(extra), capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("lang", ["c", "c++"])
@pytest.mark.parametrize("hdr", HDRS)
def test_header_compiles_alone(tmp_path, hdr, lang):
    _compile(tmp_path, f"#include <gsdr/{hdr}>\nint gsdr_header_probe(void) {{ return 0; }}\n", lang)


CALLER = r"""
#include <gsdr/gsdr.h>
#include <stddef.h>

/* written against the reference's helper names */
hipError_t filter_block(const float* taps, size_t tapCount, const hipFloatComplex* in, hipFloatComplex* out,
                        size_t n, hipStream_t stream) {
  const int32_t device = getCurrentCudaDevice();
  if (device < 0) return (hipError_t)(-device);
  CHECK_CUDA_RET("before the block");
  SAFE_CUDA_RET(gsdrFirFC(4, taps, tapCount, in, out, n, device, stream));
  SAFE_CUDA_RET(gsdrFmDemod(1.0e6f, 0.0f, 1.0e5f, 2.0e4f, 4, 0, taps, tapCount, in, (float*)out, n, device, stream));
  return hipSuccess;
}
"""


@pytest.mark.parametrize("lang", ["c", "c++"])
@pytest.mark.parametrize("debug", [False, True])
def test_reference_style_caller_compiles(tmp_path, lang, debug):
    _compile(tmp_path, CALLER, lang, ["-DDEBUG"] if debug else [])


def _lib():
    from gsdr_amd import abi

    return abi.LIB_PATH


def test_reference_style_caller_links(tmp_path):
    lib = _lib()
    src = tmp_path / "main.cpp"
    src.write_text(CALLER + "\nint main() { return filter_block(nullptr, 0, nullptr, nullptr, 0, nullptr) == hipSuccess"
                            " ? 0 : 1; }\n")
    r = subprocess.run(["g++", "-std=c++17"] + FLAGS + [str(src), "-L" + os.path.dirname(lib), "-lgsdr",
                                                         "-L/opt/rocm/lib", "-lamdhip64", "-o", str(tmp_path / "a.out")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # every gsdr symbol the caller uses resolves in libgsdr.so
    nm = subprocess.run(["nm", "-u", str(tmp_path / "a.out")], capture_output=True, text=True, check=True).stdout
    assert "gsdrFirFC" in nm and "gsdrFmDemod" in nm


@pytest.mark.skipif(shutil.which("make") is None, reason="needs make")
def test_example_builds_against_the_library():
    r = subprocess.run(["make", "-C", ROOT, "-j8", "examples"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert os.path.exists(os.path.join(ROOT, "build", "fm_receiver"))
