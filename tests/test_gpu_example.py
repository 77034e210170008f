"""GPU: the plain C++ caller (examples/fm_receiver.cpp, built by `make examples` against libgsdr.so and
include/gsdr, no Python in the process) runs, and the outputs it computed through the C ABI
(gsdrFirFC, gsdrFmDemod) match the CPU oracle (reference include/gsdr/fir.h:30-68, fm.h:42-55)."""
import os
import subprocess

import numpy as np
import pytest

from helpers import FLOAT_TOL, bound, normwise_err, wrapped_angle_err
from oracle import oracle as o

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "fm_receiver")


def test_cpp_example_against_oracle(cuda, tmp_path):
    assert os.path.exists(EXE), "build/fm_receiver missing: run `make examples` before the GPU tests"
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "chunked == monolithic: yes" in r.stdout and "int8 stream == monolithic: yes" in r.stdout, r.stdout
    taps = np.fromfile(tmp_path / "taps.f32", np.float32)
    x = np.fromfile(tmp_path / "x.c64", np.complex64)
    y = np.fromfile(tmp_path / "fir.c64", np.complex64)
    fm = np.fromfile(tmp_path / "fm.f32", np.float32)
    D, N = 4, y.size
    assert taps.size == 127 and N == 1 << 20 and x.size == N * D + taps.size
    assert normwise_err(y, o.fir(taps, x, D, N), bound(taps, x, D, N)) <= FLOAT_TOL
    ref = o.fm_demod(x, taps, 1.0e6, 0.0, 1.0e5, 2.0e4, D, 0, N)
    g = float(np.float32(1.0e6) / (np.float32(2.0) * np.float32(np.pi) * np.float32(2.0e4)))
    assert wrapped_angle_err(fm, ref, g) <= FLOAT_TOL


def test_cpp_short_call_timer_runs(cuda):
    """examples/short_call_timer.cpp: the C++ back-to-back short-call timer runs through the
    C ABI and reports every shape it times (the numbers themselves are measurements, not asserted)."""
    import json

    exe = os.path.join(ROOT, "build", "short_call_timer")
    assert os.path.exists(exe), "build/short_call_timer missing: run `make examples` before the GPU tests"
    r = subprocess.run([exe, "20"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout)
    got = {(row["what"], row["samples_per_call"]) for row in d["rows"]}
    want = {("gsdrMagnitude_256", 256)} | {(w, 1 << s) for w in ("gsdrFmDemod", "gsdrxStreamProcess_fm") for s in (16, 18, 20)}
    assert got == want, got
    assert all(row["gpu_us_per_call"] > 0 for row in d["rows"])
