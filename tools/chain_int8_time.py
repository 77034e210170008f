"""Time gsdrxFmDemodInt8 / gsdrxAmDemodInt8 on config 3's shape (2^24 outputs, D = 4, T = 127) -- the
decimation-4 matrix-core default beside the float chains on the converted samples -- and report the
parity of the default against the float chain (wrapped angle / absolute envelope), HIP events
(development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402


def timed(fn, reps=100):
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def main():
    dev = torch.device("cuda", 0)
    n, D, T = 1 << 24, 4, 127
    L = n * D + T
    idx = torch.arange(0, L, dtype=torch.float64, device=dev)
    ph = 2 * 3.141592653589793 * 0.1 * idx + 20.0 * torch.sin(2 * 3.141592653589793 * 0.001 * idx)
    x = torch.view_as_real(torch.polar(torch.ones_like(ph), ph).to(torch.complex64)).reshape(-1)
    g = torch.Generator(device=dev).manual_seed(5)
    x += torch.randn(2 * L, dtype=torch.float32, device=dev, generator=g) * 0.05
    x8 = torch.clamp(torch.round(x * 100), -128, 127).to(torch.int8)  # config 3's signal as int8 I/Q
    xf = ops.int8_to_norm_float(x8).view(torch.complex64)
    taps = torch.from_numpy(lowpass_taps(T)).to(dev)
    fs, tune, chan, dhz, n0 = 1.0e6, 0.0, 1.0e5, 2.0e4, 123
    fm8 = ops.fm_demod(x8, taps, fs, tune, chan, dhz, D, n0, n)
    fmf = ops.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, n)
    gain = fs / (2 * 3.141592653589793 * dhz)
    d = torch.remainder(fm8.double() - fmf.double() + 3.141592653589793 * gain, 2 * 3.141592653589793 * gain)
    d = d - 3.141592653589793 * gain
    print(f"FM int8 default vs float chain: max wrapped err / (pi g) = {float(d.abs().max()) / (3.14159 * gain):.3e}")
    am8 = ops.am_demod(x8, taps, fs, tune, chan, D, n0, n)
    amf = ops.am_demod(xf, taps, fs, tune, chan, D, n0, n)
    print(f"AM int8 default vs float chain: max abs err = {float((am8 - amf).abs().max()):.3e}")
    out = torch.empty(n, dtype=torch.float32, device=dev)
    t_fm8 = timed(lambda: ops.fm_demod(x8, taps, fs, tune, chan, dhz, D, n0, n, out=out))
    t_fmf = timed(lambda: ops.fm_demod(xf, taps, fs, tune, chan, dhz, D, n0, n, out=out))
    t_am8 = timed(lambda: ops.am_demod(x8, taps, fs, tune, chan, D, n0, n, out=out))
    t_amf = timed(lambda: ops.am_demod(xf, taps, fs, tune, chan, D, n0, n, out=out))
    print(f"FM int8 {t_fm8:.1f} us | FM float {t_fmf:.1f} us | AM int8 {t_am8:.1f} us | AM float {t_amf:.1f} us")


if __name__ == "__main__":
    main()
