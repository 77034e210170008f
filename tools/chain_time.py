"""Time gsdrFmDemod / gsdrAmDemod (T = 127, 2^26 input samples) per decimation with HIP events
(development tool; FIR_D = comma-separated decimations)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402


def timed(fn, args, reps=50):
    for _ in range(10):
        assert fn(*args) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(*args)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    n_in, T = 1 << 26, 127
    g = torch.Generator(device=dev).manual_seed(3)
    x = (torch.rand(2 * n_in, device=dev, generator=g) * 2 - 1).view(torch.complex64)
    taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    y0 = torch.empty((n_in - T) // 4, dtype=torch.float32, device=dev)
    timed(abi.lib.gsdrFmDemod, (1e6, 0.0, 1e5, 2e4, 4, 0, taps.data_ptr(), T, x.data_ptr(), y0.data_ptr(),
                                y0.numel(), 0, stream), reps=400)  # clock ramp before the first figure
    for D in [int(v) for v in os.environ.get("FIR_D", "1,2,3,4,5,8,10,16,32").split(",")]:
        n_fm = (n_in - T) // D
        n_am = (n_in - T) // D + 1
        y = torch.empty(n_am, dtype=torch.float32, device=dev)
        fm = timed(abi.lib.gsdrFmDemod, (1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(),
                                         n_fm, 0, stream))
        am = timed(abi.lib.gsdrAmDemod, (1e6, 0.0, 1e5, D, 0, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(), n_am,
                                         0, stream))
        print(f"D={D}: FM {fm:.1f} us ({n_in / fm:,.0f} Ms/s) | AM {am:.1f} us ({n_in / am:,.0f} Ms/s)")


if __name__ == "__main__":
    main()
