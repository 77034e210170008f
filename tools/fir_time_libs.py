"""Time the FIR entry points (gsdrFirFF / FC / CF / CC, T = 127, 2^26 input samples) with HIP events in each
given build of libgsdr.so, side by side in one process, flagging outputs that differ from the first build
(development tool). FIR_D = comma-separated decimations (default 1)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd.signals import lowpass_taps  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n_in, T = 1 << 26, 127
    g = torch.Generator(device=dev).manual_seed(1)
    xr = torch.rand(n_in, device=dev, generator=g) * 2 - 1
    xc = (torch.rand(2 * n_in, device=dev, generator=g) * 2 - 1).view(torch.complex64)
    tr = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    tc = (tr.to(torch.complex64) * (1 + 0.5j)).contiguous()
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(p) for p in sys.argv[1:]]
    outs = {}
    ds = [int(v) for v in os.environ.get("FIR_D", "1").split(",")]
    for rep, D in [(r, d) for d in ds for r in range(2 if len(libs) > 1 else 1)]:
        n_out = (n_in - T) // D + 1
        for path in libs:
            lib = ctypes.CDLL(path)
            res = []
            for name, taps, x, odt in (("gsdrFirFF", tr, xr, torch.float32), ("gsdrFirFC", tr, xc, torch.complex64),
                                       ("gsdrFirCF", tc, xr, torch.complex64), ("gsdrFirCC", tc, xc, torch.complex64)):
                fn = getattr(lib, name)
                fn.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
                y = torch.empty(n_out, dtype=odt, device=dev)
                a = (D, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(), n_out, 0, stream)
                for _ in range(30):
                    assert fn(*a) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(100):
                    fn(*a)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 100 * 1e3
                res.append(f"{name} {us:.1f} us ({n_in / us:,.0f} Ms/s)")
                key = (name, D)
                if key in outs:
                    if not torch.equal(outs[key], y):
                        res[-1] += " [differs from the first build]"
                else:
                    outs[key] = y.clone()
            print(f"D={D}", os.path.relpath(path, ROOT), " | ".join(res))


if __name__ == "__main__":
    main()
