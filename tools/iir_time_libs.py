"""Time gsdrIirFF / gsdrIirCC (4th-order Butterworth, 2^24 samples) with HIP events in each given build of
libgsdr.so, side by side in one process, flagging outputs that differ from the first build
(development tool)."""
import ctypes
import os
import sys

import torch
from scipy import signal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 24
    b, a = (torch.tensor(v, dtype=torch.float32, device=dev) for v in signal.butter(4, 0.1))
    K = b.numel()
    g = torch.Generator(device=dev).manual_seed(5)
    xs = {"FF": torch.rand(n, device=dev, generator=g) * 2 - 1,
          "CC": (torch.rand(2 * n, device=dev, generator=g) * 2 - 1).view(torch.complex64)}
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(p) for p in sys.argv[1:]]
    first = {}
    for rep in range(2):
        for path in libs:
            lib = ctypes.CDLL(path)
            res = []
            for name, x in xs.items():
                fn = getattr(lib, "gsdrIir" + name)
                y = torch.empty_like(x)
                args = (b.data_ptr(), a.data_ptr(), K, None, None, x.data_ptr(), y.data_ptr(), n, 0, stream)
                fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
                for _ in range(30):
                    assert fn(*args) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(100):
                    fn(*args)
                e1.record()
                torch.cuda.synchronize()
                tag = ""
                if name in first:
                    if not torch.equal(first[name], y):
                        tag = " [differs]"
                else:
                    first[name] = y.clone()
                res.append(f"gsdrIir{name} {e0.elapsed_time(e1) / 100 * 1e3:.1f} us{tag}")
            print(os.path.relpath(path, ROOT), " | ".join(res))


if __name__ == "__main__":
    main()
