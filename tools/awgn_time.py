"""Time gsdrxQpsk256ModulateAwgn (2^24 symbols, rectangular, sigma 0.02) with HIP events in each given
build of libgsdr.so side by side (development tool); the in-tree build first."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 24
    syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.complex64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(p) for p in sys.argv[1:]]
    for rep in range(2):
        for path in libs:
            lib = ctypes.CDLL(path)
            assert lib.gsdrQpsk256InitConstellation(ctypes.c_uint32(0), ctypes.c_float(1.0), 0, ctypes.c_void_p(stream)) == 0
            fn = lib.gsdrxQpsk256ModulateAwgn
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_void_p]
            args = (syms.data_ptr(), out.data_ptr(), n, 0, 0.02, 0x5EED0005, 0, 0, stream)
            for _ in range(200):
                fn(*args)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(200):
                fn(*args)
            e.record()
            torch.cuda.synchronize()
            print(f"{os.path.relpath(path, ROOT):32s} modulate+AWGN {s.elapsed_time(e) / 200 * 1e3:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
