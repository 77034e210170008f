"""A/B of the int8 matrix-core paths' per-launch cost (development tool): gsdrxFirFCInt8 on config 2's
int8 channel as one call, and through a gsdrxStream (CS8 FIR, D = 4) in 1 / 2 / 8 / 32 chunks a pass, plus
gsdrxFmDemodInt8 on the same channel, for the in-tree libgsdr.so and each library given as an argument,
side by side in one process (HIP events)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd.signals import lowpass_taps  # noqa: E402

D, T, N_IN = 4, 127, 67_108_987
N_OUT = (N_IN - T) // D + 1


def main():
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randint(-128, 128, (2 * N_IN,), dtype=torch.int8, device=dev, generator=g) for _ in range(3)]
    y = torch.empty(N_OUT + 1024, dtype=torch.complex64, device=dev)
    yf = torch.empty(N_OUT, dtype=torch.float32, device=dev)
    libs = [os.path.join(ROOT, "gsdr_amd", "libgsdr.so")] + [os.path.abspath(a) for a in sys.argv[1:]]

    def timed(fn, args, reps):
        k = 0
        for _ in range(max(20, reps // 5)):
            assert fn(*args[k % len(args)]) == 0
            k += 1
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn(*args[k % len(args)])
            k += 1
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    for rep in range(2):
        for path in libs:
            lib = ctypes.CDLL(path)
            res = []
            f = lib.gsdrxFirFCInt8
            f.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
            res.append("fir %.1f" % timed(f, [(D, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(), N_OUT, 0, stream)
                                              for x in xs], 100))
            fm = lib.gsdrxFmDemodInt8
            fm.argtypes = [ctypes.c_float] * 4 + [ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
                                                  ctypes.c_void_p]
            nf = (N_IN - T - D) // D
            res.append("fm %.1f" % timed(fm, [(1.0e6, 0.0, 1.0e5, 2.0e4, D, 0, taps.data_ptr(), T, x.data_ptr(),
                                               yf.data_ptr(), nf, 0, stream) for x in xs], 100))
            sp = lib.gsdrxStreamProcess
            sp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_void_p, ctypes.c_void_p]
            written = ctypes.c_size_t()
            for chunks in (1, 2, 8, 32):
                h = ctypes.c_void_p()
                lib.gsdrxStreamCreate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float, ctypes.c_float,
                                                  ctypes.c_float, ctypes.c_float, ctypes.c_size_t, ctypes.c_int32]
                assert lib.gsdrxStreamCreate(ctypes.byref(h), 0, 1, D, taps.data_ptr(), T, 1.0, 0.0, 0.0, 1.0, 0, 0) == 0
                cs = N_IN // chunks
                args = []
                for x in xs:
                    for c in range(chunks):
                        n = cs if c < chunks - 1 else N_IN - cs * (chunks - 1)
                        args.append((h, x.data_ptr() + 2 * cs * c, n, y.data_ptr(), y.numel(), ctypes.byref(written),
                                     stream))
                res.append("stream x%d %.1f" % (chunks, timed(sp, args, 30 * chunks) * chunks))
                lib.gsdrxStreamDestroy(h)
            print(os.path.relpath(path, ROOT), " | ".join(res), "(us per channel pass)", flush=True)


if __name__ == "__main__":
    main()
