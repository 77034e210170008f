"""FM chain ablation timing (development tool): gsdrFmDemod from the main library and from builds with
the NCO mix removed (build/libgsdr_ablate1.so) or the discriminator replaced by a plain store
(build/libgsdr_ablate2.so), sustained back-to-back launches on config 3's input."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd.signals import lowpass_taps  # noqa: E402

T, D, N = 127, 4, (1 << 24) - 1
L = N * D + T
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
xs = [(torch.rand(2 * L, device=dev, generator=g) * 2 - 1).view(torch.complex64) for _ in range(3)]
taps = torch.from_numpy(lowpass_taps(T)).to(dev)
out = torch.empty(N, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for name in ("gsdr_amd/libgsdr.so", "build/libgsdr_ablate1.so", "build/libgsdr_ablate2.so"):
    lib = ctypes.CDLL(os.path.join(root, name))
    f = lib.gsdrFmDemod
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_float] * 4 + [ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
                                         ctypes.c_void_p]
    args = [(1e6, 0.0, 1e5, 2e4, D, 0, taps.data_ptr(), T, x.data_ptr(), out.data_ptr(), N, 0, stream) for x in xs]
    for i in range(300):
        f(*args[i % 3])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(1000):
        f(*args[i % 3])
    e.record()
    torch.cuda.synchronize()
    print(f"{name:32s} {s.elapsed_time(e):8.3f} us/launch", flush=True)
