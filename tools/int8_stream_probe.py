"""Development probe for rocprofv3 --kernel-trace: config 2's int8 channel through a gsdrxStream (CS8 FIR,
D = 4) in C chunks (argv[1], default 32), 10 passes."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

D, T, N_IN = 4, 127, 67_108_987
chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev).cuda_stream
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
x = torch.randint(-128, 128, (2 * N_IN,), dtype=torch.int8, device=dev)
y = torch.empty(N_IN // D + 1024, dtype=torch.complex64, device=dev)
h = ctypes.c_void_p()
assert abi.lib.gsdrxStreamCreate(ctypes.byref(h), 0, 1, D, taps.data_ptr(), T, 1.0, 0.0, 0.0, 1.0, 0, 0) == 0
written = ctypes.c_size_t()
cs = N_IN // chunks
for _ in range(10):
    for c in range(chunks):
        n = cs if c < chunks - 1 else N_IN - cs * (chunks - 1)
        assert abi.lib.gsdrxStreamProcess(h, x.data_ptr() + 2 * cs * c, n, y.data_ptr(), y.numel(),
                                          ctypes.byref(written), stream) == 0
torch.cuda.synchronize()
abi.lib.gsdrxStreamDestroy(h)
