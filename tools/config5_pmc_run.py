"""Config 5's two kernels back to back (2^24 symbols: modulate + AWGN, rectangular demodulation), 20 calls each,
for a rocprofv3 trace / PMC pass (tools/pmc.sh pmc_c5 python tools/config5_pmc_run.py)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsdr_amd import abi  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
n = 1 << 24
syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
rx = torch.empty(n, dtype=torch.complex64, device=dev)
dec = torch.empty(n, dtype=torch.uint8, device=dev)
lib = abi.lib
abi.check("init", lib.gsdrQpsk256InitConstellation(0, 1.0, 0, st))
for _ in range(20):
    abi.check("mod", lib.gsdrxQpsk256ModulateAwgn(syms.data_ptr(), rx.data_ptr(), n, 0, 0.02, 0x5EED0005, 0, 0, st))
    abi.check("demod", lib.gsdrQpsk256Demodulate(rx.data_ptr(), dec.data_ptr(), n, 0, 0, st))
torch.cuda.synchronize()
print("ok")
