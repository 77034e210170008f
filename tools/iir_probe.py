"""Development probe: 20 IIR calls (4th-order Butterworth, 2^24 samples, or 2^argv[2]) for rocprofv3 --kernel-trace.
    python tools/iir_probe.py ff|cc [log2 n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from scipy import signal  # noqa: E402

from gsdr_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
b, a = (torch.tensor(v, dtype=torch.float32, device=dev) for v in signal.butter(4, 0.1))
cplx = len(sys.argv) > 1 and sys.argv[1] == "cc"
log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
x = torch.rand(1 << log2n, dtype=torch.complex64 if cplx else torch.float32, device=dev)
y = torch.empty_like(x)
for _ in range(20):
    ops.iir(b, a, x, out=y)
torch.cuda.synchronize()
