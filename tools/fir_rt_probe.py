"""Development probe for k_fir_rt (decimations without a compile-time shape): gsdrFirFC at D = argv[1]
(default 50), T = 127, 2^26 input samples, 20 launches (for rocprofv3 --kernel-trace / --pmc), then the
mean launch time by HIP events over 50 more."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 50
T, L = 127, 1 << 26
N = (L - T) // D + 1
dev = torch.device("cuda", 0)
x = (torch.rand(2 * L, device=dev) * 2 - 1).view(torch.complex64)
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
y = torch.empty(N, dtype=torch.complex64, device=dev)
for _ in range(20):
    ops.fir(taps, x, D, N, out=y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    ops.fir(taps, x, D, N, out=y)
e1.record()
torch.cuda.synchronize()
print(f"gsdrFirFC D={D} T={T} 2^26 samples: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")
