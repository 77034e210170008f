"""Debug (development tool): mismatches of the circular QPSK256 demod vs the oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from oracle import oracle as o  # noqa: E402

amp = 1.0
ops.qpsk256_init(1, amp)
table = o.qpsk256_table(1, amp)
rng = np.random.default_rng(100)
n = (1 << 22) + 4096 * 300 + 7
span = 2.2 * amp
rx = (rng.uniform(-span, span, n) + 1j * rng.uniform(-span, span, n)).astype(np.complex64)
got = ops.qpsk256_demodulate(torch.from_numpy(rx).cuda(), 1).cpu().numpy()
want = o.qpsk256_demod(table, rx)
bad = np.nonzero(got != want)[0]
print("mismatches", bad.size, "of", n)
for k in bad[:20]:
    r = rx[k]
    print(k, k % 4096, k // 4096, r, "got", got[k], "want", want[k],
          "d_got", abs(r - table[got[k]]), "d_want", abs(r - table[want[k]]))
