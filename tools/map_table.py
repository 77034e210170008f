"""Development tool: steady-state time of the memory-bound maps (QPSK, element-wise, quad demod) at
2^24 elements, as effective GB/s (bytes moved / time), beside a device copy of the same size."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 24
g = torch.Generator(device=dev).manual_seed(1)
c = torch.rand(n, dtype=torch.complex64, device=dev, generator=g) - (0.5 + 0.5j)
c2 = torch.rand(n, dtype=torch.complex64, device=dev, generator=g)
f = torch.rand(n, dtype=torch.float32, device=dev, generator=g)
i8 = torch.randint(-128, 128, (n,), dtype=torch.int8, device=dev, generator=g)
bits = torch.randint(0, 256, (n // 4,), dtype=torch.uint8, device=dev, generator=g)
oc = torch.empty(n, dtype=torch.complex64, device=dev)
of = torch.empty(n, dtype=torch.float32, device=dev)
ob = torch.empty(n // 4, dtype=torch.uint8, device=dev)
cp = torch.empty_like(c)
ops.qpsk256_init(0, 1.0)
sym256 = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
rx256 = ops.qpsk256_modulate(sym256, 0) + 0.02 * c
o256 = torch.empty(n, dtype=torch.uint8, device=dev)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


rows = [
    ("device copy (complex64)", lambda: cp.copy_(c), 16 * n),
    ("device fill (write only, complex64)", lambda: oc.fill_(1 + 1j), 8 * n),
    ("device fill (write only, float32)", lambda: of.fill_(1.0), 4 * n),
    ("gsdrQpskModulate", lambda: ops.qpsk_modulate(bits, n, 1.0, out=oc), n // 4 + 8 * n),
    ("gsdrQpskDemodulate", lambda: ops.qpsk_demodulate(c, n, out=ob), 8 * n + n // 4),
    ("gsdrMultiplyCC", lambda: ops.multiply(c, c2, out=oc), 24 * n),
    ("gsdrAddConstCC", lambda: ops.add_const(c, 1 + 2j, out=oc), 16 * n),
    ("gsdrAddToMagnitude", lambda: ops.add_to_magnitude(c, 0.5, out=oc), 16 * n),
    ("gsdrMagnitude", lambda: ops.magnitude(c, out=of), 12 * n),
    ("gsdrQuadFmDemod", lambda: ops.quad_fm_demod(c, 1.0, num_outputs=n - 1, out=of), 12 * n),
    ("gsdrCosineC", lambda: ops.cosine(0.0, 1000.0, n, True, dev, out=oc), 8 * n),
    ("gsdrInt8ToNormFloat", lambda: ops.int8_to_norm_float(i8, out=of), 5 * n),
    ("gsdrQpsk256Modulate (rect)", lambda: ops.qpsk256_modulate(sym256, 0, out=oc), 9 * n),
    ("gsdrQpsk256Demodulate (rect)", lambda: ops.qpsk256_demodulate(rx256, 0, out=o256), 9 * n),
]
print("| entry (2^24 elements) | us | effective GB/s |")
print("|---|---|---|")
for name, fn, nbytes in rows:
    t = timeit(fn)
    print(f"| {name} | {t * 1e6:.1f} | {nbytes / t / 1e9:,.0f} |", flush=True)
