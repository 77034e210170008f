#!/usr/bin/env python3
"""A few launches of each round-4 profiling target (development tool, for tools/pmc_cmd.sh): config 3 from
int8 I/Q (gsdrxFmDemodInt8), config 5's channel and rectangular demodulation (2^24 symbols), and config 3's
float FM chain. Prints the mean launch time of each (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import ops  # noqa: E402
from gsdr_amd.signals import lowpass_taps  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))
dev = torch.device("cuda", 0)
D, T, N_IN = 4, 127, 67_108_987
n_fm = (N_IN - T) // D
taps = torch.from_numpy(lowpass_taps(T, 0.1)).to(dev)
g = torch.Generator(device=dev).manual_seed(1)
x8 = torch.randint(-128, 128, (2 * N_IN,), dtype=torch.int8, device=dev, generator=g)
xf = (torch.rand(2 * N_IN, device=dev, generator=g) * 2 - 1).view(torch.complex64)
out = torch.empty(n_fm, dtype=torch.float32, device=dev)
n = 1 << 24
syms = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
rx = torch.empty(n, dtype=torch.complex64, device=dev)
dec = torch.empty(n, dtype=torch.uint8, device=dev)
ops.qpsk256_init(0, 1.0, 0)


def timed(name, fn):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / REPS * 1e3:.1f} us", flush=True)


timed("fm_chain_int8", lambda: ops.fm_demod(x8, taps, 1e6, 0.0, 1e5, 2e4, D, 0, n_fm, out=out))
timed("am_chain_int8", lambda: ops.am_demod(x8, taps, 1e6, 0.0, 1e5, D, 0, n_fm, out=out))
yc = torch.empty(n_fm + 1, dtype=torch.complex64, device=dev)
timed("fir_int8", lambda: ops.fir(taps, x8, D, n_fm + 1, out=yc))
timed("qpsk256_mod_awgn", lambda: ops.qpsk256_modulate_awgn(syms, 0, 0.02, 0x5EED0005, 0, out=rx))
timed("qpsk256_demod_rect", lambda: ops.qpsk256_demodulate(rx, 0, out=dec))
timed("qpsk256_mod", lambda: ops.qpsk256_modulate(syms, 0, 1.0, out=rx))
timed("fm_chain", lambda: ops.fm_demod(xf, taps, 1e6, 0.0, 1e5, 2e4, D, 0, n_fm, out=out))

# IIR (4th-order Butterworth, 2^24 samples) as bench.py times it (no history buffers) and with history
from scipy import signal as sps  # noqa: E402

from gsdr_amd import abi  # noqa: E402

stream = torch.cuda.current_stream(dev).cuda_stream
bb, aa = (torch.tensor(v, dtype=torch.float32, device=dev) for v in sps.butter(4, 0.1))
for dt, name in ((torch.float32, "gsdrIirFF"), (torch.complex64, "gsdrIirCC")):
    xi = torch.rand(1 << 24, dtype=dt, device=dev, generator=g)
    yi = torch.empty_like(xi)
    hx = torch.zeros(4, dtype=dt, device=dev)
    hy = torch.zeros(4, dtype=dt, device=dev)
    fn = getattr(abi.lib, name)
    timed(name, lambda: fn(bb.data_ptr(), aa.data_ptr(), 5, None, None, xi.data_ptr(), yi.data_ptr(), 1 << 24, 0, stream))
    timed(name + "+history", lambda: fn(bb.data_ptr(), aa.data_ptr(), 5, hx.data_ptr(), hy.data_ptr(), xi.data_ptr(),
                                        yi.data_ptr(), 1 << 24, 0, stream))
