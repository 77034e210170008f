"""Development tool: steady-state time of gsdrFir{FC,FF,CC,CF} over decimations and tap counts at
~64 M input samples (3 rotating batches, clock settled first), printed as a markdown table."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsdr_amd import abi  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
L = 1 << 26
CASES = [("FC", 4, 127), ("FC", 2, 127), ("FC", 8, 127), ("FC", 1, 127), ("FF", 4, 127), ("FF", 1, 63),
         ("CC", 4, 127), ("CF", 4, 127), ("FC", 4, 31), ("FC", 4, 255)]
sz = {"F": (torch.float32, 4), "C": (torch.complex64, 8)}
print("| entry | D | T | us / launch | Msamples/s | alg GB/s | alg TFLOP/s |")
print("|---|---|---|---|---|---|---|")
g = torch.Generator(device=dev).manual_seed(1)
for tt, D, T in CASES:
    tdt, tb = sz[tt[0]]
    xdt, xb = sz[tt[1]]
    ob = 8 if "C" in tt else 4
    N = (L - T) // D + 1
    taps = torch.rand(T, dtype=tdt, device=dev, generator=g)
    xs = [torch.rand(L, dtype=xdt, device=dev, generator=g) for _ in range(3)]
    y = torch.empty(N, dtype=torch.complex64 if ob == 8 else torch.float32, device=dev)
    fn = getattr(abi.lib, f"gsdrFir{tt}")
    args = [(D, taps.data_ptr(), T, x.data_ptr(), y.data_ptr(), N, 0, st) for x in xs]
    for i in range(300):  # warm + settle
        fn(*args[i % 3])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(100):
        fn(*args[i % 3])
    b.record()
    torch.cuda.synchronize()
    t = a.elapsed_time(b) / 100 * 1e-3
    flop = N * T * {"FF": 2, "FC": 4, "CF": 4, "CC": 8}[tt]
    print(f"| gsdrFir{tt} | {D} | {T} | {t * 1e6:.1f} | {L / t / 1e6:,.0f} | {(L * xb + N * ob) / t / 1e9:,.0f} | "
          f"{flop / t / 1e12:.1f} |", flush=True)
    del xs, y
