#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): 127-tap complex<float> FIR, decimate-by-4, 64 M samples per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one gsdrFirFC call (the C ABI, through ctypes) over one channel of 67,108,987 complex
samples resident in HBM -> 2^24 complex outputs. Each rank owns an independent channel (seed
0x5EED + rank): channels shard across GPUs with no data-path collective, so scaling is weak.
torch.distributed is used only for the barrier and the max-over-ranks timing reduction.

Rank 0 prints ONE JSON line: value = input samples processed by all ranks / max-over-ranks wall
time of the K timed steps (Msamples/s), plus a `roofline` object for the FIR kernel (algorithmic
bytes per launch / mean launch time from HIP events on the launch stream) and a `cpu_baseline`
object (the C oracle timed on this host, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s + achieved HBM GB/s, 127-tap cplx FIR-dec4, 64M samp, 1/2/4/8 GPU"
TAPS, DECIM, N_OUT = 127, 4, 1 << 24
N_IN = (N_OUT - 1) * DECIM + TAPS  # 67,108,987
ALG_BYTES = 8 * N_IN + 8 * N_OUT + 4 * TAPS  # 671,090,132 B per launch
ALG_FLOP = 4 * TAPS * N_OUT
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md); measured streaming ceilings reported alongside
HBM_ACHIEVABLE_GBPS = 6300.0  # MI355X_MICROARCH.md, "HBM [CDNA4]": ~6.3 TB/s achievable
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_fir_fc_d4.json")
ROTATE = 3  # input batches cycled through (see main)
CPU_SAMPLE_S = 10.0  # wall seconds of CPU-baseline work (bounded sample of the workload)


def dist_env():
    """(rank, local_rank, world) from the torchrun environment, or a single process."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def channel_seed(rank: int) -> int:
    """Channel c is generated from seed 0x5EED + c (BASELINE config 4: one channel per GPU)."""
    return 0x5EED + rank


def reduce_max(value: float, device) -> float:
    """Max over ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def aggregate(samples_per_rank: int, world: int, steps: int, seconds_max: float) -> float:
    """Whole-job Msamples/s: every rank's input samples over the slowest rank's wall time."""
    return samples_per_rank * world * steps / seconds_max / 1e6


def load_pmc_traffic():
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py), or None."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), d
    except (OSError, ValueError):
        return None, None


def host_cores():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota when one is set (a GPU
    box shares the machine, and its quota, not nproc, is what a CPU job gets). (count, how)."""
    n = len(os.sched_getaffinity(0))
    how = "sched_getaffinity"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(-(-int(quota) // int(period))))
            if q < n:
                n, how = q, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return n, how


def native_oracle():
    """Build the C oracle for this host (-O3 -march=native, no contraction: the explicit fmaf calls stay
    the only fused operations) into a temporary directory; fall back to the prebuilt in-tree build.
    Returns the compile description. Must run before `oracle` is imported."""
    import subprocess
    import tempfile

    src = os.path.join(ROOT, "oracle", "gsdr_oracle.c")
    out = os.path.join(tempfile.mkdtemp(prefix="gsdr_oracle_"), "liboracle_native.so")
    flags = ["-O3", "-march=native", "-std=c11", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math"]
    try:
        subprocess.run(["gcc"] + flags + ["-I", os.path.join(ROOT, "oracle"), src, "-o", out, "-lm", "-lpthread"],
                       check=True, capture_output=True, timeout=120)
        os.environ["GSDR_ORACLE_LIB"] = out
        return "gcc " + " ".join(flags[:2] + flags[5:]) + " (built on this host)"
    except (OSError, subprocess.SubprocessError):
        return "prebuilt oracle/build/liboracle.so (gcc -O2 -mfma -ffp-contract=off)"


def _timed(fn, min_s, min_reps=3):
    """Median wall time of repeated fn() calls, repeated for at least min_s seconds."""
    times, t_start = [], time.perf_counter()
    while len(times) < min_reps or time.perf_counter() - t_start < min_s:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    times.sort()
    return times[len(times) // 2], len(times), sum(times)


def cpu_baselines(x_host, taps_np, threads, c5):
    """The C oracle (oracle/gsdr_oracle.c: scalar restatement of the reference kernels, one output per
    loop iteration, split over `threads` pthreads by output range) timed on this host for BASELINE
    configs 1, 2, 3 and 5, each on a bounded sample of its workload, with all cores and with one."""
    import numpy as np

    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from oracle import oracle as orc

    res = {}
    # config 2 (the headline): repeated passes over the full channel, ~10 s
    med, reps, tot = _timed(lambda: orc.fir_fc_mt(taps_np, x_host, DECIM, N_OUT, threads), CPU_SAMPLE_S)
    n1 = N_OUT // 16
    xs = np.ascontiguousarray(x_host[: (n1 - 1) * DECIM + TAPS])
    one, _, _ = _timed(lambda: orc.fir_fc_mt(taps_np, xs, DECIM, n1, 1), 1.0, 1)
    res["2"] = {"workload": "127-tap complex FIR, D = 4, 67,108,987 samples (gsdrFirFC)",
                "value": round(N_IN / med / 1e6, 2), "unit": "Msamples/s",
                "sample": f"{reps} passes over the full channel, {tot:.1f} s, median pass",
                "single_thread": round(((n1 - 1) * DECIM + TAPS) / one / 1e6, 2)}
    # config 1: 63-tap real FIR, no decimation, 1 M float samples
    t63 = lowpass_taps(63, 0.1)
    x1 = np.random.default_rng(1).uniform(-1, 1, 1 << 20).astype(np.float32)
    nout1 = x1.size - 63 + 1
    med, reps, tot = _timed(lambda: orc.fir_ff_mt(t63, x1, 1, nout1, threads), 2.0)
    one, _, _ = _timed(lambda: orc.fir_ff_mt(t63, x1, 1, nout1, 1), 1.0, 2)
    res["1"] = {"workload": "63-tap real FIR, no decimation, 1,048,576 float samples (gsdrFirFF)",
                "value": round(x1.size / med / 1e6, 2), "unit": "Msamples/s",
                "sample": f"{reps} passes over the full 1 M-sample input, {tot:.1f} s, median pass",
                "single_thread": round(x1.size / one / 1e6, 2)}
    # config 3: NCO + FIR + FM discriminator on config 3's signal; the oracle mixes every tap of every
    # window as the reference's k_Fm does (fm.cu:40-63), so a 2^18-output slice of the channel
    n3 = 1 << 18
    x3 = fm_test_signal(n3 * DECIM + TAPS, noise=0.05, seed=0x5EED)
    med, reps, tot = _timed(lambda: orc.fm_demod_mt(x3, taps_np, 1.0e6, 0.0, 1.0e5, 2.0e4, DECIM, 0, n3, threads),
                            3.0)
    one, _, _ = _timed(lambda: orc.fm_demod_mt(x3, taps_np, 1.0e6, 0.0, 1.0e5, 2.0e4, DECIM, 0, n3 // 16, 1), 1.0, 1)
    res["3"] = {"workload": "NCO + 127-tap FIR (D = 4) + FM discriminator (gsdrFmDemod)",
                "value": round(n3 * DECIM / med / 1e6, 2), "unit": "Msamples/s",
                "sample": f"{n3} outputs ({n3 * DECIM + TAPS} samples) of config 3's signal, {reps} passes, "
                          f"{tot:.1f} s, median pass",
                "single_thread": round((n3 // 16) * DECIM / one / 1e6, 2)}
    # config 5: modulate -> AWGN -> demodulate (reference cuCabsf rule, exhaustive 256-point search) on a
    # 2^20-symbol slice of the GPU's symbols; the GPU's noisy symbols and decisions for that slice are
    # checked against the oracle here (the full 2^24 round trip is tests/test_gpu_qpsk.py)
    if c5 is not None:
        table = orc.qpsk256_table(0, 1.0)
        syms, rx_gpu, dec_gpu, sigma, seed = c5
        k = syms.size

        def round_trip():
            rx = orc.qpsk256_mod_awgn(table, syms, sigma, seed, 0, nthreads=threads)
            return rx, orc.qpsk256_demod(table, rx, nthreads=threads)

        med, reps, tot = _timed(round_trip, 3.0)
        rx, dec = round_trip()
        t1 = time.perf_counter()
        orc.qpsk256_demod(table, orc.qpsk256_mod_awgn(table, syms[: k // 16], sigma, seed, 0), nthreads=1)
        one = time.perf_counter() - t1
        res["5"] = {"workload": "QPSK256 rectangular modulate -> AWGN (sigma 0.02) -> demodulate",
                    "value": round(k / med / 1e6, 2), "unit": "Msymbols/s",
                    "sample": f"{k} symbols (the first of the GPU run's 2^24), {reps} passes, {tot:.1f} s, median",
                    "single_thread": round((k // 16) / one / 1e6, 2),
                    "gpu_noisy_symbols_bit_exact": bool(rx.tobytes() == rx_gpu.tobytes()),
                    "gpu_decisions_bit_exact": bool(np.array_equal(dec, dec_gpu))}
    return res


def settle_clocks(torch, step, max_launches, window=25, tol=0.01, min_launches=400):
    """The GPU ramps its clock over the first tens of milliseconds of sustained load (measured: the
    headline kernel drops from ~200 us to ~140 us per launch over ~200 launches, tools/sustained_probe.py).
    After the W warmup steps, keep launching untimed windows of `window` steps -- at least `min_launches`, then
    until two consecutive windows agree within `tol` (or `max_launches`) -- so the timed steps see the
    steady-state clock a continuously streaming receiver runs at. (Round 6: stopping at the first two windows
    within 2 %, as rounds 1-5 did, could end the settle after 50 launches with the clock still ramping: the
    headline then measured 145 us against 137 us for the same launches timed after it.) Returns the number of
    extra untimed launches."""
    n, prev = 0, None
    max_launches = max(max_launches, min_launches)
    while n < max_launches:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(window):
            step()
        b.record()
        torch.cuda.synchronize()
        n += window
        t = a.elapsed_time(b)
        if n >= min_launches and prev is not None and abs(t - prev) <= tol * prev:
            break
        prev = t
    return n


def time_abi(torch, fn, argsets, reps=50, settle=400):
    """Per-launch time of a C-ABI call rotating over pre-marshalled argument sets (one per input
    batch): untimed warm-up + clock settle, then `reps` launches inside one HIP event pair."""
    cnt = [0]

    def step():
        rc = fn(*argsets[cnt[0] % len(argsets)])
        cnt[0] += 1
        assert rc == 0, rc

    for _ in range(5):
        step()
    settle_clocks(torch, step, settle)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


PROBES_LIB = os.path.join(ROOT, "build", "probes", "libgsdr_probes.so")


def staging_ceiling(torch, xs, ys, taps, dev_index, stream):
    """Two ceilings for the headline kernel's traffic, from the separate probes build (`make probes`,
    never the product library), timed the same way on the same buffers:
      * stream: variant 111, a plain streaming kernel moving exactly the FIR's bytes (8 N_in read with
        non-temporal 16-byte loads, 8 N_out written, fully coalesced, no LDS, no arithmetic): what this
        4:1 read:write mix streams at on this box -- the device-copy ceiling the FIR is compared with;
      * staging_only / compute_only: variants 107 / 104, the headline kernel itself without its
        multiply-adds / without its staging (the power-cap split of DESIGN.md section 3.1).
    None when the probes library was not built."""
    if not os.path.exists(PROBES_LIB):
        return None
    import ctypes

    lib = ctypes.CDLL(PROBES_LIB)
    fn = lib.gsdrxFirFCVariant
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
    out = {}
    for v, name in ((111, "stream"), (107, "staging_only"), (104, "compute_only")):
        argsets = [(v, DECIM, taps.data_ptr(), TAPS, xb.data_ptr(), yb.data_ptr(), N_OUT, dev_index, stream)
                   for xb, yb in zip(xs, ys)]
        out[name] = time_abi(torch, fn, argsets, reps=100, settle=600)
    return out


def fm_channel(torch, n, device, seed, n0=0):
    """Config 3's input generated on the device: constant-envelope FM, carrier +0.1 fs,
    message tone 0.001 fs, peak deviation 0.02 fs, amplitude 1, plus AWGN sigma 0.05 per axis; samples
    n0 .. n0 + n - 1 of the channel (consecutive batches continue the same signal)."""
    import math

    idx = torch.arange(n0, n0 + n, dtype=torch.float64, device=device)
    ph = 2 * math.pi * 0.1 * idx + (0.02 / 0.001) * torch.sin(2 * math.pi * 0.001 * idx)
    del idx
    x = torch.polar(torch.ones_like(ph), ph).to(torch.complex64)
    del ph
    g = torch.Generator(device=device).manual_seed(seed)
    x += (torch.randn(2 * n, dtype=torch.float32, device=device, generator=g) * 0.05).view(torch.complex64)
    return x


def fm_reference_windows(torch, x, taps, fs, tune, chan, dev_hz, n0, starts, width):
    """Config 3's chain restated in float64 with torch, on the tensor's own device, for output windows
    [s, s + width) of one gsdrFmDemod call (decimation 4, firstSampleIndex n0): the exact-integer NCO
    phase P(n) = (n0 + n) inc mod 2^32 with inc = llround((tune - chan) / fs 2^32),
    the FIR y[k] = sum_i t_i x[4k + i] e^{j 2 pi P(4k + i) / 2^32} (fir.cu:49-71) and the discriminator
    g arg(y[k + 1] conj y[k]) with g = fs / (2 pi dev) in float32 (fm.cu:66-68, 203). An independent
    checker for the multi-GPU leg (the C oracle stays with the tests and the cpu_baseline leg)."""
    import math

    import numpy as np

    T = taps.numel()
    df = float(np.float32(tune) - np.float32(chan))
    red = math.fmod(df / float(np.float32(fs)) * 4294967296.0, 4294967296.0)
    inc = int(math.floor(abs(red) + 0.5)) * (1 if red >= 0 else -1) % (1 << 32)
    g = float(np.float32(fs) / (np.float32(2.0) * np.float32(math.pi) * np.float32(dev_hz)))
    t64 = taps.to(torch.float64)
    outs = []
    for s0 in starts:
        idx = torch.arange(4 * s0, 4 * (s0 + width) + T, dtype=torch.int64, device=x.device)
        ph = ((idx + n0) * inc) % (1 << 32)
        rot = torch.polar(torch.ones(idx.numel(), dtype=torch.float64, device=x.device),
                          ph.to(torch.float64) * (2 * math.pi / 4294967296.0))
        z = x[4 * s0:4 * (s0 + width) + T].to(torch.complex128) * rot
        y = (z.unfold(0, T, 4)[:width + 1] * t64).sum(dim=1)
        outs.append(g * torch.angle(y[1:] * torch.conj(y[:-1])))
    return outs, g


def fm_multi_gpu(torch, device, taps, rank, world, steps):
    """Config 4: one config-3 FM channel per GPU (seed 0x5EED + rank), no exchange; every rank times its
    own launches between barriers and the slowest rank sets the aggregate. Outside the timed region each
    rank checks four 4096-output windows of its own output against a float64 restatement of the chain
    (fm_reference_windows, wrapped-angle bar 1e-5 of pi g) and digests it; the per-rank flags and digests
    are gathered to rank 0 for the line."""
    from gsdr_amd import abi

    fs, tune, chan, dev_hz = 1.0e6, 0.0, 1.0e5, 2.0e4
    n_fm = (1 << 24) - 1
    n_in = n_fm * DECIM + TAPS
    stream = torch.cuda.current_stream(device).cuda_stream
    xs = [fm_channel(torch, n_in, device, channel_seed(rank) + 1000 * k, k * n_in) for k in range(ROTATE)]
    ys = [torch.empty(n_fm, dtype=torch.float32, device=device) for _ in range(ROTATE)]
    y = ys[0]
    argsets = [(fs, tune, chan, dev_hz, DECIM, 0, taps.data_ptr(), TAPS, x.data_ptr(), yb.data_ptr(), n_fm,
                device.index, stream) for x, yb in zip(xs, ys)]
    torch.cuda.synchronize()
    t_solo, t = time_solo_then_all(torch, rank, lambda: time_abi(torch, abi.lib.gsdrFmDemod, argsets, reps=steps))
    t_max = reduce_max(t, device)
    t_ranks = [r[0] for r in gather_rows(torch, [t], rank, world, device)]
    # parity of this rank's channel (batch 0), after the timed region
    assert abi.lib.gsdrFmDemod(*argsets[0]) == 0
    torch.cuda.synchronize()
    width = 4096
    starts = [0, n_fm // 3, 2 * n_fm // 3, n_fm - width]
    refs, g = fm_reference_windows(torch, xs[0], taps, fs, tune, chan, dev_hz, 0, starts, width)
    err = 0.0
    for s0, r in zip(starts, refs):
        d = torch.remainder(y[s0:s0 + width].double() - r + math.pi * g, 2 * math.pi * g) - math.pi * g
        err = max(err, float(d.abs().max()) / (math.pi * g))
    digest = int(y.view(torch.int32).to(torch.int64).sum()) % (1 << 48)
    rows = gather_rows(torch, [1.0 if err <= 1e-5 else 0.0, err, float(digest)], rank, world, device)
    del xs, ys, y
    return {"config": "BASELINE configs[3]: one NCO + 127-tap FIR + FM channel (67,108,987 samples of config 3's "
                      "signal) per GPU, independent channels, no collective",
            "n_gpus": world, "us_per_launch_max_over_ranks": round(t_max * 1e6, 2),
            "us_per_launch_per_rank": [round(v * 1e6, 2) for v in t_ranks],
            "aggregate_msamples_per_s": round(world * n_in / t_max / 1e6, 1),
            "solo_us_per_launch_rank0": round(t_solo * 1e6, 2) if t_solo else None,
            "solo_msamples_per_s_rank0": round(n_in / t_solo / 1e6, 1) if t_solo else None,
            "scaling_efficiency": round(t_solo / t_max, 4) if t_solo else None,
            "scaling_efficiency_def": "agg(n) / (n agg(1)) with agg(1) = rank 0's channel timed alone in this job "
                                      "(every other rank idle at a barrier) just before the concurrent run",
            "parity_ok": [bool(r[0] == 1.0) for r in rows],
            "parity_max_wrapped_err_over_pi_g": [float(r[1]) for r in rows],
            "output_digest": [int(r[2]) for r in rows],
            "parity_check": "per rank, 4 x 4096 outputs of its own channel vs a float64 torch restatement of the "
                            "chain (fm_reference_windows), wrapped-angle bar 1e-5 of pi g; digest = sum of the "
                            "output's int32 bit patterns mod 2^48"}


def rank_identity(torch, dev_index, backend, world):
    """What this rank ran on, for the N > 1 line: host, the device's PCI domain:bus:device and UUID (from
    the HIP runtime through torch), the process-group backend and its world size."""
    import socket

    p = torch.cuda.get_device_properties(dev_index)
    pci = f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}"
    return {"host": socket.gethostname(), "device_index": dev_index, "pci": pci, "uuid": str(getattr(p, "uuid", "")),
            "name": p.name, "backend": backend, "world_size": world}


def gather_objects(obj, world):
    """Every rank's object, in rank order (one all_gather_object; the object itself when not distributed)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def distinct_devices(idents):
    """True when no two ranks report the same physical device (host + PCI address + UUID)."""
    keys = [(d["host"], d["pci"], d["uuid"]) for d in idents]
    return len(set(keys)) == len(keys)


def validate_ranks(idents, world, rehearse):
    """The N > 1 line's self-check: every rank reports the same backend and world size as rank 0's job, and the
    ranks sit on distinct GPUs -- unless BENCH_REHEARSE=1, where ranks deliberately share one card (gloo).
    Returns a list of problems (empty = valid)."""
    bad = []
    if len(idents) != world:
        bad.append(f"{len(idents)} rank records for world size {world}")
    if any(d["world_size"] != world for d in idents):
        bad.append("ranks disagree on the world size")
    if len({d["backend"] for d in idents}) != 1:
        bad.append("ranks disagree on the process-group backend")
    want = "gloo" if rehearse else "nccl"
    if world > 1 and any(d["backend"] != want for d in idents):
        bad.append(f"backend is not {want}")
    if world > 1 and not rehearse and not distinct_devices(idents):
        bad.append("two ranks report the same GPU")
    return bad


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 for the rendezvous of a self-launched job."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n: int, port: int, argv) -> list:
    """The torchrun command a plain `python bench.py --gpus N` (N > 1) runs as a child: one rank process per GPU
    on this node, rendezvous on 127.0.0.1:port, every bench argument passed through unchanged."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_env(port: int) -> dict:
    """The child job's environment: this one plus the rendezvous address (HSA_ENABLE_IPC_MODE_LEGACY and the
    rest are inherited unchanged)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    return env


def self_launch(n: int, argv, rehearse: bool) -> int:
    """`python bench.py --gpus N` with N > 1 outside torch.distributed.run: start the N rank processes (torchrun as a
    child process; this process never initialises the GPU and never execs) and return the job's exit status. The
    ranks print the one JSON line (rank 0) to the inherited stdout. Refuses, with no child started, when fewer than
    N devices are visible and this is not a BENCH_REHEARSE=1 rehearsal (ranks sharing one card)."""
    import subprocess

    if not rehearse:
        import torch  # device_count() enumerates without creating a HIP context on this image

        ndev = torch.cuda.device_count()
        if ndev < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {ndev} (BENCH_REHEARSE=1 rehearses the N > 1 "
                  "path with ranks sharing one card)", file=sys.stderr, flush=True)
            return 2
    port = free_port()
    if os.environ.get("BENCH_LAUNCH_PRINT") == "1":  # launcher plumbing check (tests/test_multi_gloo.py)
        print(json.dumps({"cmd": launch_cmd(n, port, argv), "port": port}), flush=True)
    return subprocess.run(launch_cmd(n, port, argv), env=launch_env(port)).returncode


def time_solo(torch, rank, fn_time):
    """fn_time() on rank 0 alone, every other rank idle at a barrier: the in-job N = 1 reference. Seconds on rank
    0, None elsewhere."""
    barrier()
    solo = fn_time() if rank == 0 else None
    barrier()
    return solo


def time_solo_then_all(torch, rank, fn_time):
    """Time fn_time() on rank 0 alone (every other rank idle at a barrier), then on all ranks at once. Returns
    (solo seconds on rank 0 or None elsewhere, this rank's concurrent seconds). The solo figure is the in-job
    N = 1 reference for the scaling efficiency agg(n) / (n agg(1)) = t_solo / t_max."""
    barrier()
    solo = fn_time() if rank == 0 else None
    barrier()
    t = fn_time()
    barrier()
    return solo, t


def gather_rows(torch, vals, rank, world, device):
    """Every rank's list of floats, gathered to all ranks (rows in rank order) by one sum-reduction of a
    zero matrix whose row `rank` is this rank's values (float64: the digests are exact below 2^53)."""
    import torch.distributed as dist

    m = torch.zeros((world, len(vals)), dtype=torch.float64)
    m[rank] = torch.tensor(vals, dtype=torch.float64)
    if dist.is_available() and dist.is_initialized() and world > 1:
        if dist.get_backend() != "gloo":
            m = m.to(device)
        dist.all_reduce(m, op=dist.ReduceOp.SUM)
    return m.cpu().tolist()


def secondary_configs(torch, ops, device, taps):
    """Config 3 (fused NCO + FIR + FM, 64 M samples), the int8 I/Q front end on
    the config-2 and config-3 shapes, and config 5 (QPSK256 16 M symbols): kernel times from HIP
    events, reported beside the headline line."""
    import ctypes

    import numpy as np

    from gsdr_amd import abi

    out = {}
    fs, tune, chan, dev_hz = 1.0e6, 0.0, 1.0e5, 2.0e4
    n_fm = (1 << 24) - 1
    n_in = n_fm * DECIM + TAPS
    g = torch.Generator(device=device).manual_seed(0x5EED)
    stream = torch.cuda.current_stream(device).cuda_stream
    # config 3's signal (constant-envelope FM + AWGN), consecutive batches of one channel
    xs = [fm_channel(torch, n_in, device, 0x5EED + 1000 * k, k * n_in) for k in range(ROTATE)]
    # one output buffer per input batch: no timed launch writes (or reads) a buffer the cache still holds
    ys = [torch.empty(n_fm, dtype=torch.float32, device=device) for _ in range(ROTATE)]
    argsets = [(fs, tune, chan, dev_hz, DECIM, 0, taps.data_ptr(), TAPS, x.data_ptr(), yb.data_ptr(), n_fm,
                device.index, stream) for x, yb in zip(xs, ys)]
    t = time_abi(torch, abi.lib.gsdrFmDemod, argsets)
    b = 8 * n_in + 4 * n_fm + 4 * TAPS
    out["fm_chain"] = {"config": "NCO + 127-tap FIR (D=4) + FM discriminator, 67,108,987 samples of constant-envelope "
                                 "FM + AWGN (BASELINE configs[2])",
                       "us_per_launch": round(t * 1e6, 2), "msamples_per_s": round(n_in / t / 1e6, 1),
                       "alg_gbps": round(b / t / 1e9, 1), "alg_bytes_per_launch": b}
    # multi-channel chain: C channels from one read of the input
    for C in (4, 16):
        chans = (ctypes.c_float * C)(*[float(f) for f in np.linspace(-0.4, 0.4, C) * fs])
        devs = (ctypes.c_float * C)(*([dev_hz] * C))
        yms = [torch.empty(C * n_fm, dtype=torch.float32, device=device) for _ in range(ROTATE if C < 8 else 1)]
        argsets = [(fs, tune, chans, devs, C, DECIM, 0, taps.data_ptr(), TAPS, 0, x.data_ptr(),
                    yms[k % len(yms)].data_ptr(), n_fm, device.index, stream) for k, x in enumerate(xs)]
        t = time_abi(torch, abi.lib.gsdrxFmDemodMulti, argsets, reps=20)
        out[f"fm_multi_{C}ch"] = {
            "config": f"{C} FM channels of config 3's input in one launch (gsdrxFmDemodMulti)",
            "us_per_launch": round(t * 1e6, 2), "us_per_channel": round(t * 1e6 / C, 2),
            "channel_msamples_per_s": round(C * n_in / t / 1e6, 1),
            "speedup_vs_single_calls": round(C * out["fm_chain"]["us_per_launch"] / (t * 1e6), 2)}
        del yms
    # streaming object on complex float input: one launch per call (round 4), C equal
    # chunks per 64 M-sample channel pass, against one call
    out["fir_stream"] = stream_rate(torch, abi, device, taps, xs, stream, out_fir_call(torch, abi, device, taps, xs,
                                                                                      stream),
                                    kind=0, fmt=0, chunk_counts=(1, 8, 32), label="config 2's complex float channel "
                                    "through gsdrxStream (CF32 FIR, D = 4), C chunks a pass")
    out["fm_stream"] = stream_rate(torch, abi, device, taps, xs, stream, out["fm_chain"]["us_per_launch"] * 1e-6,
                                   kind=1, fmt=0, chunk_counts=(1, 8, 32), call_sizes=(1 << 16, 1 << 18, 1 << 20),
                                   label="config 3's channel through gsdrxStream (CF32 FM chain, D = 4), C chunks a "
                                   "pass or receiver-sized calls of 2^16 / 2^18 / 2^20 samples")
    # multi-channel stream (rows 1 x 3): 8 FM channels of one RF input, 2^20-sample calls, one grouped launch a call
    out["fm_stream_multi_8ch"] = stream_rate(
        torch, abi, device, taps, xs, stream, out["fm_chain"]["us_per_launch"] * 1e-6, kind=1, fmt=0, chunk_counts=(1,),
        call_sizes=(1 << 20,), channels=8,
        label="8 FM channels of config 3's input through one gsdrxStreamCreateMulti stream (CF32, D = 4): one grouped "
              "launch a call")
    del xs
    # int8 I/Q front end fused into the filter: 2 instead of 8 input bytes per sample; the FM chain gets
    # config 3's signal quantised to int8 (x 100), consecutive batches of one channel
    x8s = []
    for b in range(ROTATE):
        xc = fm_channel(torch, n_in, device, 0x5EED + 1000 * b, b * n_in)  # config 3's batches, as above
        x8s.append(torch.clamp(torch.round(torch.view_as_real(xc).reshape(-1) * 100), -128, 127).to(torch.int8))
        del xc
    argsets = [(fs, tune, chan, dev_hz, DECIM, 0, taps.data_ptr(), TAPS, x.data_ptr(), yb.data_ptr(), n_fm,
                device.index, stream) for x, yb in zip(x8s, ys)]
    t = time_abi(torch, abi.lib.gsdrxFmDemodInt8, argsets)
    b = 2 * n_in + 4 * n_fm + 4 * TAPS
    out["fm_chain_int8"] = {"config": "config 3 from int8 I/Q (gsdrxFmDemodInt8)", "us_per_launch": round(t * 1e6, 2),
                            "msamples_per_s": round(n_in / t / 1e6, 1), "alg_gbps": round(b / t / 1e9, 1),
                            "alg_bytes_per_launch": b}
    argsets = [(fs, tune, chan, DECIM, 0, taps.data_ptr(), TAPS, x.data_ptr(), yb.data_ptr(), n_fm, device.index,
                stream) for x, yb in zip(x8s, ys)]
    t = time_abi(torch, abi.lib.gsdrxAmDemodInt8, argsets)
    out["am_chain_int8"] = {"config": "NCO + 127-tap FIR (D = 4) + AM envelope on config 3's int8 I/Q (gsdrxAmDemodInt8)",
                            "us_per_launch": round(t * 1e6, 2), "msamples_per_s": round(n_in / t / 1e6, 1),
                            "alg_gbps": round(b / t / 1e9, 1), "alg_bytes_per_launch": b}
    del ys
    yfs = [torch.empty(N_OUT, dtype=torch.complex64, device=device) for _ in range(ROTATE)]
    argsets = [(DECIM, taps.data_ptr(), TAPS, x.data_ptr(), yf.data_ptr(), N_OUT, device.index, stream)
               for x, yf in zip(x8s, yfs)]
    t = time_abi(torch, abi.lib.gsdrxFirFCInt8, argsets)
    b = 2 * N_IN + 8 * N_OUT + 4 * TAPS
    out["fir_int8"] = {"config": "config 2 from int8 I/Q (gsdrxFirFCInt8), 67,108,987 samples",
                       "us_per_launch": round(t * 1e6, 2), "msamples_per_s": round(N_IN / t / 1e6, 1),
                       "alg_gbps": round(b / t / 1e9, 1), "alg_bytes_per_launch": b,
                       "fma_tflops": round(4 * TAPS * N_OUT / t / 1e12, 1)}
    out["fir_int8_stream"] = stream_rate(torch, abi, device, taps, x8s, stream, t, kind=0, fmt=1, chunk_counts=(1, 2, 8),
                                         label="config 2's int8 I/Q channel through gsdrxStream (CS8 FIR, D = 4), C "
                                         "chunks a pass")
    out["fm_int8_stream"] = stream_rate(torch, abi, device, taps, x8s, stream, out["fm_chain_int8"]["us_per_launch"] * 1e-6,
                                        kind=1, fmt=1, chunk_counts=(1, 8), call_sizes=(1 << 16, 1 << 18, 1 << 20),
                                        label="config 3's int8 I/Q channel through gsdrxStream (CS8 FM chain, D = 4), "
                                        "C chunks a pass or receiver-sized calls")
    del x8s, yfs
    # true recursive IIR: 4th-order Butterworth over 2^24 samples
    from scipy import signal as sps

    bb, aa = (torch.tensor(v, dtype=torch.float32, device=device) for v in sps.butter(4, 0.1))
    for dt, name, nbytes in ((torch.float32, "gsdrIirFF", 4), (torch.complex64, "gsdrIirCC", 8)):
        n = 1 << 24
        # 4 (x, y) pairs rotating: 512 MB (real) / 1 GB (complex) per cycle, so every launch streams from and to
        # HBM (rounds 1-5 timed one 2^24-sample pair, whose 128 / 256 MB the Infinity Cache could hold)
        pairs = [(torch.rand(n, dtype=dt, device=device, generator=g), torch.empty(n, dtype=dt, device=device))
                 for _ in range(4)]
        argsets = [(bb.data_ptr(), aa.data_ptr(), 5, None, None, xi.data_ptr(), yi.data_ptr(), n, device.index, stream)
                   for xi, yi in pairs]
        t = time_abi(torch, getattr(abi.lib, name), argsets, reps=100, settle=200)
        t_one = time_abi(torch, getattr(abi.lib, name), argsets[:1], reps=100, settle=50)
        out[f"iir_{'cc' if dt == torch.complex64 else 'ff'}"] = {
            "config": f"{name}, 4th-order Butterworth (K = 5), 2^24 samples, parallel scan, 4 rotating (x, y) pairs",
            "us_per_launch": round(t * 1e6, 2), "msamples_per_s": round(n / t / 1e6, 1),
            "alg_gbps": round(2 * nbytes * n / t / 1e9, 1),
            "one_pair_us_per_launch": round(t_one * 1e6, 2)}
        del pairs
    # config 1 (BASELINE configs[0]: the reference's CPU-runnable case) on the GPU: 63-tap real FIR, no
    # decimation, 1 M float samples -- one launch is a few microseconds, so launch overhead dominates
    from gsdr_amd.signals import lowpass_taps

    x1 = torch.rand(1 << 20, device=device, generator=g) * 2 - 1
    t63 = torch.from_numpy(lowpass_taps(63, 0.1)).to(device)
    n1 = x1.numel() - 63 + 1
    y1 = torch.empty(n1, dtype=torch.float32, device=device)
    argsets = [(1, t63.data_ptr(), 63, x1.data_ptr(), y1.data_ptr(), n1, device.index, stream)]
    t = time_abi(torch, abi.lib.gsdrFirFF, argsets, reps=200, settle=100)
    out["fir_ff_config1"] = {"config": "BASELINE configs[0]: 63-tap real FIR (gsdrFirFF), no decimation, 1,048,576 "
                                       "float samples", "us_per_launch": round(t * 1e6, 2),
                             "msamples_per_s": round(x1.numel() / t / 1e6, 1)}
    del x1, y1
    # BASELINE configs[4]: QPSK256 modulate -> AWGN -> demodulate, 2^24 symbols. Three rotating sets (symbols,
    # noisy symbols, decisions; 3 x 168 MB per cycle), C-ABI calls with pre-marshalled arguments (time_abi).
    n = 1 << 24
    ops.qpsk256_init(0, 1.0, device.index)
    sigma, seed = 0.02, 0x5EED0005
    fplain, fmod, fdem = abi.lib.gsdrQpsk256Modulate, abi.lib.gsdrxQpsk256ModulateAwgn, abi.lib.gsdrQpsk256Demodulate
    ffused = abi.lib.gsdrxQpsk256ModulateAwgnDemodulate
    sets = [(torch.randint(0, 256, (n,), dtype=torch.uint8, device=device, generator=g),
             torch.empty(n, dtype=torch.complex64, device=device), torch.empty(n, dtype=torch.uint8, device=device))
            for _ in range(ROTATE)]
    ptrs = [(s.data_ptr(), tx.data_ptr(), d.data_ptr()) for s, tx, d in sets]
    dv = device.index

    def round_trip(sp, tp, dp):  # the pipeline: demodulate the buffer the modulator has just written
        return fmod(sp, tp, n, 0, sigma, seed, 0, dv, stream) or fdem(tp, dp, n, 0, dv, stream)

    t_fused = time_abi(torch, ffused, [(sp, tp, dp, n, 0, sigma, seed, 0, dv, stream) for sp, tp, dp in ptrs], reps=50)
    t_rt = time_abi(torch, round_trip, ptrs, reps=50, settle=200)
    t_plain = time_abi(torch, fplain, [(sp, tp, n, 1.0, 0, dv, stream) for sp, tp, _ in ptrs])
    t_awgn = time_abi(torch, fmod, [(sp, tp, n, 0, sigma, seed, 0, dv, stream) for sp, tp, _ in ptrs])
    t_dem = time_abi(torch, fdem, [(tp, dp, n, 0, dv, stream) for _, tp, dp in ptrs])
    # rounds 1-5 timed each kernel on ONE buffer set, which the 256 MB Infinity Cache holds between launches
    t_awgn1 = time_abi(torch, fmod, [(sp, tp, n, 0, sigma, seed, 0, dv, stream) for sp, tp, _ in ptrs[:1]], settle=50)
    t_dem1 = time_abi(torch, fdem, [(tp, dp, n, 0, dv, stream) for _, tp, dp in ptrs[:1]], settle=50)
    syms, tx, rx_bytes = sets[0]
    # the fused pass on set 0 (what the cpu_baseline leg checks), and that it equals the two calls bit for bit
    assert round_trip(*ptrs[0]) == 0
    tx2, dec2 = tx.clone(), rx_bytes.clone()
    assert ffused(ptrs[0][0], ptrs[0][1], ptrs[0][2], n, 0, sigma, seed, 0, dv, stream) == 0
    torch.cuda.synchronize()
    fused_equal = bool(torch.equal(tx.view(torch.float32), tx2.view(torch.float32)) and torch.equal(rx_bytes, dec2))
    del tx2, dec2
    out["qpsk256"] = {
        "config": "QPSK256 rectangular, 2^24 symbols: modulate + counter-based AWGN sigma 0.02/axis -> demodulate, "
                  "3 rotating buffer sets",
        "round_trip_us": round(t_fused * 1e6, 2),
        "round_trip_def": "gsdrxQpsk256ModulateAwgnDemodulate: the round trip in one pass -- it writes the 2^24 noisy "
                          "symbols AND the 2^24 decisions, bit-identical to gsdrxQpsk256ModulateAwgn followed by "
                          "gsdrQpsk256Demodulate (fused_equals_two_calls), but demodulates each noisy symbol from the "
                          "registers it was formed in instead of reading the 134 MB back; buffer sets rotating",
        "fused_equals_two_calls": fused_equal,
        "round_trip_msymbols_per_s": round(n / t_fused / 1e6, 1),
        # config 5's algorithmic bytes as the two calls move them: 2^24 + 8 * 2^24 (modulate) +
        # 8 * 2^24 + 2^24 (demodulate); the fused pass moves 2^24 + 8 * 2^24 + 2^24 of them
        "round_trip_frac_of_8tbps": round(18 * n / t_fused / 1e9 / HBM_PEAK_GBPS, 4),
        "fused_moved_bytes_frac_of_8tbps": round(10 * n / t_fused / 1e9 / HBM_PEAK_GBPS, 4),
        "two_call_pipeline_us": round(t_rt * 1e6, 2),
        "two_call_pipeline_def": "gsdrxQpsk256ModulateAwgn into a buffer set, then gsdrQpsk256Demodulate of that buffer "
                                 "(the demodulation reads the noisy symbols its modulation just wrote), sets rotating",
        "two_call_pipeline_frac_of_8tbps": round(18 * n / t_rt / 1e9 / HBM_PEAK_GBPS, 4),
        "modulate_awgn_us": round(t_awgn * 1e6, 2), "demodulate_us": round(t_dem * 1e6, 2),
        "per_kernel_sum_us": round((t_awgn + t_dem) * 1e6, 2),
        "modulate_us": round(t_plain * 1e6, 2),
        "alg_gbps_mod": round(9 * n / t_plain / 1e9, 1), "alg_gbps_mod_awgn": round(9 * n / t_awgn / 1e9, 1),
        "alg_gbps_demod": round(9 * n / t_dem / 1e9, 1),
        "one_buffer_set": {"modulate_awgn_us": round(t_awgn1 * 1e6, 2), "demodulate_us": round(t_dem1 * 1e6, 2),
                           "sum_us": round((t_awgn1 + t_dem1) * 1e6, 2),
                           "what": "each kernel looping over one buffer set (cache-resident), as rounds 1-5 timed"},
        "decision_rule": "reference cuCabsf argmin (qpsk256.cu:171-181), bit-exact"}
    for rec in out.values():  # every byte-rate figure also as a fraction of the 8 TB/s HBM peak
        for k in [k for k in rec if k.startswith("alg_gbps")]:
            rec[k.replace("alg_gbps", "frac_of_8tbps")] = round(rec[k] / HBM_PEAK_GBPS, 4)
    out["qpsk256"]["ser_awgn"] = round(float((rx_bytes != syms).float().mean()), 6)
    out["qpsk256"]["squared_distance_rule_disagreements"] = sq_rule_disagreements(torch, tx, 0)
    k5 = 1 << 20
    c5 = (syms[:k5].cpu().numpy(), tx[:k5].cpu().numpy(), rx_bytes[:k5].cpu().numpy(), sigma, seed)
    # circular table (per-cell candidate lists), the same symbols, sigma 0.01/axis (torch noise), rotating sets
    ops.qpsk256_init(1, 1.0, dv)
    for s, txk, _ in sets:
        ops.qpsk256_modulate(s, 1, out=txk)
        txk += torch.randn(n, dtype=torch.complex64, device=device, generator=g) * (0.01 * np.sqrt(2.0))
    tc = time_abi(torch, fdem, [(tp, dp, n, 1, dv, stream) for _, tp, dp in ptrs])
    assert fdem(ptrs[0][1], ptrs[0][2], n, 1, dv, stream) == 0
    torch.cuda.synchronize()
    out["qpsk256"]["demodulate_circular_us"] = round(tc * 1e6, 2)
    out["qpsk256"]["ser_circular_sigma_0.01"] = round(float((rx_bytes != syms).float().mean()), 6)
    del sets
    return out, c5


def out_fir_call(torch, abi, device, taps, xs, stream):
    """One gsdrFirFC call over a whole 64 M-sample channel (the stream lines' reference)."""
    y = torch.empty(N_OUT, dtype=torch.complex64, device=device)
    argsets = [(DECIM, taps.data_ptr(), TAPS, x.data_ptr(), y.data_ptr(), N_OUT, device.index, stream) for x in xs]
    return time_abi(torch, abi.lib.gsdrFirFC, argsets)


def stream_rate(torch, abi, device, taps, xs, stream, t_call, kind, fmt, chunk_counts, label, call_sizes=(),
                channels=1):
    """SURVEY.md 8(f) row 1 (and row 2 for int8 I/Q): a 64 M-sample channel fed through a gsdrxStream in C
    equal chunks per pass, passes rotating over the batches, against one call of the entry point (t_call).
    Every gsdrxStreamProcess call is ONE launch of the kernel one monolithic call runs (seam samples from
    the history buffer, next history written by the launch: the int8 matrix-core kernels since round 3,
    the float tiled kernels since round 4), so the difference is the per-launch fixed cost times C and the
    host's issue time per call (host_us_per_call, measured over the same loop). call_sizes: passes in calls of
    that many samples (receiver-sized chunks); channels > 1: a gsdrxStreamCreateMulti stream of that many FM
    channels of the same input."""
    import ctypes

    import numpy as np

    res = {"config": label, "single_call_us": round(t_call * 1e6, 2)}
    sb = 2 if fmt == 1 else 8
    # a call can emit the history's outputs too; a C-channel stream writes channel c at c * capacity
    ycap = N_OUT + 1024
    y = torch.empty(channels * ycap, dtype=torch.complex64 if kind == 0 else torch.float32, device=device)
    yp = y.data_ptr()
    written = ctypes.c_size_t()
    wref = ctypes.byref(written)
    f = ctypes.c_float
    plan = [(c, f"{c}_chunks", N_IN // c) for c in chunk_counts]
    plan += [(-(-N_IN // size), f"per_call_{size}_samples", size) for size in call_sizes]
    for chunks, name, cs in plan:
        h = ctypes.c_void_p()
        if channels == 1:
            rc = abi.lib.gsdrxStreamCreate(ctypes.byref(h), kind, fmt, DECIM, taps.data_ptr(), TAPS, f(1.0e6), f(0.0),
                                           f(1.0e5), f(2.0e4), 0, device.index)
        else:
            chans = (f * channels)(*[float(v) for v in (np.linspace(-0.4, 0.4, channels) * 1.0e6)])
            devs = (f * channels)(*([2.0e4] * channels))
            rc = abi.lib.gsdrxStreamCreateMulti(ctypes.byref(h), kind, fmt, DECIM, taps.data_ptr(), TAPS, f(1.0e6),
                                                f(0.0), ctypes.cast(chans, ctypes.c_void_p),
                                                ctypes.cast(devs, ctypes.c_void_p), channels, 0, device.index)
        assert rc == 0, rc
        argsets = []
        for x in xs:
            for c in range(chunks):
                n = cs if c < chunks - 1 else N_IN - cs * (chunks - 1)
                argsets.append((h, x.data_ptr() + sb * cs * c, n, yp, ycap, wref, stream))
        fn = abi.lib.gsdrxStreamProcess
        k = 0
        for _ in range(max(20, min(8 * chunks, 2048))):
            assert fn(*argsets[k % len(argsets)]) == 0
            k += 1
        torch.cuda.synchronize()
        calls = max(50 * chunks, 200) if chunks <= 32 else max(2 * chunks, 256)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        h0 = time.perf_counter()
        for _ in range(calls):
            fn(*argsets[k % len(argsets)])
            k += 1
        h1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / calls * chunks * 1e-3  # per channel pass
        abi.lib.gsdrxStreamDestroy(h)
        res[name] = {"us_per_pass": round(t * 1e6, 2), "samples_per_call": cs, "calls_per_pass": chunks,
                     "us_per_call": round(t * 1e6 / chunks, 3), "msamples_per_s": round(N_IN / t / 1e6, 1),
                     "vs_single_call": round(channels * t_call / t, 3),
                     "host_us_per_call": round((h1 - h0) / calls * 1e6, 2)}
        if channels > 1:
            res[name]["channel_msamples_per_s"] = round(channels * N_IN / t / 1e6, 1)
    if channels > 1:
        res["channels"] = channels
        res["vs_single_call_def"] = "C x (one single-channel call over the whole channel) / (one pass of the C-channel stream)"
    return res


def sq_rule_disagreements(torch, rx, ctype, chunk=1 << 19):
    """Symbols (of rx) whose squared-distance argmin differs from the library's decision rule, the
    reference's cuCabsf argmin: how often the two rules part (near-ties only). Counted with torch on
    the GPU: d = (rx - c)^2 summed per axis in float32, first index of the minimum."""
    from gsdr_amd import ops

    table = ops.qpsk256_modulate(torch.arange(256, dtype=torch.uint8, device=rx.device), ctype)
    dec = ops.qpsk256_demodulate(rx, ctype)
    tr, ti = table.real[None, :], table.imag[None, :]
    n = 0
    for k in range(0, rx.numel(), chunk):
        r = rx[k:k + chunk]
        dx = r.real[:, None] - tr
        dy = r.imag[:, None] - ti
        d = dx * dx + dy * dy
        n += int((torch.argmin(d, dim=1).to(torch.uint8) != dec[k:k + chunk]).sum())
    return n


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variant", type=int, default=-1, help="FC/D=4 tile shape (gsdrxFirFCVariant), -1 = default")
    ap.add_argument("--settle-max", type=int, default=600,
                    help="max extra untimed launches while the clock ramps (0 = off); reported as clock_settle_launches")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    args = ap.parse_args()
    # BENCH_REHEARSE=1 (rehearsal only, never a reported number): gloo instead of RCCL and rank r on
    # cuda:(r mod device_count), so the N > 1 code path can run on a one-GPU box with ranks sharing it.
    rehearse = os.environ.get("BENCH_REHEARSE") == "1"
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: start the N rank processes ourselves (before any GPU call)
        sys.exit(self_launch(args.gpus, sys.argv[1:], rehearse))

    import torch
    import torch.distributed as dist

    rank, local_rank, world = dist_env()
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} does not match --gpus {args.gpus}")
    if os.environ.get("BENCH_LAUNCH_PROBE") == "1":  # launcher plumbing check: report the rank's env, touch no GPU
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world,
                          "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}), flush=True)
        return
    ndev = torch.cuda.device_count()
    if rehearse:
        dev_index = local_rank % ndev
    elif local_rank < ndev:
        dev_index = local_rank
    elif ndev == 1:
        dev_index = 0  # one visible device per rank (a per-rank HIP_VISIBLE_DEVICES); validate_ranks checks they differ
    else:
        raise SystemExit(f"local rank {local_rank} but only {ndev} visible devices")
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
    backend = dist.get_backend() if world > 1 else "none"
    idents = gather_objects(rank_identity(torch, dev_index, backend, world), world)
    problems = validate_ranks(idents, world, rehearse)
    if problems:
        raise SystemExit(f"rank {rank}: invalid multi-GPU job: {'; '.join(problems)}: {idents}")

    from gsdr_amd import ops
    from gsdr_amd.signals import lowpass_taps

    taps_np = lowpass_taps(TAPS, 0.1)
    taps = torch.from_numpy(taps_np).to(device)
    g = torch.Generator(device=device).manual_seed(channel_seed(rank))
    # The channel's samples arrive as consecutive 64 M-sample batches; ROTATE of them are resident in
    # HBM and step k filters batch k % ROTATE, so no step re-reads input the 256 MiB Infinity Cache
    # still holds from the previous step (3 x 537 MB): every step streams from HBM.
    xs = [(torch.rand(2 * N_IN, device=device, generator=g) * 2 - 1).view(torch.complex64)
          for _ in range(ROTATE)]
    x = xs[0]
    # ... and each batch has its own output buffer, so no step's 134 MB of outputs can stay in the cache
    # either: the working set of a step cycle is 3 x 671 MB, and every timed byte goes to or comes from HBM
    ys = [torch.empty(N_OUT, dtype=torch.complex64, device=device) for _ in range(ROTATE)]
    y = ys[0]
    counter = [0]
    # The timed step calls the C ABI exactly as an FFI caller would: arguments marshalled once, one
    # ctypes call per step (~2 us of host time), so launches queue ahead of the GPU instead of the
    # GPU waiting on Python (the torch-tensor wrapper in gsdr_amd.ops costs ~45 us per call).
    from gsdr_amd import abi

    stream = torch.cuda.current_stream(device).cuda_stream
    if args.variant >= 0:
        fn = abi.lib.gsdrxFirFCVariant
        argsets = [(args.variant, DECIM, taps.data_ptr(), TAPS, xb.data_ptr(), yb.data_ptr(), N_OUT, dev_index,
                    stream) for xb, yb in zip(xs, ys)]
    else:
        fn = abi.lib.gsdrFirFC
        argsets = [(DECIM, taps.data_ptr(), TAPS, xb.data_ptr(), yb.data_ptr(), N_OUT, dev_index, stream)
                   for xb, yb in zip(xs, ys)]

    def step():
        rc = fn(*argsets[counter[0] % ROTATE])
        counter[0] += 1
        if rc != 0:
            raise abi.GsdrError(fn.__name__, rc)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    settle = settle_clocks(torch, step, args.settle_max) if args.settle_max > 0 else 0
    barrier()
    solo_fir_s = None
    if world > 1:
        # the in-job N = 1 reference: rank 0's K launches with every other rank idle at the barrier
        def fir_k():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(args.steps):
                step()
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) / args.steps * 1e-3

        solo_fir_s = time_solo(torch, rank, fir_k)

    # One HIP event pair around the K timed launches, on the launch stream: an event record between
    # launches is itself a ~10 us GPU command (timestamp + cache flush) and would inflate both numbers.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    ev0.record()  # torch's current stream == the stream gsdrFirFC is launched on
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier()
    wall_max = reduce_max(wall, device)
    kern_s = ev0.elapsed_time(ev1) / args.steps * 1e-3  # mean launch duration (back-to-back launches)
    kern_s_max = reduce_max(kern_s, device)
    per_rank = gather_rows(torch, [kern_s, wall], rank, world, device)
    fm_multi = None
    if world > 1 and not args.no_secondary:
        fm_multi = fm_multi_gpu(torch, device, taps, rank, world, args.steps)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    value = aggregate(N_IN, world, args.steps, wall_max)
    achieved = ALG_BYTES / kern_s / 1e9
    traffic, pmc = load_pmc_traffic()
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: I/Q uniform[-1,1) complex64 per channel (torch generator seed 0x5EED + rank), "
                f"{ROTATE} x 64M-sample batches per channel cycled per step, "
                "127-tap Hamming-windowed sinc low-pass, fc = 0.1 fs",
        "config": {"workload": "127-tap complex<float> FIR decimate-by-4, 64M samples per GPU (BASELINE configs[1])",
                   "taps": TAPS, "decimation": DECIM, "input_samples": N_IN, "outputs": N_OUT,
                   "channels": world, "parallelism": f"independent channels, 1 per GPU x {world}",
                   "entry_point": "gsdrFirFC" if args.variant < 0 else f"gsdrxFirFCVariant({args.variant})"},
        "achieved_hbm_gbps": round(achieved, 1),
        "clock_settle_launches": settle,
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "kernel": "k_fir_poly<float, float2, D=4, R=4, JC=16, WG=256>",
            "alg_bytes_per_launch": ALG_BYTES,
            "kernel_us_mean": round(kern_s * 1e6, 2),
            "kernel_us_max_over_ranks": round(kern_s_max * 1e6, 2),
            "timing": "HIP event pair on the launch stream around the K back-to-back timed launches, input and output "
                      f"buffers rotating over {ROTATE} batches (no step re-reads or re-writes a cached buffer)",
            "alg_tflops": round(ALG_FLOP / kern_s / 1e12, 2),
        },
    }
    if world > 1:
        line["ranks"] = [dict(d, rank=r, fir_kernel_us=round(p[0] * 1e6, 2), wall_ms=round(p[1] * 1e3, 3))
                         for r, (d, p) in enumerate(zip(idents, per_rank))]
        line["multi_gpu_check"] = {
            "backend": backend, "world_size": world, "distinct_devices": distinct_devices(idents),
            "solo_fir_kernel_us_rank0": round(solo_fir_s * 1e6, 2),
            "fir_scaling_efficiency": round(solo_fir_s / kern_s_max, 4),
            "fir_scaling_efficiency_def": "agg(n) / (n agg(1)) = t_solo / t_max: rank 0's K launches timed alone in this "
                                          "job (other ranks idle at a barrier) over the slowest rank's mean launch in "
                                          "the concurrent timed region",
            "validated": "ranks report one backend and world size; device host + PCI + UUID distinct per rank"
                         + (" (not required under BENCH_REHEARSE)" if rehearse else "")}
    if rehearse:
        line["rehearsal"] = "BENCH_REHEARSE=1: gloo, ranks sharing GPUs; not a measurement"
    if pmc:
        line["roofline"]["traffic_source"] = os.path.relpath(PMC_SUMMARY, ROOT)
    line["roofline"]["guide_achievable_gbps"] = HBM_ACHIEVABLE_GBPS
    line["roofline"]["frac_of_guide_achievable"] = round(achieved / HBM_ACHIEVABLE_GBPS, 4)
    if world == 1 and not args.no_secondary:
        # the round-5 measurement (every step writing the same output buffer) beside the rotated one: what the
        # 256 MB Infinity Cache had been worth to the headline figure
        one_y = [(DECIM, taps.data_ptr(), TAPS, xb.data_ptr(), y.data_ptr(), N_OUT, dev_index, stream) for xb in xs]
        t_one = time_abi(torch, abi.lib.gsdrFirFC, one_y, reps=args.steps, settle=200)
        line["roofline"]["one_output_buffer"] = {
            "kernel_us_mean": round(t_one * 1e6, 2), "frac": round(ALG_BYTES / t_one / 1e9 / HBM_PEAK_GBPS, 4),
            "what": "the same launches with every step writing one output buffer (rounds 1-5's bench), timed after "
                    "the rotated region: the output may then stay in the 256 MB Infinity Cache"}
        ceil = staging_ceiling(torch, xs, ys, taps, dev_index, stream)
        if ceil is not None:
            cp = ALG_BYTES / ceil["stream"] / 1e9
            line["roofline"]["measured_copy_gbps"] = round(cp, 1)
            line["roofline"]["frac_of_measured_copy"] = round(achieved / cp, 4)
            line["roofline"]["measured_copy_source"] = (
                "probes build gsdrxFirFCVariant 111: a streaming kernel moving exactly this launch's bytes (8 N_in "
                "read with non-temporal 16-byte loads, 8 N_out written, coalesced, no arithmetic), same buffers")
            st_gbps = ALG_BYTES / ceil["staging_only"] / 1e9
            line["roofline"]["staging_ceiling"] = {
                "gbps": round(st_gbps, 1),
                "us": round(ceil["staging_only"] * 1e6, 2),
                "frac_of_ceiling": round(achieved / st_gbps, 4),
                "compute_only_us": round(ceil["compute_only"] * 1e6, 2),
                "source": "probes build (make probes), gsdrxFirFCVariant 107: this kernel's staging and stores "
                          "without the multiply-adds; 104: the multiply-adds without the staging",
            }
    c5 = None
    if world == 1 and not args.no_secondary:
        line["secondary"], c5 = secondary_configs(torch, ops, device, taps)
    if fm_multi is not None:
        line["secondary"] = {"fm_chain_multi_gpu": fm_multi}
    if world == 1 and not args.no_cpu_baseline:
        threads, how = host_cores()
        build = native_oracle()
        per = cpu_baselines(x.cpu().numpy(), taps_np, threads, c5)
        gpu = {"2": N_IN / kern_s / 1e6}
        sec = line.get("secondary", {})
        if "fir_ff_config1" in sec:
            gpu["1"] = sec["fir_ff_config1"]["msamples_per_s"]
        if "fm_chain" in sec:
            gpu["3"] = sec["fm_chain"]["msamples_per_s"]
        if "qpsk256" in sec:
            gpu["5"] = sec["qpsk256"]["round_trip_msymbols_per_s"]
        for k, v in per.items():
            v["cores"] = threads
            if k in gpu:
                v["gpu_value"] = round(gpu[k], 1)
                v["gpu_over_cpu"] = round(gpu[k] / v["value"], 1)
        c2 = per["2"]
        line["cpu_baseline"] = {"value": c2["value"], "unit": "Msamples/s", "cores": threads, "kind": "port",
                                "sample": c2["sample"] + " (config 2; configs 1, 3, 5 under `configs`)",
                                "cores_source": how, "build": build,
                                "single_thread_msamples_per_s": c2["single_thread"], "configs": per}
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
