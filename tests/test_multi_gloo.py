"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py (independent channels, one per rank,
no data-path collective; barrier + max-over-ranks timing; whole-job aggregate). Each rank filters
its own channel with the CPU oracle standing in for the device (no GPU here) and the test checks
the bookkeeping, not the FIR: channels differ by seed, the reduced time is the slowest rank's, and
value = world x per-rank samples / max time (weak scaling)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from gsdr_amd.signals import lowpass_taps, uniform_iq
    from oracle import oracle as orc

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert bench.dist_env() == (rank, rank, world)
        seed = bench.channel_seed(rank)
        n_out, D, T = 4096, 4, 127
        x = uniform_iq((n_out - 1) * D + T, seed=seed)
        y = orc.fir(lowpass_taps(T), x, D, n_out)
        local_time = 0.010 * (rank + 1)  # rank 1 is the slow one
        bench.barrier()
        tmax = bench.reduce_max(local_time, torch.device("cpu"))
        digest = torch.tensor([float(np.abs(y).sum())])
        gathered = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(gathered, digest)  # test-side only: compare the channels the ranks produced
        # bench's own gather of the per-rank parity flags / digests (fm_multi_gpu)
        rows = bench.gather_rows(torch, [float(rank == rank), 0.5 * rank, float(10 + rank)], rank, world,
                                 torch.device("cpu"))
        # the N > 1 line's self-check: per-rank identities gathered in rank order (each rank claims its own
        # device here, as the GPU job does with one card per rank)
        ident = {"host": "h", "device_index": rank, "pci": f"0000:{rank + 1:02x}:00", "uuid": f"u{rank}",
                 "name": "n", "backend": dist.get_backend(), "world_size": dist.get_world_size()}
        idents = bench.gather_objects(ident, world)
        problems = bench.validate_ranks(idents, world, rehearse=True)
        # rank 0 alone, then all ranks: the solo figure exists on rank 0 only
        solo, conc = bench.time_solo_then_all(torch, rank, lambda: 1.0 + rank)
        q.put((rank, seed, tmax, [float(g) for g in gathered], rows, idents, problems, solo, conc))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_channels_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [r[1] for r in results]
    assert seeds == [0x5EED, 0x5EED + 1]  # one independent channel per rank
    assert all(abs(r[2] - 0.020) < 1e-12 for r in results)  # every rank sees the slowest rank's time
    digests = results[0][3]
    assert digests == results[1][3] and digests[0] != digests[1]  # channels really differ
    for r in results:  # every rank holds every rank's row, in rank order
        assert r[4] == [[1.0, 0.0, 10.0], [1.0, 0.5, 11.0]]
        assert [d["pci"] for d in r[5]] == ["0000:01:00", "0000:02:00"] and r[6] == []
    assert results[0][7] == 1.0 and results[1][7] is None
    assert [r[8] for r in results] == [1.0, 2.0]


def _ident(rank, pci, backend="nccl", world=2, host="h"):
    return {"host": host, "device_index": rank, "pci": pci, "uuid": "u" + pci, "name": "MI355X", "backend": backend,
            "world_size": world}


def test_validate_ranks_rules():
    """bench.validate_ranks: distinct GPUs required for a measured N > 1 line, shared ones allowed only under the
    rehearsal flag; backend and world size must agree across ranks."""
    sys.path.insert(0, ROOT)
    import bench

    good = [_ident(0, "0000:05:00"), _ident(1, "0000:15:00")]
    assert bench.validate_ranks(good, 2, rehearse=False) == []
    shared = [_ident(0, "0000:05:00"), _ident(1, "0000:05:00")]
    assert any("same GPU" in p for p in bench.validate_ranks(shared, 2, rehearse=False))
    assert bench.validate_ranks([dict(d, backend="gloo") for d in shared], 2, rehearse=True) == []
    # same PCI address on two hosts is two GPUs
    assert bench.validate_ranks([_ident(0, "0000:05:00", host="a"), _ident(1, "0000:05:00", host="b")], 2,
                                rehearse=False) == []
    assert bench.validate_ranks([_ident(0, "0000:05:00"), _ident(1, "0000:15:00", world=3)], 2, rehearse=False)
    assert bench.validate_ranks([_ident(0, "0000:05:00"), _ident(1, "0000:15:00", backend="gloo")], 2,
                                rehearse=False)
    assert bench.validate_ranks(good, 2, rehearse=True)  # a rehearsal must run over gloo
    assert bench.validate_ranks(good[:1], 2, rehearse=False)  # a missing rank
    assert bench.validate_ranks([_ident(0, "0000:05:00", backend="none", world=1)], 1, rehearse=False) == []


def test_fm_reference_windows_matches_oracle():
    """bench.fm_reference_windows (the float64 checker of the multi-GPU leg) against the C oracle's FM chain
    on config 3's signal, on the CPU."""
    sys.path.insert(0, ROOT)
    import math

    import bench
    from gsdr_amd.signals import fm_test_signal, lowpass_taps
    from oracle import oracle as orc

    T, n, n0 = 127, 3000, 0
    fs, tune, chan, dev = 1.0e6, 0.0, 1.0e5, 2.0e4
    x = fm_test_signal(n * 4 + T + 8, noise=0.05, seed=3)
    taps = lowpass_taps(T, 0.1)
    refs, g = bench.fm_reference_windows(torch, torch.from_numpy(x), torch.from_numpy(taps), fs, tune, chan, dev, n0,
                                         [0, 1000, n - 512], 512)
    want = orc.fm_demod(x, taps, fs, tune, chan, dev, 4, n0, n)
    for s0, r in zip([0, 1000, n - 512], refs):
        d = np.remainder(r.numpy() - want[s0:s0 + 512] + math.pi * g, 2 * math.pi * g) - math.pi * g
        assert np.max(np.abs(d)) / (math.pi * g) <= 2e-6


def test_aggregate_is_weak_scaling():
    sys.path.insert(0, ROOT)
    import bench

    one = bench.aggregate(bench.N_IN, 1, 10, 1.0e-3)
    eight = bench.aggregate(bench.N_IN, 8, 10, 1.0e-3)
    assert eight == pytest.approx(8 * one)
    assert one == pytest.approx(bench.N_IN * 10 / 1.0e-3 / 1e6)


def test_launch_cmd_and_env():
    """bench.launch_cmd / launch_env: the torchrun child a plain `python bench.py --gpus N` starts."""
    sys.path.insert(0, ROOT)
    import bench

    cmd = bench.launch_cmd(8, 29512, ["--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29512" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "20", "--warmup", "5"]
    os.environ["RANK"] = "3"  # stale rank variables of an outer job must not leak into the child
    try:
        env = bench.launch_env(29512)
    finally:
        del os.environ["RANK"]
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29512" and "RANK" not in env


@pytest.mark.timeout(240)
def test_plain_bench_self_launches_ranks():
    """`python bench.py --gpus 2` outside torchrun starts its own two rank processes: each rank sees RANK /
    LOCAL_RANK / WORLD_SIZE and the 127.0.0.1 rendezvous the parent chose (BENCH_LAUNCH_PROBE: the ranks
    report their environment and stop before any device work, so this runs on the CPU)."""
    import json
    import subprocess

    env = dict(os.environ, BENCH_REHEARSE="1", BENCH_LAUNCH_PROBE="1", BENCH_LAUNCH_PRINT="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    launch = [d for d in lines if "cmd" in d]
    ranks = sorted((d for d in lines if "rank" in d), key=lambda d: d["rank"])
    assert len(launch) == 1 and "--nproc-per-node=2" in launch[0]["cmd"]
    port = str(launch[0]["port"])
    assert [(d["rank"], d["local_rank"], d["world"]) for d in ranks] == [(0, 0, 2), (1, 1, 2)]
    assert all(d["master"] == ["127.0.0.1", port] for d in ranks)


@pytest.mark.timeout(120)
def test_plain_bench_refuses_without_enough_gpus():
    """Without BENCH_REHEARSE, `python bench.py --gpus 2` on a box with fewer than two visible GPUs (here: none)
    refuses before starting any rank, with a message and no JSON line."""
    import subprocess

    env = dict(os.environ)
    for k in ("BENCH_REHEARSE", "RANK", "LOCAL_RANK", "WORLD_SIZE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 2 and "needs 2 visible GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
