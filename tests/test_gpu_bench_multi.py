"""GPU: the N > 1 bench path (BASELINE configs[3]: independent channels, one process per GPU, no
data-path collective) run end to end as a fresh `torch.distributed.run` job with two ranks.

On a one-GPU box the ranks share cuda:0 and talk over gloo (BENCH_REHEARSE=1, bench.py); the
driver's 8-GPU run uses RCCL with one rank per GPU. The line must carry n_gpus = 2, the weak-scaling
aggregate (both ranks' samples over the slowest rank's time) and the config-4 FM record. This is a
rehearsal of the code path, not a scaling measurement."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("launcher", ["torchrun", "plain"])
def test_bench_two_ranks_rehearsal(cuda, launcher):
    """launcher = torchrun: the driver's form; plain: `python bench.py --gpus 2`, which starts its own rank
    processes (bench.self_launch) and must produce the same validated line."""
    env = dict(os.environ, BENCH_REHEARSE="1", MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        env.pop(k, None)
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2", "--settle-max", "50",
            "--no-cpu-baseline"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 5 and line["scaling"] == "weak"
    assert line["config"]["channels"] == 2 and "rehearsal" in line
    # value = both ranks' input samples over the slowest rank's wall time
    per_step_s = line["ms_per_step"] * 1e-3
    want = 2 * line["config"]["input_samples"] / per_step_s / 1e6
    assert abs(line["value"] - want) <= 0.01 * want
    fm = line["secondary"]["fm_chain_multi_gpu"]
    assert fm["n_gpus"] == 2 and fm["us_per_launch_max_over_ranks"] > 0
    assert fm["aggregate_msamples_per_s"] > 0
    # each rank checked its own channel's output against the float64 restatement, outside the timed region
    assert fm["parity_ok"] == [True, True], fm
    assert all(e <= 1e-5 for e in fm["parity_max_wrapped_err_over_pi_g"])
    assert len(fm["output_digest"]) == 2 and fm["output_digest"][0] != fm["output_digest"][1]  # independent channels
    # the line validates itself: per-rank device identity, backend, world size, per-rank times, in-job N = 1 figure
    ranks = line["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert all(r["backend"] == "gloo" and r["world_size"] == 2 for r in ranks)
    assert all(r["fir_kernel_us"] > 0 and r["wall_ms"] > 0 for r in ranks)
    # rehearsal: both ranks on cuda:0, so the identities coincide -- accepted only because of the flag
    assert ranks[0]["pci"] == ranks[1]["pci"] and ranks[0]["uuid"] == ranks[1]["uuid"]
    chk = line["multi_gpu_check"]
    assert chk["backend"] == "gloo" and chk["world_size"] == 2 and chk["distinct_devices"] is False
    assert chk["solo_fir_kernel_us_rank0"] > 0 and 0 < chk["fir_scaling_efficiency"] < 10
    assert max(r["fir_kernel_us"] for r in ranks) == pytest.approx(line["roofline"]["kernel_us_max_over_ranks"], rel=1e-3)
    assert len(fm["us_per_launch_per_rank"]) == 2 and all(v > 0 for v in fm["us_per_launch_per_rank"])
    assert max(fm["us_per_launch_per_rank"]) == pytest.approx(fm["us_per_launch_max_over_ranks"], rel=1e-3)
    assert fm["solo_us_per_launch_rank0"] > 0
    assert fm["scaling_efficiency"] == pytest.approx(fm["solo_us_per_launch_rank0"] / fm["us_per_launch_max_over_ranks"],
                                                     rel=1e-2)

