"""bench.py's multi-GPU launch path on CPU: ``--gpus N`` without WORLD_SIZE
starts N fresh rank processes (spawn) that see world_size N and rendezvous on
127.0.0.1; under torch.distributed.run the ranks come from the environment.
``--dry-run`` swaps the GPU work for a gloo all-reduce."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(cmd, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_bench_gpus_flag_spawns_ranks(n):
    out = _run([sys.executable, "bench.py", "--gpus", str(n), "--dry-run"])
    assert out["n_gpus"] == n and out["rank_sum"] == n * (n + 1) / 2


def test_bench_under_torchrun():
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--dry-run"])
    assert out["n_gpus"] == 2 and out["rank_sum"] == 3


def _settle_worker(rank, world, port, outfile):
    """Ctx.settle around a collective with the ranks entering it 30 ms apart:
    they must run the same number of iterations (a rank leaving the loop alone
    would leave the other waiting in its all_reduce)."""
    import time

    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(ROOT))
    import bench
    torch.cuda.synchronize = lambda *a, **k: None  # CPU: nothing to wait for
    cx = bench.Ctx.__new__(bench.Ctx)
    cx.dev, cx.world, cx.rank, cx.dist, cx.backend = torch.device("cpu"), world, rank, True, "gloo"
    n = [0]

    def fn():
        t = torch.ones(1)
        dist.all_reduce(t)
        n[0] += 1

    time.sleep(0.03 * rank)
    for ms in (5.0, 20.0, 50.0):
        cx.settle(fn, ms)
    t = torch.tensor([float(n[0])])
    lo, hi = t.clone(), t.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if rank == 0:
        with open(outfile, "w") as f:
            json.dump({"min": lo.item(), "max": hi.item()}, f)
    dist.destroy_process_group()


def test_settle_keeps_ranks_in_step(tmp_path):
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "settle.json"
    mp.spawn(_settle_worker, args=(2, port, str(out)), nprocs=2, join=True)
    r = json.loads(out.read_text())
    assert r["min"] == r["max"] > 0
