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
