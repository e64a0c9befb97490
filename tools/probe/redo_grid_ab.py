"""A/B of the range policy's per-call cost (bench.py vocoder headline shape,
stage1 B=32 T=500): the "report" policy against "fallback" with the guarded
redo launch at several grid sizes (M2_REDO_GRID), alternated in one process."""
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
m = bench.fixture_model(bench.STAGE1, dev)
mel = torch.randn(32, 64, 500, generator=torch.Generator().manual_seed(0)).to(dev)
variants = [("report", None), ("fallback", "-1"), ("fallback", "8"), ("fallback", "64"), ("fallback", "0")]
res = {f"{p}:{g}": [] for p, g in variants}
for _ in range(200):
    m.vocoder(mel)
torch.cuda.synchronize()
for rnd in range(5):
    for pol, g in variants:
        if g is None:
            os.environ.pop("M2_REDO_GRID", None)
        else:
            os.environ["M2_REDO_GRID"] = g
        _lib.reload_switches()
        m.set_range_policy(pol)
        for _ in range(20):
            m.vocoder(mel)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(300):
            m.vocoder(mel)
        torch.cuda.synchronize()
        res[f"{pol}:{g}"].append((time.perf_counter() - t0) / 300 * 1e3)
for k, v in res.items():
    v.sort()
    print(f"{k:14s} median {v[len(v) // 2]:.5f} ms  all {[round(x, 5) for x in v]}")
