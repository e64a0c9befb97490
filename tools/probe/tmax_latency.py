#!/usr/bin/env python3
"""Round-trip latency of the T_max read: frame_counts + .item() vs the
mailbox (frame_counts_sync), GPU idle and behind a queued vocoder pass.
    python tools/probe/tmax_latency.py
"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
model = bench.fixture_model(bench.STAGE1, dev)
d = (torch.rand(32, 100) * 10).to(dev)
mel = torch.randn(32, 64, 500, device=dev)


def old():
    _, _, tmax = ops.frame_counts(d, 1.0)
    return int(tmax.item())


def new():
    return ops.frame_counts_sync(d, 1.0)[3]


for name, f in (("item", old), ("mailbox", new)):
    for behind in (False, True):
        ts = []
        for i in range(400):
            if behind:
                model.vocoder(mel)
            torch.cuda.synchronize() if not behind else None
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e6)
        ts = sorted(ts[100:])
        print(f"{name:8s} behind_vocoder={behind}: median {ts[len(ts) // 2]:7.1f} us  p10 {ts[len(ts) // 10]:7.1f}")
