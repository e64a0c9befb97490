#!/usr/bin/env python3
"""Timing-order probe: the stage1 B=32 vocoder step timed in several
back-to-back loops (no events, events every step, every 8th step) to separate
event cost from clock / warm-up drift.  python tools/probe/timing_order.py"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
model = bench.fixture_model(bench.STAGE1, dev)
mel = torch.randn(32, 64, 500, device=dev)
h = model._hip(dev).handle


def loop(n, stride=0):
    if stride:
        lib.m2_profile_select(h, 1 << 2)
        lib.m2_profile_stride(h, stride)
        lib.m2_profile_enable(h, (n + stride - 1) // stride)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        model.vocoder(mel)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / n * 1e6
    if stride:
        lib.m2_profile_disable(h)
        lib.m2_profile_stride(h, 1)
    return el


for _ in range(20):
    model.vocoder(mel)
for name, st in [("none", 0), ("every", 1), ("stride8", 8), ("none", 0), ("stride8", 8), ("every", 1), ("none", 0)]:
    print(f"{name:8s} {loop(400, st):7.2f} us/step", flush=True)
