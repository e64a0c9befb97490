#!/usr/bin/env python3
"""The headline vocoder call (stage1, B=32, T=500) in a plain loop with no
profiling events, for a rocprofv3 --kernel-trace run (tools/runs/r05o.sh
summarises the time line); "f32": the exact-f32 kernels (the strict line):
    python3 tools/probe/voc_gaps.py [calls] [f32]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
m = bench.fixture_model(bench.STAGE1, dev)
if len(sys.argv) > 2 and sys.argv[2] == "f32":
    m._hip(dev).vocoder_select(1)
mel = torch.randn(32, 64, 500, device=dev)
for _ in range(n):
    m.vocoder(mel)
torch.cuda.synchronize()
