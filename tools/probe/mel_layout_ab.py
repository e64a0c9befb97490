#!/usr/bin/env python3
"""Vocoder step time with the mel read in place from the decoder's [B,T,M]
output (inference path) vs the module's [B,M,T] input, alternated in one
process (stage1, B=32, T=500).
    python tools/probe/mel_layout_ab.py
"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
model = bench.fixture_model(bench.STAGE1, dev)
hm = model._hip(dev)
g = torch.Generator().manual_seed(0)
mel_btm = torch.randn(32, 500, 64, generator=g).to(dev)
mel_bmt = mel_btm.transpose(1, 2).contiguous()
res = {"[B,T,M]": [], "[B,M,T]": []}
for rep in range(8):
    for name, mel, btm in (("[B,T,M]", mel_btm, True), ("[B,M,T]", mel_bmt, False)):
        for _ in range(200):
            hm.vocoder(mel, layout_btm=btm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(1000):
            hm.vocoder(mel, layout_btm=btm)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 1000 * 1e6)
for k, v in res.items():
    print(f"{k}: " + " ".join(f"{x:.2f}" for x in v) + f"   min {min(v):.2f} us/step")
