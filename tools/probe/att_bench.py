"""Attention microbenchmark: m2_attention (the split-f16 flash kernel the
transformer layers use) on decoder-shaped qkv, timed with HIP events over
many launches; reports us per launch and algorithmic TF/s (4*hd*N^2 FLOP per
(utterance, head)) vs the split peak 838.9.

    python tools/probe/att_bench.py [--iters 200]
"""
import argparse, json, sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
from m2amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--shapes", default="32x500x64,64x500x96,8x500x96,16x2600x96,128x2600x96")
args = ap.parse_args()
dev = torch.device("cuda", 0)
res = {}
for sh in args.shapes.split(","):
    B, N, H = (int(v) for v in sh.split("x"))
    qkv = torch.randn(B, N, 3 * H, device=dev)
    for _ in range(5):
        ops.attention_core(qkv, 2, None)
    torch.cuda.synchronize()
    it = max(5, args.iters if N <= 600 else args.iters // 10)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        ops.attention_core(qkv, 2, None)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    flop = 4.0 * (H // 2) * N * N * B * 2
    res[sh] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1), "frac": round(flop / us / 1e6 / 838.9, 3)}
print(json.dumps(res))
