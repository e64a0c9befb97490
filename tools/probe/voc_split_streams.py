#!/usr/bin/env python3
"""Headline vocoder (stage1, B=32, T=500): one m2_vocoder call of the whole
batch on one stream against the batch cut into P parts, each part's call on a
stream of its own (own workspace), all parts forked from and joined back to
the caller's stream.  Prints ms per batch for each form, alternated, and
whether the audio is bit-equal.   python3 tools/probe/voc_split_streams.py"""
import ctypes
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
B, M, T = 32, 64, 500
m = bench.fixture_model(bench.STAGE1, dev)
hm = m._hip(dev)
lib = _lib.load()
h = hm.handle
g = torch.Generator().manual_seed(7)
mel = torch.randn(B, M, T, generator=g).to(dev)
main = torch.cuda.current_stream(dev)


def make(parts):
    cuts = [B * i // parts for i in range(parts + 1)]
    sts = [torch.cuda.Stream(dev) for _ in range(parts)]
    ws = []
    for i in range(parts):
        b = cuts[i + 1] - cuts[i]
        n = int(lib.m2_workspace_bytes(h, b, 0, T))
        ws.append(torch.empty(max(n, 1 << 20), dtype=torch.uint8, device=dev))
    audio = torch.empty(B, 1, 64 * T, device=dev)

    def step():
        if parts == 1:
            _lib.check(lib.m2_vocoder(h, mel.data_ptr(), 0, B, T, audio.data_ptr(), ws[0].data_ptr(), ws[0].numel(),
                                      main.cuda_stream), "m2_vocoder")
            return
        for i, s in enumerate(sts):
            s.wait_stream(main)
            b0, b1 = cuts[i], cuts[i + 1]
            _lib.check(lib.m2_vocoder(h, mel[b0].data_ptr(), 0, b1 - b0, T, audio[b0].data_ptr(), ws[i].data_ptr(),
                                      ws[i].numel(), s.cuda_stream), "m2_vocoder")
        for s in sts:
            main.wait_stream(s)
    return step, audio


def timeit(step, n=200):
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


# range policy "report": concurrent calls on one handle share the redo words
lib.m2_set_range_policy(h, 0)
forms = {p: make(p) for p in (1, 2, 4)}
ref = None
for p, (step, audio) in forms.items():
    step()
    torch.cuda.synchronize()
    if ref is None:
        ref = audio.clone()
    print(f"parts {p}: bit-equal {torch.equal(audio, ref)}", flush=True)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    forms[1][0]()
torch.cuda.synchronize()
res = {p: [] for p in forms}
for rep in range(5):
    for p, (step, _) in forms.items():
        res[p].append(timeit(step))
for p, v in res.items():
    v = sorted(v)
    print(f"parts {p}: ms per batch median {v[len(v) // 2]:.5f}  all {[round(x, 5) for x in v]}", flush=True)
