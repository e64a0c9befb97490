#!/usr/bin/env python3
"""Host-side time of one pipeline step (M2TTSModel.inference, B=32 S=100),
split at the T_max read: enqueue before it, the wait inside it, enqueue after;
then the staged path against M2TTSModel.inference (two library calls).
    python tools/probe/host_phases.py
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
g = torch.Generator().manual_seed(0)
ids = torch.randint(0, 42, (32, 100), generator=g).to(dev)
lens = torch.full((32,), 100, dtype=torch.int64).to(dev)
ph = {"hip": [], "enc": [], "dur": [], "count": [], "item": [], "expand": [], "dec": [], "voc": [], "total": []}


def step():
    t0 = time.perf_counter()
    with torch.no_grad():
        hm = model._hip(dev)
        t1 = time.perf_counter()
        enc, _ = hm.text_encoder(ids, lens)
        t2 = time.perf_counter()
        dur = hm.duration(enc)
        t3 = time.perf_counter()
        cum, _, tmax = ops.frame_counts(dur, 1.0)
        t4 = time.perf_counter()
        T = max(1, int(tmax.item()))
        t5 = time.perf_counter()
        reg = ops.expand_frames(enc, cum, T)
        t6 = time.perf_counter()
        mel = hm.decoder(reg)
        t7 = time.perf_counter()
        hm.vocoder(mel, layout_btm=True)
        t8 = time.perf_counter()
    return [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t7 - t6, t8 - t7, t8 - t0]


for _ in range(300):
    step()
torch.cuda.synchronize()
for _ in range(300):
    for k, v in zip(ph, step()):
        ph[k].append(v * 1e6)
torch.cuda.synchronize()
for k, v in ph.items():
    v.sort()
    print(f"{k:7s} median {v[len(v) // 2]:7.1f} us")
t0 = time.perf_counter()
for _ in range(300):
    model.inference(ids, lens)
torch.cuda.synchronize()
print(f"inference() {(time.perf_counter() - t0) / 300 * 1e6:.1f} us/step")

# A/B in one process: six stage calls from Python (the staged path above) vs
# the two-call m2_inference_front / m2_inference_back path, alternated


def staged(ids, lens):
    with torch.no_grad():
        hm = model._hip(dev)
        enc, _ = hm.text_encoder(ids, lens)
        dur = hm.duration(enc)
        reg = ops.regulate(enc, dur, None)
        mel = hm.decoder(reg)
        return mel, hm.vocoder(mel, layout_btm=True)


res = {"staged": [], "front_back": []}
for rep in range(6):
    for name, fn in (("staged", staged), ("front_back", model.inference)):
        for _ in range(50):
            fn(ids, lens)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(300):
            fn(ids, lens)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 300 * 1e6)
for k, v in res.items():
    print(f"inference() via {k:10s}: " + " ".join(f"{x:.1f}" for x in v))
