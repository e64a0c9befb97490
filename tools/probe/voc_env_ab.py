#!/usr/bin/env python3
"""In-process A/B of an M2_* switch on one vocoder call shape: alternates the
values of VAR every `steps` calls for `rounds` rounds in ONE process, timing
each block with events on the launch stream, and checks that every value's
audio is bit-equal to the first value's.
    python tools/probe/voc_env_ab.py VAR v1,v2 path(1=exact-f32|2=split) stage B T [rounds] [steps]"""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))


def main():
    import bench
    from m2amd import _lib
    var, vals, path, stage = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3]), sys.argv[4]
    B, T = int(sys.argv[5]), int(sys.argv[6])
    rounds = int(sys.argv[7]) if len(sys.argv) > 7 else 8
    steps = int(sys.argv[8]) if len(sys.argv) > 8 else 50
    dev = torch.device("cuda", 0)
    cfg = bench.STAGE1 if stage == "s1" else bench.STAGE2
    m = bench.fixture_model(cfg, dev)
    m._hip(dev).vocoder_select(path)
    g = torch.Generator().manual_seed(11)
    mel = torch.randn(B, cfg["mel_channels"], T, generator=g).to(dev)
    res = {v: [] for v in vals}
    ref = None

    def setv(v):
        if v == "unset":
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        _lib.reload_switches()

    for v in vals:
        setv(v)
        a = m.vocoder(mel)
        torch.cuda.synchronize()
        if ref is None:
            ref = a.clone()
        print(f"{var}={v}: bit-equal to {vals[0]}: {torch.equal(a, ref)}  max-abs {(a - ref).abs().max().item():.3g}",
              flush=True)
    import time
    t_end = time.perf_counter() + 0.6  # clock settling (bench.py settle_ms)
    while time.perf_counter() < t_end:
        m.vocoder(mel)
        torch.cuda.synchronize()
    for _ in range(rounds):
        for v in vals:
            setv(v)
            m.vocoder(mel)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps):
                m.vocoder(mel)
            e1.record()
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) / steps)
    for v in vals:
        x = sorted(res[v])
        print(f"{var}={v} path {path} {stage} B={B} T={T}: median {x[len(x) // 2]:.5f} ms/call  min {x[0]:.5f}  "
              f"all {[round(t, 5) for t in res[v]]}", flush=True)


if __name__ == "__main__":
    main()
