#!/usr/bin/env python3
"""CPU simulation of the split-f16 (3xf16) vocoder arithmetic vs fp64 / fp32 / plain f16.

Every conv / convT of the oracle vocoder is replaced by its emulated form on the golden
stage1/stage2 weights; prints waveform RMS / max error vs an fp64 evaluation.
Test infrastructure (uses the oracle), not part of the product path.
    python tools/probe/split_sim.py
"""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'oracle'))
import m2tts_oracle as O  # noqa: E402

G = Path(__file__).resolve().parents[2] / 'tests' / 'golden'
for stage, cfg in (('s1', O.STAGE1), ('s2', O.STAGE2)):
    w = np.load(G / f'weights_{stage}.npz')
    sd = {k: torch.from_numpy(w[k]) for k in w.files}
    torch.manual_seed(0)
    B, T = 2, 120
    mel = torch.randn(B, cfg.mel_channels, T)
    def run(mode):
        conv1d0, convt0 = F.conv1d, F.conv_transpose1d
        def split16(x, lo_scale=2.0**11):
            h = x.half().float(); l = ((x - h) * lo_scale).half().float(); return h, l
        def splitbf(x):
            h = x.bfloat16().float(); l = (x - h).bfloat16().float(); return h, l
        def wrap(fn):
            def f(x, wt, b=None, *a, **k):
                if mode == 'f64':
                    return fn(x.double(), wt.double(), None if b is None else b.double(), *a, **k).float()
                if mode == 'f32':
                    return fn(x, wt, b, *a, **k)
                if mode == 'f16x3':
                    xh, xl = split16(x); wh, wl = split16(wt)
                    y = fn(xh, wh, None, *a, **k) + (fn(xh, wl, None, *a, **k) + fn(xl, wh, None, *a, **k)) / 2.0**11
                elif mode == 'f16x3u':  # the kernels' format: lo = f16(x - hi), unscaled (may be subnormal)
                    xh, xl = split16(x, 1.0); wh, wl = split16(wt, 1.0)
                    y = fn(xh, wh, None, *a, **k) + (fn(xh, wl, None, *a, **k) + fn(xl, wh, None, *a, **k))
                elif mode == 'bf16x3':
                    xh, xl = splitbf(x); wh, wl = splitbf(wt)
                    y = fn(xh, wh, None, *a, **k) + fn(xh, wl, None, *a, **k) + fn(xl, wh, None, *a, **k)
                elif mode == 'f16':
                    y = fn(x.half().float(), wt.half().float(), None, *a, **k)
                return y if b is None else y + b[None, :, None]
            return f
        F.conv1d, F.conv_transpose1d = wrap(conv1d0), wrap(convt0)
        try:
            return O.vocoder(sd, mel)
        finally:
            F.conv1d, F.conv_transpose1d = conv1d0, convt0
    ref = run('f64')
    rms = lambda a: float(torch.sqrt(torch.mean(a.double() ** 2)))
    print(stage, 'audio rms', rms(ref))
    for mode in ('f32', 'f16x3', 'f16x3u', 'bf16x3', 'f16'):
        y = run(mode)
        print(f'  {mode:7s} rms err {rms(y - ref):.3e}  max {float((y - ref).abs().max()):.3e}')
