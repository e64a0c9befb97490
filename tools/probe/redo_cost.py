#!/usr/bin/env python3
"""The default range policy's per-call cost at several guard-launch grids
(M2_REDO_GRID), timed exactly like bench.py's headline (same steps, the same
fence-free events on the dominant kernel every stride-th call), alternated
with the "report" policy in one process (stage1 B=32 T=500)."""
import os
import sys
import types
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cx = bench.Ctx(dev, 1, 0, False)
    args = types.SimpleNamespace(steps=200, warmup=20)
    head = bench.vocoder_line(cx, "s1", 32, 500, args, 100.0, 0)
    roof = head["roofline"]
    dom = [d["index"] for d in head["vocoder_kernels"] if d["kernel"] == roof["kernel"]][0]
    m = cx.model("s1")
    hm = m._hip(dev)
    mel = torch.randn(32, 64, 500, generator=torch.Generator().manual_seed(7)).to(dev)
    step = lambda: m.vocoder(mel)  # noqa: E731
    variants = [("fallback", None), ("fallback", "1"), ("fallback", "8"), ("report", None)]
    res = {f"{p}:{g}": [] for p, g in variants}
    for _ in range(3):
        for pol, g in variants:
            if g is None:
                os.environ.pop("M2_REDO_GRID", None)
            else:
                os.environ["M2_REDO_GRID"] = g
            _lib.reload_switches()
            m.set_range_policy(pol)
            cx.settle(step, 20.0)
            el, _ = cx.timed(step, args.steps, 3, hm, kernel_mask=1 << dom, stride=roof["event_stride"])
            res[f"{pol}:{g}"].append(el / args.steps * 1e3)
    m.set_range_policy("fallback")
    os.environ.pop("M2_REDO_GRID", None)
    _lib.reload_switches()
    med = {k: sorted(v)[1] for k, v in res.items()}
    for k, v in res.items():
        print(f"{k:14s} median {med[k]:.5f} ms  cost vs report {1e3 * (med[k] - med['report:None']):+.2f} us  "
              f"all {[round(x, 5) for x in v]}")


if __name__ == "__main__":
    main()
