#!/usr/bin/env python3
"""Per-kernel fused-vocoder time vs batch size (workgroup-count / occupancy probe).

    python tools/scan_batch.py [--batches 4,8,...] [--frames 500]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="4,8,12,16,20,24,28,32,40,48,64")
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    model = bench.fixture_model(dev)
    hm = model._hip(dev)
    nk = lib.m2_profile_kernel_count()
    print("B, " + ", ".join(lib.m2_profile_kernel_name_for(hm.handle, i).decode().split()[0] for i in range(nk)) + ", total_ms")
    for B in [int(x) for x in a.batches.split(",")]:
        mel = torch.randn(B, 64, a.frames, device=dev)
        for _ in range(3):
            model.vocoder(mel)
        lib.m2_profile_enable(hm.handle, a.iters)
        for _ in range(a.iters):
            model.vocoder(mel)
        torch.cuda.synchronize()
        buf = (ctypes.c_float * (a.iters * nk))()
        n = ctypes.c_int32()
        lib.m2_profile_read(hm.handle, buf, a.iters * nk, ctypes.byref(n))
        ms = [sorted(buf[i::nk][: n.value // nk])[len(buf[i::nk][: n.value // nk]) // 2] for i in range(nk)]
        print(f"{B}, " + ", ".join(f"{m * 1e3:.1f}" for m in ms) + f", {sum(ms):.4f}", flush=True)


if __name__ == "__main__":
    main()
