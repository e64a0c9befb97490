#!/usr/bin/env python3
"""Run the stage2 mel decoder (one-launch layers) on random rows, for rocprofv3
PMC passes: python tools/probe/tfl_run.py [BxT] [reps]."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))


def main():
    import bench
    B, T = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "8x500").split("x"))
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    m = bench.fixture_model(bench.STAGE2, dev)
    hm = m._hip(dev)
    x = torch.randn(B, T, hm.H, device=dev)
    for _ in range(reps):
        hm.decoder(x)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
