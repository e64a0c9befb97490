#!/usr/bin/env python3
"""The stage2 mel decoder alone on random rows (fixed B x T, no duration
predictor: a diagnostic build's garbage cannot change the frame count), for
per-kernel timing under rocprofv3 --kernel-trace --stats:
    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/probe/dec_time.py 128 2600 [iters]
Prints the mean ms per decoder call (events around the loop)."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))


def main():
    import bench
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 2600
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda", 0)
    m = bench.fixture_model(bench.STAGE2, dev)
    x = torch.randn(B, T, bench.STAGE2["hidden_dim"], generator=torch.Generator().manual_seed(3)).to(dev)
    with torch.no_grad():
        for _ in range(3):
            m.decoder(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()  # (the handle may launch on its own stream: host clock around syncs)
        for _ in range(iters):
            m.decoder(x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"decoder B={B} T={T}: {dt * 1e3 / iters:.3f} ms per call")


if __name__ == "__main__":
    main()
