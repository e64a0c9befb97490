"""Key-split layer tiles against the unsplit ones (M2_TFL_SPLIT=0/1) on the
mel decoder: max |diff|, differing elements, and split run twice
(determinism).  python tools/probe/split_diff.py"""
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
    dev = torch.device("cuda", 0)
    for stage, B, T, rb in (("s1", 1, 500, "1"), ("s1", 1, 64, "1"), ("s2", 8, 500, "2"), ("s2", 1, 500, "1")):
        m = bench.fixture_model(bench.STAGE1 if stage == "s1" else bench.STAGE2, dev)
        H = (bench.STAGE1 if stage == "s1" else bench.STAGE2)["hidden_dim"]
        x = torch.randn(B, T, H, generator=torch.Generator().manual_seed(5)).to(dev)
        os.environ["M2_TFL_RB"] = rb
        out = {}
        for v in ("0", "1", "1b"):
            os.environ["M2_TFL_SPLIT"] = v[0]
            _lib.reload_switches()
            with torch.no_grad():
                out[v] = m.decoder(x).float()
            torch.cuda.synchronize()
        d = (out["0"] - out["1"]).abs()
        d2 = (out["1"] - out["1b"]).abs()
        print(f"{stage} B={B} T={T} rb={rb}: split vs unsplit max {d.max().item():.3g} n {(d > 0).sum().item()}"
              f" of {d.numel()}; split twice max {d2.max().item():.3g}", flush=True)


if __name__ == "__main__":
    main()
