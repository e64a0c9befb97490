#!/usr/bin/env python3
"""In-process A/B of a per-call environment switch on stage2 / stage1
inference: alternates the values of VAR every `steps` steps for `rounds`
rounds in ONE process (no process-order or box effects), timing each block
with events on the launch stream; prints the median ms/step per value.
    python tools/probe/env_ab.py VAR v1,v2 stage B S [rounds] [steps]"""
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
    var, vals, stage, B, S = sys.argv[1], sys.argv[2].split(","), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 8
    steps = int(sys.argv[7]) if len(sys.argv) > 7 else 30
    dev = torch.device("cuda", 0)
    m = bench.fixture_model(bench.STAGE1 if stage == "s1" else bench.STAGE2, dev)
    m.set_range_policy("report")
    g = torch.Generator().manual_seed(2024)
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    res = {v: [] for v in vals}
    with torch.no_grad():
        for _ in range(20):
            m.inference(ids, lens)
        for _ in range(rounds):
            for v in vals:
                if v == "unset":
                    os.environ.pop(var, None)
                else:
                    os.environ[var] = v
                _lib.reload_switches()  # the library reads the M2_* switches once, not per call
                m.inference(ids, lens)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(steps):
                    m.inference(ids, lens)
                e1.record()
                e1.synchronize()
                res[v].append(e0.elapsed_time(e1) / steps)
    for v in vals:
        x = sorted(res[v])
        print(f"{var}={v} {stage} B={B} S={S}: median {x[len(x) // 2]:.4f} ms/step  min {x[0]:.4f}  all {[round(t, 4) for t in res[v]]}")


if __name__ == "__main__":
    main()
