#!/usr/bin/env python3
"""Global batches in flight per rank (ShardedPipeline depth) for one rank's
share of a sharded stage2 step, at world 1: ms per global batch for each
depth, alternated in rounds in ONE process (no box effects between depths).
    python tools/probe/depth_sweep.py B S depths [rounds] [steps]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))


def main():
    import bench
    from m2amd.parallel import ShardedPipeline, hip_stages, sharded_inference
    B, S = int(sys.argv[1]), int(sys.argv[2])
    depths = [int(d) for d in sys.argv[3].split(",")]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 40
    dev = torch.device("cuda", 0)
    m = bench.fixture_model(bench.STAGE2, dev)
    m.set_range_policy("report")
    g = torch.Generator().manual_seed(2024)
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    st = hip_stages(m)
    ref = sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)
    torch.cuda.synchronize()
    steps_fn = {}
    for d in depths:
        if d == 1:
            steps_fn[d] = lambda: sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)
            continue
        pipe = ShardedPipeline(m, depth=d, gather_to=0)
        q = []

        def step(pipe=pipe, q=q, d=d):
            q.append(pipe.submit(ids, lens))
            if len(q) >= d:
                return q.pop(0).wait()
            return None

        def drain(q=q):
            out = None
            while q:
                out = q.pop(0).wait()
            return out
        step.drain = drain
        steps_fn[d] = step
        mel, audio = pipe.submit(ids, lens).wait()
        assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1]), f"depth {d}: results differ"
    res = {d: [] for d in depths}
    with torch.no_grad():
        for d in depths:
            for _ in range(20):
                steps_fn[d]()
            getattr(steps_fn[d], "drain", lambda: None)()
        for _ in range(rounds):
            for d in depths:
                fn = steps_fn[d]
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(steps):
                    fn()
                getattr(fn, "drain", lambda: None)()
                e1.record()
                torch.cuda.synchronize()
                res[d].append(e0.elapsed_time(e1) / steps)
    for d in depths:
        x = sorted(res[d])
        print(f"depth {d} B={B} S={S}: median {x[len(x) // 2]:.4f} ms/global batch  min {x[0]:.4f}  "
              f"all {[round(t, 4) for t in res[d]]}", flush=True)


if __name__ == "__main__":
    main()
