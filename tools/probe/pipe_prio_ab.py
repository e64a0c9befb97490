#!/usr/bin/env python3
"""ShardedPipeline's back-stream priority, alternated in one process: depth-2
pipelines with the back stream at torch priority 0 and -1 (and the default) at stage2
B=8 S=100 (configs[3]'s per-GPU share) and B=64 S=100 (configs[3] at world
1), ms per step over 200 steps, three rounds.
    python3 tools/probe/pipe_prio_ab.py
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent


def main():
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    from m2amd.parallel import ShardedPipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    for B, steps in ((8, 200), (64, 60)):
        ids = torch.randint(0, 42, (B, 100), generator=g).to(dev)
        lens = torch.full((B,), 100, dtype=torch.long, device=dev)
        def make(prio):  # the pipeline with its back stream at that torch priority
            pipe = ShardedPipeline(m, depth=2, gather_to=0)
            if prio is not None:
                pipe.back_stream = torch.cuda.Stream(priority=prio)
                pipe._bs_h = pipe.back_stream.cuda_stream
            return pipe

        # (round 6 ran this against a constructor argument, None = -1 for
        # shards <= 2048 tokens; that argument is gone, None is now the default)
        pipes = {p: make(p) for p in (0, -1, None)}

        def run(pipe, n):
            prev = None
            for _ in range(n):
                r = pipe.submit(ids, lens)
                if prev is not None:
                    prev.wait()
                prev = r
            prev.wait()

        for p in pipes.values():
            run(p, 20)
        torch.cuda.synchronize()
        res = {p: [] for p in pipes}
        for _ in range(3):
            for p, pipe in pipes.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(pipe, steps)
                torch.cuda.synchronize()
                res[p].append((time.perf_counter() - t0) / steps * 1e3)
        for p, v in res.items():
            print(f"B={B} back_priority {p}: " + ", ".join(f"{x:.4f}" for x in v) + " ms/step", flush=True)


if __name__ == "__main__":
    main()
