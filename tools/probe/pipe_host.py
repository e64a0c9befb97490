#!/usr/bin/env python3
"""Host cost of ShardedPipeline's submit / wait at configs[3]'s per-GPU share
(stage2 B=8 S=100, world 1): ms/step over many steps at depths 1-3 and the
host time inside submit() and wait() per step.
    python3 tools/probe/pipe_host.py [steps]
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
    from m2amd.parallel import ShardedPipeline, hip_stages, sharded_inference
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    B, S = 8, 100
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    st = hip_stages(m)
    one = lambda: sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)  # noqa: E731
    for _ in range(30):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    print(f"depth 1 (sharded_inference): {(time.perf_counter() - t0) / steps * 1e3:.4f} ms/step", flush=True)
    for depth in (2, 3):
        pipe = ShardedPipeline(m, depth=depth, gather_to=0)
        pend = []
        ts, tw = [], []

        def step():
            a = time.perf_counter()
            pend.append(pipe.submit(ids, lens))
            b = time.perf_counter()
            if len(pend) > depth - 1:
                pend.pop(0).wait()
            c = time.perf_counter()
            ts.append(b - a)
            tw.append(c - b)

        for _ in range(30):
            step()
        torch.cuda.synchronize()
        ts.clear()
        tw.clear()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        med = lambda v: sorted(v)[len(v) // 2] * 1e3  # noqa: E731
        print(f"depth {depth}: {el:.4f} ms/step; host submit {med(ts):.4f} ms, wait {med(tw):.4f} ms (medians)",
              flush=True)
        while pend:
            pend.pop(0).wait()
        # the driver's form: 20 timed steps after 2 warm-up steps
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        print(f"depth {depth}, 20 steps: {(time.perf_counter() - t0) / 20 * 1e3:.4f} ms/step", flush=True)
        while pend:
            pend.pop(0).wait()




def profile_submit(steps=300):
    """cProfile of ShardedPipeline.submit + wait at depth 2 (host cost breakdown)."""
    import cProfile
    import pstats
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    from m2amd.parallel import ShardedPipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    ids = torch.randint(0, 42, (8, 100), generator=g).to(dev)
    lens = torch.full((8,), 100, dtype=torch.long, device=dev)
    pipe = ShardedPipeline(m, depth=2, gather_to=0)
    pend = []

    def run(n):
        for _ in range(n):
            pend.append(pipe.submit(ids, lens))
            if len(pend) > 1:
                pend.pop(0).wait()

    run(30)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    run(steps)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--profile":
        profile_submit()
    else:
        main()
