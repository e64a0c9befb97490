#!/usr/bin/env python3
"""Front-half tilings for the pipelined B=8 share: with ShardedPipeline the
front half runs beside the previous step's back half, so its CU-time (not
its latency) is what the back half pays.  Alternates, in one process, the
default encoder / duration tiles with larger ones (M2_TFL_RB_MASKED = 2 / 4:
32- / 64-row encoder tiles; M2_DUR_RB = 2: 30-phoneme duration tiles) and
times the depth-2 pipeline and the one-step share (stage2 B=8 S=100).
    python3 tools/probe/front_tiles.py
"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent

VARIANTS = {"default": {}, "enc32": {"M2_TFL_RB_MASKED": "2"}, "enc64": {"M2_TFL_RB_MASKED": "4"},
            "dur30": {"M2_DUR_RB": "2"}, "enc64+dur30": {"M2_TFL_RB_MASKED": "4", "M2_DUR_RB": "2"},
            "enc32+dur30": {"M2_TFL_RB_MASKED": "2", "M2_DUR_RB": "2"}}
if "--dec" in sys.argv:  # the decoder's tiles instead (its K / V stream per workgroup is the same at any rows)
    VARIANTS = {"default": {}, "dec32": {"M2_TFL_RB_UNMASKED": "2"}, "dec64": {"M2_TFL_RB_UNMASKED": "4"}}
ENV_KEYS = ("M2_TFL_RB_MASKED", "M2_DUR_RB", "M2_TFL_RB_UNMASKED")


def main():
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    from m2amd import _lib
    from m2amd.parallel import ShardedPipeline, hip_stages, sharded_inference
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    ids = torch.randint(0, 42, (8, 100), generator=g).to(dev)
    lens = torch.full((8,), 100, dtype=torch.long, device=dev)
    st = hip_stages(m)
    pipe = ShardedPipeline(m, depth=2, gather_to=0)

    def run_pipe(n):
        prev = None
        for _ in range(n):
            r = pipe.submit(ids, lens)
            if prev is not None:
                prev.wait()
            prev = r
        return prev.wait()

    def run_one(n):
        for _ in range(n):
            out = sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)
        return out

    def timeit(fn, n):
        fn(10)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    res = {k: ([], []) for k in VARIANTS}
    ref = None
    rounds = 4 if "--dec" in sys.argv else 2
    for _ in range(rounds):
        for name, env in VARIANTS.items():
            for k in ENV_KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            _lib.reload_switches()
            res[name][0].append(timeit(run_pipe, 200))
            res[name][1].append(timeit(run_one, 200))
            mel, audio = run_pipe(1)
            if ref is None:
                ref = (mel.clone(), audio.clone())
            d = float((mel - ref[0]).abs().max())
            print(f"{name:12s} pipelined {res[name][0][-1]:.4f}  one step {res[name][1][-1]:.4f} ms/step  "
                  f"mel max-abs vs default {d:.2e}", flush=True)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    for name, (p, o) in res.items():
        print(f"median {name:12s} pipelined {med(p):.4f}  one step {med(o):.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
