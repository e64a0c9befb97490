#!/usr/bin/env python3
"""Kernel trace of ShardedPipeline at configs[3]'s per-GPU share (stage2
B=8 S=100, world 1, two lanes): do step i + 1's front-half kernels run beside
step i's back-half kernels?
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/probe/pipe_trace.py [depth]
    python3 tools/probe/pipe_trace.py --summarize DIR/run_kernel_trace.csv
The summary takes the last 40 steps: span per step, and for the front-half
kernels (encoder first launch and layers, duration) the fraction of their
time that overlaps a back-half kernel (decoder, vocoder).
"""
import csv
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent


def is_front(name):
    # encoder: first_kernel<96, 1 (SRC_EMBED), ...>, masked layer_kernel<96, true, ...>; the duration kernel
    return ("first_kernel<96, 1," in name or "layer_kernel<96, true" in name or "duration_kernel" in name
            or "lr_count" in name)


def summarize(path, steps=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in rows if "m2::" in r["Kernel_Name"]]
    starts = [i for i, (n, _, _) in enumerate(ks) if "first_kernel<96, 1," in n]
    starts = starts[-steps - 1:]
    a, b = starts[0], starts[-1]
    win = ks[a:b]
    front = [(s, e) for n, s, e in win if is_front(n)]
    back = [(s, e) for n, s, e in win if not is_front(n)]
    tot, ov = 0, 0
    for s, e in front:
        tot += e - s
        cover = 0
        for bs, be in back:
            lo, hi = max(s, bs), min(e, be)
            if hi > lo:
                cover += hi - lo
        ov += min(cover, e - s)
    span = (ks[b][1] - ks[a][1]) / 1e3 / (len(starts) - 1)
    busy_back = sum(e - s for s, e in back) / 1e3 / (len(starts) - 1)
    busy_front = tot / 1e3 / (len(starts) - 1)
    print(f"steps {len(starts) - 1}: span {span:.1f} us per step; back-half kernels {busy_back:.1f} us, "
          f"front-half kernels {busy_front:.1f} us per step; {100 * ov / max(tot, 1):.0f} % of the front-half "
          f"kernel time overlaps a back-half kernel")
    t0 = ks[a][1]
    print("one step (start, end relative to the step's first encoder launch, us):")
    nxt = starts[1]
    for n, s, e in ks[a:min(len(ks), nxt + 8)]:
        print(f"  {'F' if is_front(n) else 'B'} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  {n[:64]}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
        return
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
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    pipe = ShardedPipeline(m, depth=depth, gather_to=0)
    prev = None
    for _ in range(200):
        r = pipe.submit(ids, lens)
        if prev is not None:
            prev.wait()
        prev = r
    prev.wait()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
