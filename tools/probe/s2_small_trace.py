#!/usr/bin/env python3
"""stage2 inference at a small per-GPU batch (configs[3]'s share at N=8:
B=8, S=100), front + back per step, for a rocprofv3 --kernel-trace run
(the trace then shows each kernel's duration and the launch gaps):
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/probe/s2_small_trace.py
    python3 tools/probe/s2_small_trace.py --summarize DIR/run_kernel_trace.csv
"""
import csv
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent


def summarize(path, steps=20):
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else steps
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "")[:70] for r in rows]
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    # a step starts at the embedding kernel (first kernel of m2_inference_front;
    # with the fused first layer, ln_gemm_kernel<..., SRC_EMBED = 1>)
    # (one-launch layers: m2::tfl::first_kernel<H, SRC_EMBED = 1, ...>)
    starts = [i for i, n in enumerate(names) if "embed" in n or (n.startswith("m2::tfx::ln_gemm_kernel") and
                                                                   n.endswith(", 1>")) or
              (n.startswith("m2::tfl::first_kernel") and ", 1," in n)]
    starts = starts[-steps - 1:]
    per = {}
    spans, busy = [], []
    for a, b in zip(starts, starts[1:]):
        spans.append((st[b] - st[a]) / 1e3)
        busy.append(sum(en[i] - st[i] for i in range(a, b)) / 1e3)
        for i in range(a, b):
            gap = (st[i] - en[i - 1]) / 1e3 if i > a else 0.0
            per.setdefault((i - a, names[i]), []).append(((en[i] - st[i]) / 1e3, (st[i] - st[a]) / 1e3, gap))
    n = len(spans)
    print(f"steps {n}: span median {sorted(spans)[n // 2]:.1f} us, kernel-busy median {sorted(busy)[n // 2]:.1f} us")
    print("  #  duration  start@   gap-before (medians, us)")
    for (i, nm), v in sorted(per.items()):
        med = [sorted(c)[len(c) // 2] for c in zip(*v)]
        print(f"{i:3d} {med[0]:7.2f} {med[1]:8.1f} {med[2]:7.2f}  {nm}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
        return
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import os
    m = bench.fixture_model(bench.STAGE1 if os.environ.get("M2_TRACE_STAGE") == "s1" else bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    m.set_range_policy("report")
    hm = m._hip(dev)
    mode = sys.argv[2] if len(sys.argv) > 2 else "two"
    one = mode == "one"  # the one-call m2_inference (speculative back half)
    if mode == "dev":  # one rank's sharded flow on the device-T path
        from m2amd.parallel import hip_stages, sharded_inference
        st = hip_stages(m)
    with torch.no_grad():
        for _ in range(200 if S <= 100 else 30):
            if mode == "dev":
                sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)
            elif one:
                hm.inference(ids, lens, 1.0)
            else:
                state, tl = hm.inference_front(ids, lens, 1.0)
                hm.inference_back(state, max(1, tl))
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
