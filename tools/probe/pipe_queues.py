#!/usr/bin/env python3
"""Does ShardedPipeline's speed depend on which hardware queues its two
streams land on?  HIP maps streams onto GPU_MAX_HW_QUEUES (4 on the box)
hardware queues round robin, so two streams can share one in-order queue.
Runs the depth-2 pipeline at stage2 B=8 S=100 and B=64 S=100 after creating
k = 0..4 unused streams first (rotating the assignment), with torch streams
and with full-CU-mask streams (hipExtStreamCreateWithCUMask: a queue of their
own), each in a fresh ShardedPipeline.
    python3 tools/probe/pipe_queues.py
"""
import ctypes
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
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    batches = {}
    for B in (8, 64):
        batches[B] = (torch.randint(0, 42, (B, 100), generator=g).to(dev),
                      torch.full((B,), 100, dtype=torch.long, device=dev))

    def prio_stream(prio):  # raw stream in the hardware-queue pool of that priority
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, prio) == 0
        return torch.cuda.ExternalStream(s.value)

    def ext_stream():
        words = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
        s = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), words) == 0
        return torch.cuda.ExternalStream(s.value)

    def run(pipe, ids, lens, n):
        prev = None
        for _ in range(n):
            r = pipe.submit(ids, lens)
            if prev is not None:
                prev.wait()
            prev = r
        prev.wait()

    keep = []
    KINDS = [a for a in sys.argv[1:] if not a.startswith("-")] or ["torch", "lo/hi", "hi/lo"]
    for k in range(5):
        for kind in KINDS:
            out = []
            for B, (ids, lens) in batches.items():
                pipe = ShardedPipeline(m, depth=2, gather_to=0, host_wait=(kind == "hostwait"))
                if kind in ("lo/hi", "hi/lo"):
                    pf, pb = (1, -1) if kind == "lo/hi" else (-1, 1)
                    pipe.front_stream = prio_stream(pf)
                    pipe._fs_h = pipe.front_stream.cuda_stream
                    pipe.back_stream = prio_stream(pb)
                    pipe._bs_h = pipe.back_stream.cuda_stream
                if kind == "ext":
                    pipe.front_stream = ext_stream()
                    pipe._fs_h = pipe.front_stream.cuda_stream
                    pipe.back_stream = ext_stream()
                    pipe._bs_h = pipe.back_stream.cuda_stream
                run(pipe, ids, lens, 20)
                torch.cuda.synchronize()
                steps = 200 if B == 8 else 60
                t0 = time.perf_counter()
                run(pipe, ids, lens, steps)
                torch.cuda.synchronize()
                out.append(f"B={B} {(time.perf_counter() - t0) / steps * 1e3:.4f}")
            print(f"extra streams {k}, {kind}: " + ", ".join(out) + " ms/step", flush=True)
        keep.append(torch.cuda.Stream())  # one more stream: rotates the next pipeline's queue assignment
        torch.zeros(1, device=dev).add_(1)  # touch it? (streams get a queue on first use)
        with torch.cuda.stream(keep[-1]):
            torch.zeros(1, device=dev).add_(1)


if __name__ == "__main__":
    main()
