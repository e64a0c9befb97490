#!/usr/bin/env python3
"""Feasibility probe for CU-partitioned lanes: configs[3]'s
per-GPU share (stage2, B=8, S=100) with the front half (encoder, durations)
and the back half (decoder, vocoder) on streams restricted to disjoint CU
sets (hipExtStreamCreateWithCUMask), so step i+1's front runs beside step i's
back.  Prints ms/step for:
  base      front_dev + back_dev on one stream, one step at a time
  iso F/B   each half alone on its masked stream (what a CU set costs it)
  pipe      front stream (mask F) || back stream (mask B), two handles
              alternating, event dependencies only
    python3 tools/probe/cumask_share.py [n_front_cus ...]
"""
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent


def masked_stream(bits, ncu):
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def main():
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    B, S, T = 8, 100, 500
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    hms = [m._hip(dev, lane) for lane in (1, 2)]
    outs = [(torch.empty(B * T * 80, device=dev), torch.empty(B * 64 * T, device=dev)) for _ in hms]
    tws = [torch.empty(1, dtype=torch.int32, device=dev) for _ in hms]
    # learn the capacity the way the sharded flow does
    with torch.no_grad():
        for hm in hms:
            st, t = hm.inference_front(ids, lens, 1.0)
            assert t == T
            hm.inference_back(st, t)
    torch.cuda.synchronize()
    ref_mel = None

    def one(hm, tw, out, fs=None, bs=None, ev=None):
        cur = torch.cuda.current_stream()
        with torch.cuda.stream(fs or cur):
            st = hm.inference_front_dev(ids, lens, 1.0, tw)
        if fs is not None:
            e = torch.cuda.Event()
            e.record(fs)
            (bs or cur).wait_event(e)
        with torch.cuda.stream(bs or cur):
            hm.inference_back_dev(st, T, tw, out[0], out[1])
        return st

    def timeit(fn, steps=200, warm=30):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    with torch.no_grad():
        base = timeit(lambda: one(hms[0], tws[0], outs[0]))
        ref_mel = outs[0][0].clone()
        ref_aud = outs[0][1].clone()
        print(f"base (one stream, one step at a time): {base:.4f} ms/step", flush=True)
        full = masked_stream(range(ncu), ncu)
        with torch.cuda.stream(full):
            print(f"base on a full-mask ext stream: {timeit(lambda: one(hms[0], tws[0], outs[0])):.4f} ms/step",
                  flush=True)
        nfs = [int(a) for a in sys.argv[1:]] or [32, 48, 64]
        for layout in ("low", "strided"):
            for nf in nfs:
                if layout == "low":
                    fb = list(range(nf))
                else:
                    step = ncu // nf
                    fb = list(range(0, step * nf, step))
                bb = [c for c in range(ncu) if c not in set(fb)]
                fs, bs = masked_stream(fb, ncu), masked_stream(bb, ncu)
                # each half alone on its CU set
                st0 = hms[0].inference_front_dev(ids, lens, 1.0, tws[0])
                torch.cuda.synchronize()
                with torch.cuda.stream(fs):
                    tf = timeit(lambda: hms[1].inference_front_dev(ids, lens, 1.0, tws[1]))
                with torch.cuda.stream(bs):
                    tb = timeit(lambda: hms[0].inference_back_dev(st0, T, tws[0], outs[0][0], outs[0][1]))
                torch.cuda.synchronize()
                # pipelined: step i on handle i % 2; front(i) waits back(i - 2) (same handle)
                back_done = [None, None]
                k = [0]

                def pipe_step():
                    h = k[0] % 2
                    k[0] += 1
                    if back_done[h] is not None:
                        fs.wait_event(back_done[h])
                    with torch.cuda.stream(fs):
                        st = hms[h].inference_front_dev(ids, lens, 1.0, tws[h])
                    e = torch.cuda.Event()
                    e.record(fs)
                    bs.wait_event(e)
                    with torch.cuda.stream(bs):
                        hms[h].inference_back_dev(st, T, tws[h], outs[h][0], outs[h][1])
                    d = torch.cuda.Event()
                    d.record(bs)
                    back_done[h] = d

                tp = timeit(pipe_step)
                ok = all(torch.equal(outs[h][0], ref_mel) and torch.equal(outs[h][1], ref_aud) for h in (0, 1))
                print(f"{layout:7s} F={nf:3d} B={len(bb):3d}: front alone {tf:.4f}  back alone {tb:.4f}  "
                      f"pipelined {tp:.4f} ms/step  bit-equal {ok}", flush=True)
        # the same pipelined schedule with both streams unmasked (what ShardedPipeline does today)
        fs, bs = torch.cuda.Stream(), torch.cuda.Stream()
        back_done = [None, None]
        k = [0]

        def pipe_plain():
            h = k[0] % 2
            k[0] += 1
            if back_done[h] is not None:
                fs.wait_event(back_done[h])
            with torch.cuda.stream(fs):
                st = hms[h].inference_front_dev(ids, lens, 1.0, tws[h])
            e = torch.cuda.Event()
            e.record(fs)
            bs.wait_event(e)
            with torch.cuda.stream(bs):
                hms[h].inference_back_dev(st, T, tws[h], outs[h][0], outs[h][1])
            d = torch.cuda.Event()
            d.record(bs)
            back_done[h] = d

        print(f"unmasked split streams pipelined: {timeit(pipe_plain):.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
