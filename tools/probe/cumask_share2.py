#!/usr/bin/env python3
"""Second CU-partition probe (after r06b_cumask.txt): is the split-stream
pipeline of configs[3]'s per-GPU share (stage2 B=8 S=100) host-bound?  The
same schedule as cumask_share.py's "pipe" (front stream || back stream, two
handles alternating, front(i) waits back(i-2)), issued with raw ctypes calls
on raw stream / event handles (no torch stream contexts), and the host's
enqueue time per step measured separately (enqueue only, then drain).
    python3 tools/probe/cumask_share2.py
"""
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent

hip = ctypes.CDLL("libamdhip64.so")


def stream(mask_bits=None, ncu=256):
    s = ctypes.c_void_p()
    if mask_bits is None:
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0  # non-blocking
    else:
        words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
        for b in mask_bits:
            words[b // 32] |= 1 << (b % 32)
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words) == 0
    return s


def event():
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
    return e


def main():
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    import bench
    from m2amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    B, S, T = 8, 100, 500
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    hms = [m._hip(dev, lane) for lane in (1, 2)]
    with torch.no_grad():
        for hm in hms:
            st, t = hm.inference_front(ids, lens, 1.0)
            hm.inference_back(st, t)
    torch.cuda.synchronize()
    lanes = []
    for hm in hms:
        front = hm._scratch("_front", hm._size("m2_front_bytes", B, S))
        ws = hm._scratch("_ws", hm._size("m2_inference_workspace_bytes", B, S, T))
        mel = torch.empty(B * T * 80, device=dev)
        aud = torch.empty(B * 64 * T, device=dev)
        tw = torch.empty(1, dtype=torch.int32, device=dev)
        lanes.append((hm.handle, front, ws, mel, aud, tw))
    torch.cuda.synchronize()
    F, Bk = lib.m2_inference_front_dev, lib.m2_inference_back_dev

    def front_call(h, s):
        hd, front, ws, mel, aud, tw = lanes[h]
        rc = F(hd, ids.data_ptr(), lens.data_ptr(), B, S, ctypes.c_float(1.0), front.data_ptr(), front.numel(),
               ws.data_ptr(), ws.numel(), tw.data_ptr(), s)
        assert rc == 0, rc

    def back_call(h, s):
        hd, front, ws, mel, aud, tw = lanes[h]
        rc = Bk(hd, B, S, T, tw.data_ptr(), front.data_ptr(), front.numel(), mel.data_ptr(), aud.data_ptr(),
                ws.data_ptr(), ws.numel(), s)
        assert rc == 0, rc

    ev_front = [event(), event()]
    ev_back = [event(), event()]

    def run(fs, bs, steps, pipelined=True):
        """Returns (host enqueue ms/step, wall ms/step incl. drain)."""
        used = [False, False]
        t0 = time.perf_counter()
        for i in range(steps):
            h = i % 2
            if not pipelined:
                front_call(0, fs)
                back_call(0, fs)
                continue
            if used[h]:
                hip.hipStreamWaitEvent(fs, ev_back[h], 0)
            front_call(h, fs)
            hip.hipEventRecord(ev_front[h], fs)
            hip.hipStreamWaitEvent(bs, ev_front[h], 0)
            back_call(h, bs)
            hip.hipEventRecord(ev_back[h], bs)
            used[h] = True
        t1 = time.perf_counter()
        hip.hipDeviceSynchronize()
        t2 = time.perf_counter()
        return (t1 - t0) / steps * 1e3, (t2 - t0) / steps * 1e3

    def best(fs, bs, pipelined=True, steps=60, reps=5):
        run(fs, bs, 20, pipelined)
        res = [run(fs, bs, steps, pipelined) for _ in range(reps)]
        return min(r[1] for r in res), min(r[0] for r in res)

    def prio_stream(prio):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, prio) == 0
        return s

    lo_p, hi_p = ctypes.c_int(0), ctypes.c_int(0)
    hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo_p), ctypes.byref(hi_p))
    print(f"stream priority range: least {lo_p.value}, greatest {hi_p.value}", flush=True)
    if "--prio" in sys.argv:
        pf, pb = stream(), stream()
        for name, (a, c) in {"both default": (pf, pb),
                             "front low, back high": (prio_stream(lo_p.value), prio_stream(hi_p.value)),
                             "front high, back low": (prio_stream(hi_p.value), prio_stream(lo_p.value))}.items():
            rs = [best(a, c) for _ in range(3)]
            print(f"pipelined, {name}: " + ", ".join(f"{w:.4f}" for w, _ in rs) + " ms/step", flush=True)
        return
    plain_f, plain_b = stream(), stream()
    w, h = best(plain_f, plain_f, pipelined=False)
    print(f"serial, one raw stream: {w:.4f} ms/step (host enqueue {h:.4f})", flush=True)
    w, h = best(plain_f, plain_b)
    print(f"pipelined, two raw unmasked streams: {w:.4f} ms/step (host enqueue {h:.4f})", flush=True)
    # strided masks: every k-th CU id to the front
    for k in (8, 4):
        fb = list(range(0, ncu, k))
        bb = [c for c in range(ncu) if c % k]
        fs, bs = stream(fb, ncu), stream(bb, ncu)
        w1, _ = best(fs, fs, pipelined=False)
        w2, _ = best(bs, bs, pipelined=False)
        w, h = best(fs, bs)
        print(f"strided 1/{k}: F={len(fb)} B={len(bb)}: serial on F {w1:.4f}, serial on B {w2:.4f}, "
              f"pipelined {w:.4f} ms/step (host enqueue {h:.4f})", flush=True)
        wb = best(plain_f, bs)[0]
        print(f"   front unmasked || back on B: {wb:.4f}", flush=True)
    ref = lanes[0][3].clone(), lanes[0][4].clone()
    ok = all(torch.equal(lanes[i][3], ref[0]) and torch.equal(lanes[i][4], ref[1]) for i in (0, 1))
    print("lanes bit-equal:", ok)
    # which CU ids land where: front alone on single 32-id blocks (XCD mapping)
    for lo in (0, 32, 64, 96, 128, 160, 192, 224):
        fs = stream(list(range(lo, lo + 32)), ncu)
        w, _ = best(fs, fs, pipelined=False, steps=20, reps=2)
        print(f"serial on CU ids [{lo},{lo + 32}): {w:.4f}", flush=True)
    for k in (2, 8, 16):
        fs = stream(list(range(0, ncu, k)), ncu)
        w, _ = best(fs, fs, pipelined=False, steps=20, reps=2)
        print(f"serial on CU ids 0::{k} ({ncu // k}): {w:.4f}", flush=True)


if __name__ == "__main__":
    main()
