#!/usr/bin/env python3
"""Phase stamps of the one-launch transformer layer (tfl::layer_kernel) from the
-DTFL_STAMPS diagnostic build (never the product):
  make -C m2-tts_amd/csrc OBJDIR=build_tst EXTRA=-DTFL_STAMPS OUT=build_tst/libm2tts_hip_tst.so
  M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so python tools/probe/tfl_stamps.py s2 8x500
Runs the mel decoder (unmasked layers) or, with 'enc', the text encoder on
random rows; the stamps of the LAST layer launch remain (NEXT = 2 / 0 layers
stamp slots 0-5 only)."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))
from m2amd import _lib  # noqa: E402

NAMES = ["attention loop", "merge", "out-proj", "LN2", "FFN1", "FFN2", "LN1'", "QKV'"]


def main():
    import bench
    stage = sys.argv[1] if len(sys.argv) > 1 else "s2"
    shapes = sys.argv[2:] or ["8x500"]
    lib = _lib.load()
    fn = lib.m2_debug_stamps_tfl
    fn.restype = ctypes.c_int32
    dev = torch.device("cuda", 0)
    m = bench.fixture_model(bench.STAGE1 if stage == "s1" else bench.STAGE2, dev)
    hm = m._hip(dev)
    H = hm.H
    for sh in shapes:
        enc = sh.startswith("enc")
        B, N = (int(v) for v in sh.replace("enc", "").split("x"))
        # stamp the FIRST layer of the decoder (NEXT = 1): a one-layer run would be
        # NEXT = 2; use the whole stack and keep what the last launch left
        x = torch.randn(B, N, H, device=dev)
        ids = torch.randint(0, 42, (B, N), device=dev)
        lens = torch.full((B,), N, device=dev, dtype=torch.long)
        for _ in range(30):
            if enc:
                hm.text_encoder(ids, lens)
            else:
                hm.decoder(x)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 8 * 16, dtype=np.uint64)
        fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
        st = buf.reshape(4096, 8, 16).astype(np.int64)
        used = st[:, 0, 0] != 0
        st = st[used]
        rt0, rt1 = st[:, 0, 14], st[:, 0, 15]
        ok_rt = rt1 != 0
        print(f"{stage} {sh}: WGs={st.shape[0]}; realtime: last start {(rt0.max() - rt0.min()) * 10} ns, "
              f"median WG duration {np.median((rt1 - rt0)[ok_rt]) * 10 if ok_rt.any() else -1:.0f} ns, "
              f"last end {(rt1[ok_rt].max() - rt0.min()) * 10 if ok_rt.any() else -1} ns")
        prev = st[:, :, 0]
        for i in range(1, 9):
            cur = st[:, :, i]
            ok = (cur != 0).all(axis=1)
            if ok.sum() == 0:
                continue
            d = (cur[ok] - prev[ok]).max(axis=1)
            print(f"   {NAMES[i - 1]:16s} {np.median(d):8.0f} cycles  (p90 {np.percentile(d, 90):8.0f}, WGs {ok.sum()})")
            prev = np.where(cur != 0, cur, prev)
        s0, s1, s2 = st[:, :, 0], st[:, :, 1], st[:, :, 2]
        ok = (s1 != 0).all(axis=1) & (s2 != 0).all(axis=1)
        if ok.any():
            spread = s1[ok].max(axis=1) - s1[ok].min(axis=1)
            after = s2[ok].max(axis=1) - s1[ok].max(axis=1)
            att = s1[ok] - s0[ok]
            print(f"   attention-end spread over waves {np.median(spread):8.0f} cycles; merge after the last wave "
                  f"{np.median(after):8.0f}; per-wave attention min/median/max {np.median(att.min(axis=1)):.0f} / "
                  f"{np.median(np.median(att, axis=1)):.0f} / {np.median(att.max(axis=1)):.0f}")
            print("   attention loop by wave index (median): " + " ".join(f"{np.median(att[:, w]):.0f}" for w in range(8)))
        last = max(i for i in range(1, 9) if (st[:, :, i] != 0).all(axis=1).any())
        tot = (st[:, :, last] - st[:, :, 0]).max(axis=1)
        print(f"   total            {np.median(tot):8.0f} cycles")
        buf[:] = 0
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
