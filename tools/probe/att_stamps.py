#!/usr/bin/env python3
"""Phase stamps of attention_split_kernel from the -DATT_STAMPS diagnostic build
(never the product):
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_ast/libm2tts_hip_ast.so python tools/probe/att_stamps.py 32x500x64"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
from m2amd import _lib, ops  # noqa: E402

NAMES = ["prologue(Q,fetch)", "stash0+bar"] + [f"pair{p}" for p in range(9)] + ["merge+bar", "out"]
lib = _lib.load()
fn = lib.m2_debug_stamps_att
fn.restype = ctypes.c_int32
dev = torch.device("cuda", 0)
for sh in (sys.argv[1:] or ["32x500x64"]):
    B, N, H = (int(v) for v in sh.split("x"))
    qkv = torch.randn(B, N, 3 * H, device=dev)
    for _ in range(20):
        ops.attention_core(qkv, 2, None)
    torch.cuda.synchronize()
    buf = np.zeros(2048 * 8 * 16, dtype=np.uint64)
    fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    st = buf.reshape(2048, 8, 16).astype(np.int64)
    used = st[:, 0, 0] != 0
    st = st[used]
    nwg = st.shape[0]
    rt0 = st[:, 0, 14]
    rt1 = st[:, 0, 15]
    print(f"{sh}: WGs={nwg}; realtime (10 ns): first start {0}, last start {(rt0.max() - rt0.min()) * 10} ns, "
          f"last end {(rt1.max() - rt0.min()) * 10} ns, median WG duration {np.median(rt1 - rt0) * 10:.0f} ns")
    # phase durations (shader clock cycles), median over WGs of the max over waves
    cols = [0, 1, 2] + [3 + p for p in range(9)] + [12, 13]
    prev = st[:, :, 0]
    for i, c in enumerate(cols[1:]):
        cur = st[:, :, c]
        ok = (cur != 0).all(axis=1)
        if ok.sum() == 0:
            continue
        d = (cur[ok] - prev[ok])
        dd = d.max(axis=1) if c != 13 else d[:, :4].max(axis=1)
        print(f"   {NAMES[i]:18s} {np.median(dd):8.0f} cycles (WGs {ok.sum()})")
        prev = np.where(cur != 0, cur, prev)
    tot = st[:, :4, 13] - st[:, :4, 0]
    print(f"   total (kh0 waves)  {np.median(tot.max(axis=1)):8.0f} cycles")
