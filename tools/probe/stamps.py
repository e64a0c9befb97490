#!/usr/bin/env python3
"""Per-wave phase stamps from the M2_STAMPS diagnostic build (never the product).
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_stamps/libm2tts_hip_stamps.so python tools/probe/stamps.py B [--x3]
(--x3: the split-f16 kernels, whose phases are [layer, barrier] pairs)"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
import bench  # noqa: E402
from m2amd import _lib  # noqa: E402

PHASES = {
    0: ["gload", "bar", "inconv", "bar", "convT1", "bar", "rb1c1", "bar", "rb1c2", "bar", "gstore"],
    1: ["gload", "bar", "convT2", "bar", "rb2c1", "bar", "rb2c2", "bar", "gstore"],
    2: ["gload+bar", "convT3", "bar", "rb3c1", "bar", "rb3c2", "bar", "convT4", "bar", "rb4c1", "bar", "rb4c2", "bar",
        "outconv"],
}
X3 = {
    0: ["gload", "bar", "inconv", "bar", "convT1", "bar", "rb1c1", "bar", "rb1c2", "bar", "gstore"],
    1: ["gload", "bar", "convT2", "bar", "rb2c1", "bar", "rb2c2", "bar", "gstore"],
    2: ["gload", "bar", "convT3", "bar", "rb3c1", "bar", "rb3c2", "bar", "convT4", "bar", "rb4c1", "bar", "rb4c2",
        "bar", "outconv"],
}
x3 = "--x3" in sys.argv
s2 = "--s2" in sys.argv  # stage2 (C=256, M=80; random-init weights), T from --T=
argv = [a for a in sys.argv[1:] if a not in ("--x3", "--s2") and not a.startswith("--T=")]
T = int(next((a[4:] for a in sys.argv if a.startswith("--T=")), "500"))
if x3:
    PHASES = X3
B = int(argv[0]) if argv else 4
dev = torch.device("cuda", 0)
lib = _lib.load()
if s2:
    from models.tts_model import M2TTSModel
    sys.path.insert(0, str(ROOT / "oracle"))
    import m2tts_oracle as orc
    torch.manual_seed(0)
    model = M2TTSModel(**orc.STAGE2.as_dict()).to(dev).eval()
    mel = torch.randn(B, 80, T, device=dev)
else:
    model = bench.fixture_model(bench.STAGE1, dev)
    mel = torch.randn(B, 64, T, device=dev)
import os  # noqa: E402
for _ in range(int(os.environ.get("STAMPS_WARM", "3"))):  # STAMPS_WARM=2000: a settled clock
    model.vocoder(mel)
torch.cuda.synchronize()
buf = np.zeros(3 * 4096 * 16 * 16, dtype=np.uint64)
fn = lib.m2_debug_stamps_x3 if x3 else lib.m2_debug_stamps
fn.restype = ctypes.c_int32
fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
all_st = buf.reshape(3, 4096, 16, 16).astype(np.int64)
for k, names in PHASES.items():
    st = all_st[k]
    used = st[:, 0, 0] != 0
    st = st[used]
    if st.shape[0] == 0:  # a pipelined kernel (no x3 stamps)
        continue
    nph = len(names)
    nw = int((st[0, :, 0] != 0).sum())
    st = st[:, :nw, : nph + 1]
    d = np.diff(st, axis=2)
    tot = (st[:, :, nph] - st[:, :, 0]).max(axis=1)
    print(f"kernel {k}: WGs={st.shape[0]} waves={nw}; cycles: median over WGs of (max over waves | mean over waves)")
    for i, nm in enumerate(names):
        print(f"   {nm:10s} {np.median(d[:, :, i].max(axis=1)):8.0f} | {np.median(d[:, :, i].mean(axis=1)):8.0f}")
    print(f"   total      {np.median(tot):8.0f}")
if x3:  # head: shader clock per wave from s_memtime (slots 0, 9) over s_memrealtime (14, 15, 100 MHz)
    st = all_st[0]
    st = st[st[:, 0, 0] != 0]
    ok = (st[:, :, 15] > st[:, :, 14]) & (st[:, :, 9] > st[:, :, 0])
    ghz = (st[:, :, 9] - st[:, :, 0])[ok] / ((st[:, :, 15] - st[:, :, 14])[ok] / 100e6) / 1e9
    if ghz.size:
        print(f"head shader clock (GHz, per wave): median {np.median(ghz):.3f}  p10 {np.percentile(ghz, 10):.3f}  "
              f"p90 {np.percentile(ghz, 90):.3f}  over {ghz.size} waves")

