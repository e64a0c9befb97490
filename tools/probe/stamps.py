#!/usr/bin/env python3
"""Read per-wave phase stamps from the M2_STAMPS diagnostic build.
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_stamps/libm2tts_hip_stamps.so python tools/probe/stamps.py B"""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device("cuda", 0)
lib = _lib.load()
model = bench.fixture_model(dev)
mel = torch.randn(B, 64, 500, device=dev)
for _ in range(3):
    model.vocoder(mel)
torch.cuda.synchronize()
n = 3 * 4096 * 8 * 16
buf = np.zeros(n, dtype=np.uint64)
lib.m2_debug_stamps.restype = ctypes.c_int32
rc = lib.m2_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
st = buf.reshape(3, 4096, 8, 16)[0]
nwg = B * 18
st = st[:nwg].astype(np.int64)
names = ["gload", "bar", "inconv", "bar", "convT1", "bar", "rb1c1", "bar", "rb1c2", "bar", "gstore"]
d = np.diff(st[:, :, :12], axis=2)  # [wg][wave][11]
print(f"B={B} WGs={nwg}  cycles (median over WGs of the max over waves | mean over waves)")
tot = (st[:, :, 11] - st[:, :, 0]).max(axis=1)
for i, nm in enumerate(names):
    print(f"  {nm:8s} max-wave {np.median(d[:, :, i].max(axis=1)):8.0f}   mean-wave {np.median(d[:, :, i].mean(axis=1)):8.0f}")
print(f"  total(wave0 start -> last gstore) median {np.median(tot):.0f} cycles; kernel span {st[:, :, 11].max() - st[:, :, 0].min()} cycles")
