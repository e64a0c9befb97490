#!/usr/bin/env python3
"""Per-step stamps of the pipelined tail (vocoder_tailp.hip, M2_STAMPS build only).

    make -C m2-tts_amd/csrc OBJDIR=build_stamps OUT=build_stamps/libm2tts_hip_stamps.so EXTRA=-DM2_STAMPS
    M2TTS_HIP_LIB=m2-tts_amd/csrc/build_stamps/libm2tts_hip_stamps.so python tools/probe/stamps_tailp.py [B]

Prints, per wave role, the median over workgroups of the mean over busy steps
of (compute = before-barrier - step start) and (barrier wait = next step
start - before-barrier), and the workgroup time line (entry / exit spread)."""
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

ROLES = ["L0 convT3", "L1 rb3c1", "L2 rb3c2 (+x)", "L3 convT4", "L4 rb4c1", "L5 rb4c2 (+x)", "L6 out", "loader"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = 500
dev = torch.device("cuda", 0)
lib = _lib.load()
model = bench.fixture_model(bench.STAGE1, dev)
mel = torch.randn(B, 64, T, device=dev)
for _ in range(3):
    model.vocoder(mel)
torch.cuda.synchronize()
NW = len(ROLES)
buf = np.zeros(1024 * NW * 64 * 2, dtype=np.uint64)
fn = lib.m2_debug_stamps_tailp
fn.restype = ctypes.c_int32
fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
st = buf.reshape(1024, NW, 64, 2).astype(np.int64)
used = st[:, 0, 62, 0] != 0
st = st[used]
nwg = st.shape[0]
nsteps = int((st[0, 0, :62, 0] != 0).sum())
print(f"WGs recorded {nwg}, steps {nsteps}")
start = st[:, :, :nsteps, 0]
end = st[:, :, :nsteps, 1]
comp = end - start                       # [wg, wave, step]
wait = np.zeros_like(comp)
wait[:, :, :-1] = start[:, :, 1:] - end[:, :, :-1]
step_len = np.diff(start[:, 0, :], axis=1)  # per WG, wave 0's step starts
print(f"step length (wave-0 start to start): median {np.median(step_len):.0f} cycles, "
      f"p10 {np.percentile(step_len, 10):.0f}, p90 {np.percentile(step_len, 90):.0f}")
print(f"{'role':16s} {'compute':>9s} {'max-comp':>9s} {'wait':>8s}   (cycles/step, median over WGs)")
for w, name in enumerate(ROLES):
    c = np.median(comp[:, w, 2:-2].mean(axis=1))
    cm = np.median(comp[:, w, 2:-2].max(axis=1))
    wt = np.median(wait[:, w, 2:-3].mean(axis=1))
    print(f"{name:16s} {c:9.0f} {cm:9.0f} {wt:8.0f}")
ent = st[:, 0, 62, 0]
ex = st[:, :, 63, 0].max(axis=1)
t0 = ent.min()
dur = ex - ent
print(f"WG duration median {np.median(dur):.0f} cycles; entries span {ent.max() - t0:.0f}, "
      f"last exit {ex.max() - t0:.0f} cycles after the first entry")
# which step is slowest: per step index, median over WGs of the max compute over waves
slow = np.median(comp.max(axis=1), axis=0)
print("per-step max compute over waves (median over WGs):", " ".join(f"{v:.0f}" for v in slow))
