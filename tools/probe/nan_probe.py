"""Locate non-finite vocoder output: per kernel-variant env, stage, NaN count and first NaN sample index."""
import os, subprocess, sys, json
code = r'''
import sys, torch, json
sys.path.insert(0, "m2-tts_amd/src"); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from conftest import golden_state, stage_config
from models.tts_model import M2TTSModel
out = {}
for stage in ("s1", "s2"):
    m = M2TTSModel(**stage_config(stage).as_dict()); m.load_state_dict(golden_state(stage)); m = m.cuda().eval()
    for T in (7, 64, 500):
        mel = torch.randn(2, stage_config(stage).mel_channels, T, generator=torch.Generator().manual_seed(1)).cuda()
        a = m.vocoder(mel)
        m._hip(mel.device).check()
        bad = (~torch.isfinite(a)).nonzero()
        cols = sorted(set((bad[:, 2] // 256).tolist()))  # U1-column-ish buckets of 256 samples
        out[f"{stage}_T{T}"] = [int(bad.shape[0]), a.numel(), bad[:3].tolist(), cols[:20]]
print(json.dumps(out))
'''
for env in ({}, {"M2_VOC_MID_X3": "1"}, {"M2_VOC_TAIL_X3": "1"}):
    e = dict(os.environ); e.update(env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    print(env, r.stdout.strip()[-800:], r.stderr.strip()[-300:] if r.returncode else "")
