"""Probe: which transformer forms stay finite when the decoder's attention
scores leave the f16 range (the test_gpu_range.py case)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "m2-tts_amd", "src"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import m2tts_oracle as orc  # noqa: E402
from conftest import golden_state, stage_config  # noqa: E402
from models.tts_model import M2TTSModel  # noqa: E402

dev = torch.device("cuda", 0)
cfg = stage_config("s2")
H, hd = cfg.hidden_dim, cfg.hidden_dim // 2
sd = golden_state("s2")
w = sd["decoder.layers.0.self_attn.qkv.weight"].clone()
u = torch.randn(H, generator=torch.Generator().manual_seed(3))
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
T = int(sys.argv[2]) if len(sys.argv) > 2 else 300
envs = ({"M2_TFL_RB": "4"}, {"M2_TFL_RB": "4", "M2_TFL_QS2": "3"}, {"M2_TFL_RB": "4", "M2_TFL_QS2": "0"},
        {"M2_TFL_RB": "1"}, {"M2_TFL_RB": "2"}, {"M2_TF_LAYER": "0"}, {"M2_TF_UNFUSED": "1"})
if len(sys.argv) > 3:
    envs = ({"M2_TFL_RB": "4"}, {"M2_TFL_RB": "4", "M2_TFL_QS2": "3"}, {"M2_TFL_RB": "4", "M2_TFL_QS2": "2"},
            {"M2_TFL_RB": "4", "M2_TFL_QS2": "4"}, {"M2_TFL_RB": "4", "M2_TFL_QS2": "0"})
w[: 2 * H] = scale * u
sd["decoder.layers.0.self_attn.qkv.weight"] = w
x = torch.randn(2, T, H, generator=torch.Generator().manual_seed(4))
ref = orc.mel_decoder(sd, cfg, x)
import torch.nn.functional as F  # noqa: E402
xn = F.layer_norm(x, (H,), sd["decoder.layers.0.norm1.weight"], sd["decoder.layers.0.norm1.bias"])
q = xn @ w[:hd].T
sc = (q @ q.transpose(1, 2)) / hd ** 0.5 * 1.4426950408889634
print(f"scale {scale} T {T}: max score {float(sc.amax()):.4g}, max row range {float((sc.amax(-1) - sc.amin(-1)).amax()):.4g}; "
      f"ref finite", bool(torch.isfinite(ref).all()))
for env in envs:
    for k in ("M2_TFL_RB", "M2_TFL_QS2", "M2_TF_LAYER", "M2_TF_UNFUSED"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = M2TTSModel(**cfg.as_dict())
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    with torch.no_grad():
        mel = m.decoder(x.to(dev)).cpu()
    fin = torch.isfinite(mel)
    err = float((mel[fin] - ref[fin]).abs().max()) if fin.any() else float("nan")
    bad = (~fin).any(-1)  # [B, T] frames with a non-finite mel value
    where = [(b, int(bad[b].nonzero()[0])) for b in range(bad.shape[0]) if bad[b].any()]
    print(env, "finite frac", round(float(fin.float().mean()), 4), "maxabs(finite)", err,
          "bad frames per utt", bad.sum(-1).tolist(), "first", where, flush=True)
