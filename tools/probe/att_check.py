"""Attention correctness vs a torch fp32 reference (masked and unmasked)."""
import sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
from m2amd import ops  # noqa: E402
dev = torch.device("cuda", 0)
worst = 0.0
for B, N, H in ((2, 37, 64), (3, 500, 64), (2, 511, 96), (1, 2600, 96), (4, 129, 32)):
    for masked in (False, True):
        g = torch.Generator().manual_seed(N)
        qkv = torch.randn(B, N, 3 * H, generator=g)
        mask = None
        if masked:
            lens = torch.randint(1, N + 1, (B,), generator=g)
            mask = torch.arange(N)[None, :] < lens[:, None]
        out = ops.attention_core(qkv.to(dev), 2, None if mask is None else mask.to(dev)).cpu().double()
        q, k, v = qkv.double().view(B, N, 3, 2, H // 2).permute(2, 0, 3, 1, 4)
        s = q @ k.transpose(-1, -2) / (H // 2) ** 0.5
        if mask is not None:
            s = s.masked_fill(~mask[:, None, None, :], -1e9)
        ref = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, N, H)
        err = float((out - ref).abs().max())
        worst = max(worst, err)
        print(B, N, H, masked, f"{err:.2e}")
print("WORST", worst)
assert worst < 1e-4
