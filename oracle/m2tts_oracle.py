"""CPU oracle for the m2-tts mel-synthesis + vocoder forward path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``m2-tts_amd/``) may
import this module.  It is used by ``tests/`` (as the parity checker), by
``__graft_entry__.smoke()`` (as the checker) and by ``bench.py``'s
``cpu_baseline`` leg (timed on the host cores as the reference CPU path).

What it is: a functional restatement of ``M2TTSModel.forward`` /
``M2TTSModel.inference`` (reference ``src/models/tts_model.py:350-438``) in
the reference's own op order, written against a plain ``state_dict`` so it
needs no ``nn.Module``.  Every ATen op is the one the reference calls, so on
the same CPU build it reproduces the reference bit for bit; this is checked
against an import of the reference by ``tests/golden/make_golden.py`` and the
committed fixtures pin it from then on (see DESIGN.md "Oracle").

Deliberately kept reference quirks (they are the behaviour being matched):
  * the length regulator is the Python double loop with one ``.item()`` per
    phoneme and ``int()`` truncation (tts_model.py:146-162);
  * ``inference`` runs the vocoder twice - once inside ``forward`` and again
    on the (possibly re-decoded) mel (tts_model.py:388-391, 435-436).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# SimpleVocoder upsample schedule, hard-coded in the reference
# (tts_model.py:244).
UPSAMPLE_RATES = (4, 4, 2, 2)
LN_EPS = 1e-5          # nn.LayerNorm default (components.py:136-137)
BN_EPS = 1e-5          # nn.BatchNorm1d default (components.py:160)
MASK_FILL = -1e9       # components.py:81 masked_fill_ value
LEAKY = 0.1            # tts_model.py:291, components.py:198


@dataclass(frozen=True)
class OracleConfig:
    """The 8 constructor arguments of ``M2TTSModel`` (tts_model.py:303-313)."""
    vocab_size: int = 256
    hidden_dim: int = 64
    mel_channels: int = 64
    text_encoder_layers: int = 2
    decoder_layers: int = 2
    num_heads: int = 2
    dropout: float = 0.1
    vocoder_channels: int = 128

    def as_dict(self):
        return asdict(self)


STAGE1 = OracleConfig()                                     # configs/stage1_poc.yaml:4-27
STAGE2 = OracleConfig(hidden_dim=96, mel_channels=80, text_encoder_layers=3,
                      decoder_layers=3, vocoder_channels=256)  # configs/stage2_quality.yaml:4-28


# ----------------------------------------------------------------------------
# components.py restatements
# ----------------------------------------------------------------------------
def padding_mask(lengths: Tensor, max_length: int) -> Tensor:
    """components.py:226-241: ``arange(S) < lengths[:, None]``."""
    b = lengths.size(0)
    return torch.arange(max_length, device=lengths.device).expand(b, max_length) < lengths.unsqueeze(1)


def _layer_norm(x: Tensor, sd: Dict[str, Tensor], p: str) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], LN_EPS)


def attention(sd: Dict[str, Tensor], p: str, x: Tensor, heads: int,
              mask: Optional[Tensor]) -> Tensor:
    """MultiHeadAttention.forward, components.py:59-90.

    qkv projection without bias, scale applied after the QK^T matmul, key
    mask filled with -1e9 (not -inf), softmax, AV, out_proj with bias.
    """
    b, n, h = x.shape
    hd = h // heads
    qkv = F.linear(x, sd[p + ".qkv.weight"]).reshape(b, n, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    scores = torch.matmul(q, k.transpose(-2, -1)) * (1.0 / math.sqrt(hd))
    if mask is not None:
        m = mask.unsqueeze(1).unsqueeze(1).expand(b, heads, n, n)
        scores.masked_fill_(m == 0, MASK_FILL)
    attn = F.softmax(scores, dim=-1)
    out = torch.matmul(attn, v).transpose(1, 2).reshape(b, n, h)
    return F.linear(out, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"])


def feed_forward(sd: Dict[str, Tensor], p: str, x: Tensor) -> Tensor:
    """FeedForward.forward, components.py:102-103 (dropout = identity in eval)."""
    hdn = F.relu(F.linear(x, sd[p + ".linear1.weight"], sd[p + ".linear1.bias"]))
    return F.linear(hdn, sd[p + ".linear2.weight"], sd[p + ".linear2.bias"])


def encoder_layer(sd: Dict[str, Tensor], p: str, x: Tensor, heads: int,
                  mask: Optional[Tensor]) -> Tensor:
    """TransformerEncoderLayer._forward, components.py:131-140 (pre-LN)."""
    x = x + attention(sd, p + ".self_attn", _layer_norm(x, sd, p + ".norm1"), heads, mask)
    x = x + feed_forward(sd, p + ".ffn", _layer_norm(x, sd, p + ".norm2"))
    return x


def conv_block(sd: Dict[str, Tensor], p: str, x: Tensor) -> Tensor:
    """ConvBlock.forward in eval mode, components.py:163-174."""
    x = F.conv1d(x, sd[p + ".conv.weight"], sd[p + ".conv.bias"], padding=sd[p + ".conv.weight"].shape[-1] // 2)
    x = F.batch_norm(x, sd[p + ".norm.running_mean"], sd[p + ".norm.running_var"],
                     sd[p + ".norm.weight"], sd[p + ".norm.bias"], False, 0.1, BN_EPS)
    return F.relu(x)


def resblock(sd: Dict[str, Tensor], p: str, x: Tensor, dilation: int = 1) -> Tensor:
    """LightweightResBlock.forward, components.py:196-200: conv1 with
    `dilation` and padding (k-1)*dilation//2 (components.py:180-189), conv2
    undilated with padding (k-1)//2 (the vocoder uses k=3, dilation 1)."""
    k = sd[p + ".conv1.weight"].shape[-1]
    y = F.leaky_relu(F.conv1d(x, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], padding=(k - 1) * dilation // 2,
                              dilation=dilation), LEAKY)
    y = F.conv1d(y, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], padding=(k - 1) // 2)
    return y + x


def conv_transpose(sd: Dict[str, Tensor], p: str, x: Tensor, rate: int) -> Tensor:
    """ConvTranspose1d(c, c/2, k=2r, s=r, p=r/2), tts_model.py:255-263."""
    return F.conv_transpose1d(x, sd[p + ".weight"], sd[p + ".bias"], stride=rate, padding=rate // 2)


# ----------------------------------------------------------------------------
# tts_model.py restatements
# ----------------------------------------------------------------------------
def text_encoder(sd: Dict[str, Tensor], cfg: OracleConfig, ids: Tensor,
                 lengths: Optional[Tensor]) -> Tuple[Tensor, Optional[Tensor]]:
    """TextEncoder.forward, tts_model.py:57-89."""
    _, s = ids.shape
    mask = padding_mask(lengths, s) if lengths is not None else None
    x = F.embedding(ids, sd["text_encoder.embedding.weight"])
    x = x * (cfg.hidden_dim ** 0.5)
    x = x + sd["text_encoder.pos_encoding.pe"][:, :s]
    for i in range(cfg.text_encoder_layers):
        x = encoder_layer(sd, f"text_encoder.layers.{i}", x, cfg.num_heads, mask)
    return _layer_norm(x, sd, "text_encoder.norm"), mask


def duration_predictor(sd: Dict[str, Tensor], enc: Tensor) -> Tensor:
    """DurationPredictor.forward, tts_model.py:99-117 (no padding mask)."""
    x = enc.transpose(1, 2)
    p = "duration_predictor.predictor"
    for j in range(2):
        x = conv_block(sd, f"{p}.conv_layers.{j}", x)
    x = F.conv1d(x, sd[p + ".projection.weight"], sd[p + ".projection.bias"])
    return F.softplus(x.squeeze(1))


def length_regulator(enc: Tensor, durations: Tensor, max_length: Optional[int] = None) -> Tensor:
    """LengthRegulator.forward, tts_model.py:126-178 - the Python loop as written."""
    b, s, h = enc.shape
    seqs = []
    for bi in range(b):
        parts = []
        for si in range(s):
            d = int(durations[bi, si].item())
            if d > 0:
                parts.append(enc[bi, si].unsqueeze(0).repeat(d, 1))
        seqs.append(torch.cat(parts, dim=0) if parts else torch.zeros(1, h, device=enc.device))
    if max_length is None:
        max_length = max(q.size(0) for q in seqs)
    out = []
    for q in seqs:
        if q.size(0) < max_length:
            q = torch.cat([q, torch.zeros(max_length - q.size(0), h, device=enc.device)], dim=0)
        elif q.size(0) > max_length:
            q = q[:max_length]
        out.append(q)
    return torch.stack(out, dim=0)


def mel_decoder(sd: Dict[str, Tensor], cfg: OracleConfig, x: Tensor) -> Tensor:
    """MelDecoder.forward, tts_model.py:211-228 (mask=None: padded frames attend)."""
    for i in range(cfg.decoder_layers):
        x = encoder_layer(sd, f"decoder.layers.{i}", x, cfg.num_heads, None)
    x = _layer_norm(x, sd, "decoder.norm")
    return F.linear(x, sd["decoder.mel_projection.weight"], sd["decoder.mel_projection.bias"])


def vocoder_pre_tanh(sd: Dict[str, Tensor], mel_bmt: Tensor) -> Tensor:
    """SimpleVocoder.forward up to the output conv (tts_model.py:279-296), the
    value tanh is applied to at :297 (the stress tests' conditioning check)."""
    ks = sd["vocoder.input_conv.weight"].shape[-1]
    x = F.conv1d(mel_bmt, sd["vocoder.input_conv.weight"], sd["vocoder.input_conv.bias"], padding=ks // 2)
    for k, r in enumerate(UPSAMPLE_RATES):
        x = F.leaky_relu(conv_transpose(sd, f"vocoder.upsamples.{k}", x, r), LEAKY)
        x = resblock(sd, f"vocoder.resblocks.{k}", x)
    return F.conv1d(x, sd["vocoder.output_conv.weight"], sd["vocoder.output_conv.bias"], padding=ks // 2)


def vocoder(sd: Dict[str, Tensor], mel_bmt: Tensor) -> Tensor:
    """SimpleVocoder.forward, tts_model.py:279-297; mel [B,M,T] -> audio [B,1,64T].
    Convs pad kernel_size // 2 (tts_model.py:246, 272; kernel_size 3 in M2TTSModel)."""
    return torch.tanh(vocoder_pre_tanh(sd, mel_bmt))


def forward(sd: Dict[str, Tensor], cfg: OracleConfig, ids: Tensor,
            lengths: Optional[Tensor] = None, target_durations: Optional[Tensor] = None,
            max_target_length: Optional[int] = None, run_vocoder: bool = True) -> Dict[str, Tensor]:
    """M2TTSModel.forward in eval mode, tts_model.py:350-400."""
    with torch.no_grad():
        enc, mask = text_encoder(sd, cfg, ids, lengths)
        dur = duration_predictor(sd, enc)
        durations = target_durations if target_durations is not None else dur
        reg = length_regulator(enc, durations, max_target_length)
        mel = mel_decoder(sd, cfg, reg)
        audio = vocoder(sd, mel.transpose(1, 2)) if run_vocoder else None
    return {"encoder_output": enc, "duration_pred": dur, "regulated_output": reg,
            "mel_output": mel, "audio_output": audio, "padding_mask": mask}


def inference(sd: Dict[str, Tensor], cfg: OracleConfig, ids: Tensor,
              lengths: Optional[Tensor] = None, duration_scale: float = 1.0,
              as_written: bool = True) -> Tuple[Tensor, Tensor]:
    """M2TTSModel.inference, tts_model.py:402-438.

    ``as_written=True`` keeps the reference's redundant first vocoder pass
    inside ``forward`` (the CPU baseline times it that way); ``False`` runs
    the vocoder once.  Outputs are identical either way.
    """
    with torch.no_grad():
        out = forward(sd, cfg, ids, lengths, run_vocoder=as_written)
        if duration_scale != 1.0:
            reg = length_regulator(out["encoder_output"], out["duration_pred"] * duration_scale)
            out["mel_output"] = mel_decoder(sd, cfg, reg)
        audio = vocoder(sd, out["mel_output"].transpose(1, 2))
    return out["mel_output"], audio


# ----------------------------------------------------------------------------
# Fixture weights: deterministic, durations pinned to 5.5.
# ----------------------------------------------------------------------------
def pin_durations(sd: Dict[str, Tensor], bias: float = 5.5, weight_scale: float = 0.01) -> Dict[str, Tensor]:
    """Make every predicted duration ~= ``bias`` (0.49 from an integer at 5.5).

    softplus(5.5 + small) ~ 5.504, so int() gives exactly 5 frames/phoneme.
    """
    sd = dict(sd)
    p = "duration_predictor.predictor.projection"
    sd[p + ".weight"] = sd[p + ".weight"] * weight_scale
    sd[p + ".bias"] = torch.full_like(sd[p + ".bias"], bias)
    return sd


def vocoder_audio_len(t_frames: int) -> int:
    """64 samples per mel frame: each ConvT(k=2r, s=r, p=r/2) maps L -> r*L."""
    n = t_frames
    for r in UPSAMPLE_RATES:
        n *= r
    return n
