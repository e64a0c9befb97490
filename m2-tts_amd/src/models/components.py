"""Drop-in ``models.components`` for MI355X: same classes, constructor
signatures, parameter names and init as the reference
(``src/models/components.py``), with every forward executed by the gfx950
HIP kernels of ``m2amd`` (no CPU path; CPU tensors raise).

Semantics are the reference's EVAL-mode forward.  Training-time behaviour
(dropout, BatchNorm batch statistics, gradient checkpointing, autograd) is
out of scope; a module in training mode computes the eval
function and warns once.
"""
from __future__ import annotations

import math
import warnings
from typing import Optional, Tuple

import torch
import torch.nn as nn

from m2amd import ops

Tensor = torch.Tensor

_WARNED = set()


def _eval_only(module: nn.Module):
    if module.training and type(module).__name__ not in _WARNED:
        _WARNED.add(type(module).__name__)
        warnings.warn(f"m2-tts_amd {type(module).__name__}: inference kernels only - training-mode "
                      f"dropout/BatchNorm statistics are not applied", RuntimeWarning, stacklevel=3)


class PositionalEncoding(nn.Module):
    """Sinusoidal table as a persistent buffer ``pe`` [1, max_length, H]
    (reference components.py:15-39).  forward: x + pe[:, :S]."""

    def __init__(self, hidden_dim: int, max_length: int = 5000):
        super().__init__()
        pos = torch.arange(0, max_length).unsqueeze(1).float()
        freq = torch.exp(torch.arange(0, hidden_dim, 2).float() * -(math.log(10000.0) / hidden_dim))
        table = torch.zeros(max_length, hidden_dim)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", table.unsqueeze(0))

    def forward(self, x: Tensor) -> Tensor:
        return ops.add_positional(x, self.pe[0])


class MultiHeadAttention(nn.Module):
    """qkv projection (no bias) -> softmax(QK^T/sqrt(hd), -1e9 key mask) V ->
    out_proj (reference components.py:42-90).  ``mask`` is the [B, N] key
    padding mask (True/1 = attend)."""

    def __init__(self, hidden_dim: int, num_heads: int, dropout: float = 0.1):
        super().__init__()
        assert hidden_dim % num_heads == 0
        self.hidden_dim = hidden_dim
        self.num_heads = num_heads
        self.head_dim = hidden_dim // num_heads
        self.scale = 1.0 / math.sqrt(self.head_dim)
        self.qkv = nn.Linear(hidden_dim, hidden_dim * 3, bias=False)
        self.out_proj = nn.Linear(hidden_dim, hidden_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: Tensor, mask: Optional[Tensor] = None) -> Tensor:
        _eval_only(self)
        qkv = ops.linear(x, self.qkv.weight)
        att = ops.attention_core(qkv, self.num_heads, mask)
        return ops.linear(att, self.out_proj.weight, self.out_proj.bias)


class FeedForward(nn.Module):
    """linear2(relu(linear1(x))) (reference components.py:93-103)."""

    def __init__(self, hidden_dim: int, ffn_dim: int, dropout: float = 0.1):
        super().__init__()
        self.linear1 = nn.Linear(hidden_dim, ffn_dim)
        self.linear2 = nn.Linear(ffn_dim, hidden_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: Tensor) -> Tensor:
        _eval_only(self)
        h = ops.linear(x, self.linear1.weight, self.linear1.bias, act=ops.ACT_RELU)
        return ops.linear(h, self.linear2.weight, self.linear2.bias)


class TransformerEncoderLayer(nn.Module):
    """Pre-LN block x += MHA(LN1 x); x += FFN(LN2 x) (reference
    components.py:106-140).  LayerNorms are fused into the projection that
    consumes them and the residual adds into the projection epilogues."""

    def __init__(self, hidden_dim: int, num_heads: int, ffn_dim: int, dropout: float = 0.1,
                 use_checkpointing: bool = True):
        super().__init__()
        self.self_attn = MultiHeadAttention(hidden_dim, num_heads, dropout)
        self.ffn = FeedForward(hidden_dim, ffn_dim, dropout)
        self.norm1 = nn.LayerNorm(hidden_dim)
        self.norm2 = nn.LayerNorm(hidden_dim)
        self.dropout = nn.Dropout(dropout)
        self.use_checkpointing = use_checkpointing

    def forward(self, x: Tensor, mask: Optional[Tensor] = None) -> Tensor:
        _eval_only(self)
        a = self.self_attn
        qkv = ops.linear(x, a.qkv.weight, ln=(self.norm1.weight, self.norm1.bias))
        att = ops.attention_core(qkv, a.num_heads, mask)
        x = ops.linear(att, a.out_proj.weight, a.out_proj.bias, residual=x)
        h = ops.linear(x, self.ffn.linear1.weight, self.ffn.linear1.bias,
                       ln=(self.norm2.weight, self.norm2.bias), act=ops.ACT_RELU)
        return ops.linear(h, self.ffn.linear2.weight, self.ffn.linear2.bias, residual=x)


class ConvBlock(nn.Module):
    """Conv1d(k, pad k//2) -> BatchNorm1d (running statistics) -> ReLU
    (reference components.py:143-174), one fused kernel."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3, dropout: float = 0.1):
        super().__init__()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, padding=kernel_size // 2)
        self.norm = nn.BatchNorm1d(out_channels)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: Tensor) -> Tensor:
        _eval_only(self)
        n = self.norm
        affine = ops.batchnorm_eval_affine(n.weight, n.bias, n.running_mean, n.running_var, n.eps)
        return ops.conv1d(x, self.conv.weight, self.conv.bias, affine=affine, act=ops.ACT_RELU,
                          padding=self.conv.padding[0])


class LightweightResBlock(nn.Module):
    """conv2(leaky(conv1(x), 0.1)) + x (reference components.py:177-200): conv1
    with ``dilation`` and padding (k-1)*dilation//2, conv2 undilated.  An even
    kernel size changes the length, so the residual add fails, as in the
    reference."""

    def __init__(self, channels: int, kernel_size: int = 3, dilation: int = 1):
        super().__init__()
        self.conv1 = nn.Conv1d(channels, channels, kernel_size,
                               padding=self._get_padding(kernel_size, dilation), dilation=dilation)
        self.conv2 = nn.Conv1d(channels, channels, kernel_size, padding=self._get_padding(kernel_size, 1), dilation=1)

    @staticmethod
    def _get_padding(kernel_size: int, dilation: int) -> int:
        return (kernel_size - 1) * dilation // 2

    def forward(self, x: Tensor) -> Tensor:
        h = ops.conv1d(x, self.conv1.weight, self.conv1.bias, act=ops.ACT_LEAKY, dilation=self.conv1.dilation[0],
                       padding=self.conv1.padding[0])
        return ops.conv1d(h, self.conv2.weight, self.conv2.bias, residual=x, padding=self.conv2.padding[0])


class VariancePredictor(nn.Module):
    """2 x ConvBlock -> Conv1d(H, 1, 1) (reference components.py:203-223)."""

    def __init__(self, hidden_dim: int, kernel_size: int = 3, dropout: float = 0.1):
        super().__init__()
        self.conv_layers = nn.ModuleList([ConvBlock(hidden_dim, hidden_dim, kernel_size, dropout),
                                          ConvBlock(hidden_dim, hidden_dim, kernel_size, dropout)])
        self.projection = nn.Conv1d(hidden_dim, 1, 1)

    def forward(self, x: Tensor, _act: int = ops.ACT_NONE) -> Tensor:
        for blk in self.conv_layers:
            x = blk(x)
        return ops.conv1d(x, self.projection.weight, self.projection.bias, act=_act, padding=0)


def create_padding_mask(lengths: Tensor, max_length: int) -> Tensor:
    """``mask[b, s] = s < lengths[b]`` (reference components.py:226-241)."""
    b = lengths.size(0)
    return torch.arange(max_length, device=lengths.device).expand(b, max_length) < lengths.unsqueeze(1)


def apply_spectral_norm(module: nn.Module) -> nn.Module:
    """Training utility kept for import compatibility (reference components.py:244-248)."""
    if isinstance(module, (nn.Conv1d, nn.Conv2d, nn.Linear)):
        return nn.utils.spectral_norm(module)
    return module


class GradientClipping:
    """Training utility kept for import compatibility (reference components.py:251-259)."""

    def __init__(self, clip_value: float = 5.0):
        self.clip_value = clip_value

    def __call__(self, model: nn.Module) -> float:
        return torch.nn.utils.clip_grad_norm_(model.parameters(), self.clip_value)


def count_parameters(model: nn.Module) -> Tuple[int, int]:
    """(total, trainable) parameter counts (reference components.py:262-271)."""
    params = list(model.parameters())
    return sum(p.numel() for p in params), sum(p.numel() for p in params if p.requires_grad)


def initialize_weights(module: nn.Module) -> None:
    """Reference init (components.py:274-286): xavier-uniform Linear,
    kaiming-normal Conv1d, zero biases, unit LayerNorm.  ConvTranspose1d,
    Embedding and BatchNorm keep PyTorch defaults, as in the reference."""
    if isinstance(module, nn.Linear):
        nn.init.xavier_uniform_(module.weight)
        if module.bias is not None:
            nn.init.constant_(module.bias, 0)
    elif isinstance(module, nn.Conv1d):
        nn.init.kaiming_normal_(module.weight)
        if module.bias is not None:
            nn.init.constant_(module.bias, 0)
    elif isinstance(module, nn.LayerNorm):
        nn.init.constant_(module.weight, 1)
        nn.init.constant_(module.bias, 0)
