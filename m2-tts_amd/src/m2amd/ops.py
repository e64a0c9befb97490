"""Tensor-level wrappers of the C-ABI kernels (one function per entry point).

Every function takes torch tensors that live on a ROCm device, allocates its
outputs with torch (caching allocator), and launches on the current torch
stream.  Nothing here computes on the CPU: a CPU tensor is an error.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from . import _lib
from ._lib import ACT_LEAKY, ACT_NONE, ACT_RELU, ACT_SOFTPLUS, ACT_TANH, M2Error  # noqa: F401

Tensor = torch.Tensor


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors: Optional[Tensor], what: str = "m2-tts_amd"):
    """Fail loudly on CPU tensors: the product path has no CPU fallback."""
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(
                f"{what}: tensors must be on a ROCm GPU device (got {t.device}); move the module "
                f"and its inputs with .to('cuda').  m2-tts_amd has no CPU execution path.")


def f32c(t: Tensor) -> Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"m2-tts_amd computes in fp32; got {t.dtype}")
    return t.contiguous()


def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None, *, ln: Optional[tuple] = None,
           act: int = ACT_NONE, residual: Optional[Tensor] = None, out: Optional[Tensor] = None) -> Tensor:
    """y = act(LN?(x) @ W^T + b) (+ residual) over the last dim (nn.Linear layout W [N, K])."""
    require_device(x, weight, what="linear")
    x = f32c(x)
    K = x.shape[-1]
    N = weight.shape[0]
    R = x.numel() // K if K else 0
    y = out if out is not None else torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
    g, b_ = (ln if ln is not None else (None, None))
    res = f32c(residual) if residual is not None else None
    _lib.call("m2_linear", _ptr(x), _ptr(g), _ptr(b_), _ptr(f32c(weight)), _ptr(bias), _ptr(res), act,
              R, K, N, _ptr(y), stream_handle(x.device))
    return y


def layer_norm(x: Tensor, weight: Tensor, bias: Tensor) -> Tensor:
    require_device(x, what="layer_norm")
    x = f32c(x)
    K = x.shape[-1]
    y = torch.empty_like(x)
    _lib.call("m2_layer_norm", _ptr(x), _ptr(weight), _ptr(bias), x.numel() // K, K, _ptr(y),
              stream_handle(x.device))
    return y


def attention_core(qkv: Tensor, heads: int, key_mask: Optional[Tensor]) -> Tensor:
    """softmax(QK^T/sqrt(hd) with -1e9 key mask) V for qkv [B,N,3H] -> [B,N,H]."""
    require_device(qkv, what="attention")
    qkv = f32c(qkv)
    B, N, H3 = qkv.shape
    H = H3 // 3
    out = torch.empty(B, N, H, device=qkv.device, dtype=torch.float32)
    m = None
    if key_mask is not None:
        m = key_mask.to(torch.uint8).contiguous() if key_mask.dtype != torch.bool else key_mask.contiguous()
    _lib.call("m2_attention", _ptr(qkv), _ptr(m), B, N, H, heads, _ptr(out), stream_handle(qkv.device))
    return out


def conv1d(x: Tensor, weight: Tensor, bias: Tensor, *, act: int = ACT_NONE,
           affine: Optional[tuple] = None, residual: Optional[Tensor] = None, dilation: int = 1,
           padding: Optional[int] = None) -> Tensor:
    """Conv1d(k, dilation, zero padding (default k//2)) [+ per-channel affine]
    [+ act] [+ residual], x [B,Cin,L] -> [B,Cout,L + 2 pad - dil (k - 1)].
    k = 1 | 3 with dilation 1 and padding k//2 run the tiled kernel
    (m2_conv1d); every other geometry the general one (m2_conv1d_ex)."""
    require_device(x, weight, what="conv1d")
    x = f32c(x)
    B, Cin, L = x.shape
    Cout, _, K = weight.shape
    pad = K // 2 if padding is None else int(padding)
    Lo = L + 2 * pad - dilation * (K - 1)
    if residual is not None and Lo != L:
        raise RuntimeError(f"conv1d: output length {Lo} != input length {L}: the residual add has mismatched shapes")
    y = torch.empty(B, Cout, max(Lo, 0), device=x.device, dtype=torch.float32)
    al, be = affine if affine is not None else (None, None)
    res = f32c(residual) if residual is not None else None
    if K in (1, 3) and dilation == 1 and pad == K // 2:
        _lib.call("m2_conv1d", _ptr(x), _ptr(f32c(weight)), _ptr(f32c(bias)), _ptr(al), _ptr(be), _ptr(res), K, act,
                  B, Cin, Cout, L, _ptr(y), stream_handle(x.device))
    else:
        _lib.call("m2_conv1d_ex", _ptr(x), _ptr(f32c(weight)), _ptr(f32c(bias)), _ptr(al), _ptr(be), _ptr(res), K,
                  int(dilation), pad, act, B, Cin, Cout, L, _ptr(y), stream_handle(x.device))
    return y


def conv_transpose1d(x: Tensor, weight: Tensor, bias: Tensor, rate: int, *, act: int = ACT_NONE) -> Tensor:
    """ConvTranspose1d(k=2r, stride=r, padding=r/2) [+ act]; weight [Cin, Cout, 2r]."""
    require_device(x, weight, what="conv_transpose1d")
    x = f32c(x)
    B, Cin, L = x.shape
    Cout = weight.shape[1]
    y = torch.empty(B, Cout, L * rate, device=x.device, dtype=torch.float32)
    _lib.call("m2_conv_transpose1d", _ptr(x), _ptr(f32c(weight)), _ptr(f32c(bias)), rate, act, B, Cin, Cout, L,
              _ptr(y), stream_handle(x.device))
    return y


def embed_positional(ids: Tensor, emb: Tensor, pe: Tensor, scale: float) -> Tensor:
    require_device(ids, emb, what="embedding")
    ids = ids.to(torch.int64).contiguous()
    B, S = ids.shape
    H = emb.shape[1]
    y = torch.empty(B, S, H, device=emb.device, dtype=torch.float32)
    _lib.call("m2_embed_positional", _ptr(ids), _ptr(f32c(emb)), _ptr(f32c(pe)), B, S, H, emb.shape[0],
              float(scale), _ptr(y), stream_handle(emb.device))
    return y


def add_positional(x: Tensor, pe: Tensor) -> Tensor:
    require_device(x, pe, what="positional encoding")
    x = f32c(x)
    B, S, H = x.shape
    if S > pe.shape[-2]:
        raise RuntimeError(f"sequence length {S} exceeds the positional table ({pe.shape[-2]})")
    y = torch.empty_like(x)
    _lib.call("m2_add_positional", _ptr(x), _ptr(f32c(pe)), B, S, H, _ptr(y), stream_handle(x.device))
    return y


def durations_for_regulator(durations: Tensor):
    """Return (tensor, is_int) in the form m2_length_regulator_count reads.

    fp32 durations are passed as-is (int() truncation happens in the kernel);
    integer durations become int32; other float dtypes are truncated toward
    zero in their own precision first (what int(d.item()) does)."""
    if durations.dtype == torch.float32:
        return durations.contiguous(), 0
    if durations.is_floating_point():
        return torch.trunc(durations).clamp(-2**30, 2**30).to(torch.int32).contiguous(), 1
    return durations.clamp(-2**30, 2**30).to(torch.int32).contiguous(), 1


def frame_counts(durations: Tensor, scale: float = 1.0):
    """Counting half of the length regulator (m2_length_regulator_count):
    returns (cum [B,S+1] int32 exclusive prefix sums, T [B] int32, Tmax [1] int32)."""
    require_device(durations, what="length_regulator")
    B, S = durations.shape
    d, is_int = durations_for_regulator(durations)
    dev = durations.device
    cum = torch.empty(B, S + 1, device=dev, dtype=torch.int32)
    tot = torch.empty(B, device=dev, dtype=torch.int32)
    tmax = torch.empty(1, device=dev, dtype=torch.int32)
    _lib.call("m2_length_regulator_count", _ptr(d), is_int, float(scale), B, S, _ptr(cum), _ptr(tot), _ptr(tmax),
              stream_handle(dev))
    return cum, tot, tmax


def frame_counts_sync(durations: Tensor, scale: float = 1.0):
    """frame_counts plus the host read of T_max (m2_length_regulator_count_sync:
    a host-mapped mailbox the count kernel posts to, polled in C with the GIL
    released): returns (cum, T, Tmax device tensors, Tmax as an int)."""
    require_device(durations, what="length_regulator")
    B, S = durations.shape
    d, is_int = durations_for_regulator(durations)
    dev = durations.device
    cum = torch.empty(B, S + 1, device=dev, dtype=torch.int32)
    tot = torch.empty(B, device=dev, dtype=torch.int32)
    tmax = torch.empty(1, device=dev, dtype=torch.int32)
    host = ctypes.c_int32(0)
    _lib.call("m2_length_regulator_count_sync", _ptr(d), is_int, float(scale), B, S, _ptr(cum), _ptr(tot), _ptr(tmax),
              ctypes.addressof(host), stream_handle(dev))
    return cum, tot, tmax, int(host.value)


def expand_frames(enc: Tensor, cum: Tensor, T_out: int) -> Tensor:
    """Expanding half (m2_length_regulator_expand): [B,S,H] -> [B,T_out,H]."""
    enc = f32c(enc)
    B, S, H = enc.shape
    out = torch.empty(B, T_out, H, device=enc.device, dtype=torch.float32)
    _lib.call("m2_length_regulator_expand", _ptr(enc), _ptr(cum), B, S, H, T_out, _ptr(out), stream_handle(enc.device))
    return out


def regulate(enc: Tensor, durations: Tensor, max_length: Optional[int] = None, scale: float = 1.0) -> Tensor:
    """LengthRegulator.forward (tts_model.py:126-178) on the GPU: scan + gather.

    One device->host read of the batch maximum frame count, only when
    max_length is not given (it sizes the output)."""
    require_device(enc, durations, what="length_regulator")
    if max_length is not None:
        cum, _, _ = frame_counts(durations, scale)
        return expand_frames(enc, cum, max_length)
    cum, _, _, t_max = frame_counts_sync(durations, scale)
    # an utterance with no frames becomes one zero frame (tts_model.py:158-160)
    return expand_frames(enc, cum, max(1, t_max))


def batchnorm_eval_affine(weight: Tensor, bias: Tensor, mean: Tensor, var: Tensor, eps: float):
    """alpha = w / sqrt(var + eps), beta = b - mean * alpha (ATen's eval-mode form).

    Parameter preprocessing on the device (a few elementwise ops on H-sized
    vectors), not part of the per-frame work."""
    invstd = 1.0 / torch.sqrt(var + eps)
    alpha = invstd * weight
    return alpha.contiguous(), (bias - mean * alpha).contiguous()


def sqrt_hidden(h: int) -> float:
    return h ** 0.5


def inv_sqrt(hd: int) -> float:
    return 1.0 / math.sqrt(hd)
