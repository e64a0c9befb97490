"""Model-level runtime: one packed ``m2_model`` handle per (model, device).

``HipModel`` uploads the weights of an ``M2TTSModel`` once
(``m2_model_create``) and exposes the stage entry points of the C ABI with
torch tensors.  ``M2TTSModel`` (models/tts_model.py) keeps one HipModel per
device in a side table and rebuilds it when any parameter/buffer changes
storage or version (``load_state_dict``, ``.to()``, in-place edits).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from .ops import f32c, require_device, stream_handle

Tensor = torch.Tensor


def make_config(vocab_size: int, hidden_dim: int, mel_channels: int, text_encoder_layers: int,
                decoder_layers: int, num_heads: int, vocoder_channels: int, max_positions: int) -> _lib.M2Config:
    return _lib.M2Config(vocab_size, hidden_dim, mel_channels, text_encoder_layers, decoder_layers,
                         num_heads, vocoder_channels, max_positions)


def weight_names(cfg: _lib.M2Config):
    lib = _lib.load()
    n = lib.m2_weight_count(ctypes.byref(cfg))
    _lib.check(0 if n >= 0 else n, "m2_weight_count")
    buf = ctypes.create_string_buffer(256)
    names = []
    for i in range(n):
        _lib.check(lib.m2_weight_name(ctypes.byref(cfg), i, buf, 256), "m2_weight_name")
        names.append((buf.value.decode(), int(lib.m2_weight_numel(ctypes.byref(cfg), i))))
    return names


# Structural changes (a parameter, buffer or submodule registered or replaced
# anywhere) bump this generation; in-place updates (load_state_dict's copy_,
# optimizer steps, param.data = ...) show up in the tensors' version counters
# and storage pointers.  Walking state_dict() on every call cost ~150 us of
# host time per forward - more than the vocoder's GPU time at B=32.
_GEN = [0]


def _bump(*_args):
    _GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump)
torch.nn.modules.module.register_module_module_registration_hook(_bump)


def state_key(module: torch.nn.Module) -> Tuple:
    """Identity of the weights as stored right now (storage + version counters)."""
    cache = module.__dict__.get("_m2_state_tensors")
    if cache is None or cache[0] != _GEN[0] or cache[1] != id(module):
        cache = (_GEN[0], id(module), list(module.state_dict(keep_vars=True).values()))
        module.__dict__["_m2_state_tensors"] = cache
    return (cache[0],) + tuple([(t.data_ptr(), t._version) for t in cache[2]])


class HipModel:
    def __init__(self, state: Dict[str, Tensor], cfg: _lib.M2Config, device: torch.device):
        lib = _lib.load()
        self.cfg = cfg
        self.device = torch.device(device)
        self.H = cfg.hidden_dim
        self.M = cfg.mel_channels
        names = weight_names(cfg)
        ptrs = (ctypes.c_void_p * len(names))()
        keep = []
        for i, (name, numel) in enumerate(names):
            if name not in state:
                raise KeyError(f"m2-tts_amd: state_dict is missing {name!r}")
            t = state[name]
            if t.dtype == torch.int64:  # num_batches_tracked: not used by the forward path
                ptrs[i] = t.data_ptr() if t.is_cuda else None
                continue
            require_device(t, what=f"weight {name}")
            t = f32c(t.detach())
            if t.numel() != numel:
                raise ValueError(f"m2-tts_amd: {name} has {t.numel()} elements, expected {numel}")
            keep.append(t)
            ptrs[i] = t.data_ptr()
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.m2_model_create(ctypes.byref(cfg), ptrs, len(names), stream_handle(self.device),
                                           ctypes.byref(handle)), "m2_model_create")
        self.handle = handle
        self._ws: Optional[Tensor] = None
        self._ws_chunk: Optional[Tensor] = None
        self._front: Optional[Tensor] = None
        self.chunk_frames = 0
        self._sizes: Dict[Tuple, int] = {}
        self._tcap: Dict[Tuple[int, int], int] = {}
        self._finalizer = weakref.finalize(self, lib.m2_model_destroy, handle)

    # ------------------------------------------------------------------ scratch
    def workspace(self, B: int, S: int, T: int) -> Tensor:
        return self._scratch("_ws", self._size("m2_workspace_bytes", B, S, T))

    def _size(self, fn: str, *args) -> int:
        key = (fn,) + args
        n = self._sizes.get(key)
        if n is None:
            n = self._sizes[key] = int(getattr(_lib.load(), fn)(self.handle, *args))
        return n

    def _scratch(self, attr: str, need: int) -> Tensor:
        buf = getattr(self, attr)
        if buf is None or buf.numel() < need:
            buf = torch.empty(max(need, 1 << 20), dtype=torch.uint8, device=self.device)
            setattr(self, attr, buf)
        return buf

    # ------------------------------------------------------------------ whole path
    def inference(self, ids: Tensor, lengths: Optional[Tensor], scale: float) -> Tuple[Tensor, Tensor]:
        """M2TTSModel.inference (tts_model.py:402-438), normally ONE library call
        (m2_inference): encoder, durations, frame counts, the T_max read, then
        expansion, decoder and vocoder enqueued from C right after the read.

        The outputs are allocated before T is known, for a frame capacity per
        (B, S) learnt from earlier calls (the last T that exceeded it, or fell
        under half of it); the result is the contiguous [B,T,M] / [B,1,64T]
        prefix of those buffers.  With a capacity the back half is enqueued
        before the host reads T (kernels take T from the device).  A call whose
        T exceeds the capacity allocates exactly and finishes with
        m2_inference_back."""
        require_device(ids, lengths, what="M2TTSModel")
        if ids.dtype != torch.int64 or not ids.is_contiguous():
            ids = ids.to(torch.int64).contiguous()
        B, S = ids.shape
        if S > self.cfg.max_positions:
            raise RuntimeError(f"sequence length {S} exceeds the positional table ({self.cfg.max_positions})")
        lens = None
        if lengths is not None:
            lens = lengths if lengths.dtype == torch.int64 and lengths.is_contiguous() else \
                lengths.to(torch.int64).contiguous()
        lib = _lib.load()
        st = stream_handle(self.device)
        M, dev, f32 = self.M, self.device, torch.float32
        cap = self._tcap.get((B, S), 0)
        front = self._scratch("_front", self._size("m2_front_bytes", B, S))
        ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, cap))
        mel_buf = torch.empty(B * cap * M, device=dev, dtype=f32)
        audio_buf = torch.empty(B * 64 * cap, device=dev, dtype=f32)
        T = ctypes.c_int32(0)
        done = ctypes.c_int32(0)
        _lib.check(lib.m2_inference(self.handle, ids.data_ptr(), None if lens is None else lens.data_ptr(), B, S,
                                    float(scale), front.data_ptr(), front.numel(), ws.data_ptr(), ws.numel(),
                                    mel_buf.data_ptr(), mel_buf.numel(), audio_buf.data_ptr(), audio_buf.numel(),
                                    ctypes.byref(T), ctypes.byref(done), st), "m2_inference")
        T = T.value
        if done.value:
            mel = mel_buf[:B * T * M].view(B, T, M)
            audio = audio_buf[:B * 64 * T].view(B, 1, 64 * T)
        else:
            mel = torch.empty(B, T, M, device=dev, dtype=f32)
            audio = torch.empty(B, 1, 64 * T, device=dev, dtype=f32)
            ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, T))
            _lib.check(lib.m2_inference_back(self.handle, B, S, T, front.data_ptr(), front.numel(), mel.data_ptr(),
                                             audio.data_ptr(), ws.data_ptr(), ws.numel(), st), "m2_inference_back")
        if T > cap or 2 * T < cap:
            # the exact T: the launch configurations chosen from the capacity
            # (e.g. the stage1 tail's strip length) are then those of T itself
            self._tcap[(B, S)] = T
        return mel, audio

    def inference_front(self, ids: Tensor, lengths: Optional[Tensor], scale: float) -> Tuple[Tuple, int]:
        """Front half of inference (m2_inference_front): encoder, durations,
        frame counts; returns (hand-off state, this batch's T_max) after the
        one host read.  The hand-off lives in this model's front buffer, so
        the matching inference_back must come before the next front call."""
        require_device(ids, lengths, what="M2TTSModel")
        ids = ids.to(torch.int64).contiguous()
        B, S = ids.shape
        lens = lengths.to(torch.int64).contiguous() if lengths is not None else None
        front = self._scratch("_front", self._size("m2_front_bytes", B, S))
        ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, 0))
        tmax = ctypes.c_int32(0)
        _lib.call("m2_inference_front", self.handle, ids.data_ptr(), None if lens is None else lens.data_ptr(), B, S,
                  float(scale), front.data_ptr(), front.numel(), ws.data_ptr(), ws.numel(), ctypes.byref(tmax),
                  stream_handle(self.device))
        return (B, S, front, ids, lens), int(tmax.value)

    def inference_back(self, state: Tuple, T: int) -> Tuple[Tensor, Tensor]:
        """Back half (m2_inference_back): expansion to exactly T frames (a
        batch-global T when sharded), mel decoder, vocoder."""
        B, S, front, _ids, _lens = state
        mel = torch.empty(B, T, self.M, device=self.device, dtype=torch.float32)
        audio = torch.empty(B, 1, 64 * T, device=self.device, dtype=torch.float32)
        ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, T))
        _lib.call("m2_inference_back", self.handle, B, S, T, front.data_ptr(), front.numel(), mel.data_ptr(),
                  audio.data_ptr(), ws.data_ptr(), ws.numel(), stream_handle(self.device))
        return mel, audio

    # ------------------------------------------------- device-side frame count
    def dev_supported(self, T_cap: int) -> bool:
        """True when the back half can take its frame count from the device
        at a capacity of T_cap frames (m2_inference_dev_supported)."""
        return T_cap > 0 and bool(_lib.load().m2_inference_dev_supported(self.handle, int(T_cap)))

    def inference_front_dev(self, ids: Tensor, lengths: Optional[Tensor], scale: float, tword: Tensor) -> Tuple:
        """Front half with no host read (m2_inference_front_dev): this shard's
        T_max goes to the device word tword[0] (int32, e.g. the payload of the
        ranks' all-reduce), stream-ordered.  Returns the hand-off state."""
        require_device(ids, lengths, tword, what="M2TTSModel")
        if tword.dtype != torch.int32 or not tword.is_contiguous():
            raise ValueError("inference_front_dev: tword must be a contiguous int32 device tensor")
        ids = ids.to(torch.int64).contiguous()
        B, S = ids.shape
        lens = lengths.to(torch.int64).contiguous() if lengths is not None else None
        front = self._scratch("_front", self._size("m2_front_bytes", B, S))
        ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, 0))
        _lib.call("m2_inference_front_dev", self.handle, ids.data_ptr(), None if lens is None else lens.data_ptr(),
                  B, S, float(scale), front.data_ptr(), front.numel(), ws.data_ptr(), ws.numel(), tword.data_ptr(),
                  stream_handle(self.device))
        return (B, S, front, ids, lens)

    def inference_back_dev(self, state: Tuple, T_cap: int, tword: Tensor, mel_out: Tensor,
                           audio_out: Tensor) -> None:
        """Back half for a capacity of T_cap frames taking T = max(1, tword[0])
        from the device (m2_inference_back_dev): mel [B,T,M] written at the
        start of mel_out (>= B*T_cap*M floats), audio [B,1,64T] at the start
        of audio_out (>= B*64*T_cap floats).  Nothing is written when
        T > T_cap (the caller then runs inference_back(T))."""
        B, S, front, _ids, _lens = state
        for t, n in ((mel_out, B * T_cap * self.M), (audio_out, B * 64 * T_cap)):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < n or t.data_ptr() % 16:
                raise ValueError("inference_back_dev: output buffers must be 16-B aligned contiguous float32 "
                                 "tensors of B*T_cap*M and B*64*T_cap elements")
        ws = self._scratch("_ws", self._size("m2_inference_workspace_bytes", B, S, T_cap))
        _lib.call("m2_inference_back_dev", self.handle, B, S, int(T_cap), tword.data_ptr(), front.data_ptr(),
                  front.numel(), mel_out.data_ptr(), audio_out.data_ptr(), ws.data_ptr(), ws.numel(),
                  stream_handle(self.device))

    def frames_wait(self) -> int:
        """T of this model's latest inference_back_dev call, as its first
        launch posted it (m2_frames_wait): blocks until that launch has run,
        not until the back half is done."""
        T = ctypes.c_int32(0)
        _lib.call("m2_frames_wait", self.handle, stream_handle(self.device), ctypes.byref(T))
        return int(T.value)

    # ------------------------------------------------------------------ vocoder modes
    def vocoder_select(self, path: int):
        """1 = exact-f32 MFMA kernels, 2 = split-f16 MFMA kernels (m2_vocoder_select)."""
        _lib.call("m2_vocoder_select", self.handle, int(path))

    def vocoder_path(self) -> int:
        return int(_lib.load().m2_vocoder_path(self.handle))

    def set_range_policy(self, policy: str):
        """What a non-finite split-path result does (m2_set_range_policy):
        "report" - the next call raises M2Error (M2_E_RANGE), check() reports
        it at once; "fallback" - a call whose audio is not finite is re-run on
        the exact-f32 kernels (on the device, no host wait, for the fused
        vocoders; otherwise after a stream synchronisation)."""
        if policy not in RANGE_POLICIES:
            raise ValueError(f"range policy {policy!r}: expected one of {sorted(RANGE_POLICIES)}")
        _lib.call("m2_set_range_policy", self.handle, RANGE_POLICIES[policy])

    def check(self) -> bool:
        """Synchronise the current stream; True if a split-path vocoder call
        since the last check produced non-finite audio (flag cleared)."""
        flagged = ctypes.c_int32(0)
        _lib.call("m2_model_check", self.handle, stream_handle(self.device), ctypes.byref(flagged))
        return bool(flagged.value)

    def set_chunking(self, chunk_frames: int):
        """Stream the vocoder in chunks of chunk_frames mel frames (0 = off)."""
        _lib.call("m2_vocoder_set_chunking", self.handle, int(chunk_frames))
        self._sizes.clear()  # workspace sizes depend on it
        self.chunk_frames = int(chunk_frames)

    def vocoder_stream(self, mel: Tensor, chunk_frames: int, layout_btm: bool = False):
        """Yield the audio of mel frames [f0, f0 + chunk_frames) as [B,1,64*n]
        tensors in order (m2_vocoder_chunk); concatenated they equal
        vocoder(mel) bit for bit."""
        mel = f32c(mel)
        require_device(mel, what="SimpleVocoder")
        B = mel.shape[0]
        T = mel.shape[1] if layout_btm else mel.shape[2]
        if chunk_frames <= 0:
            raise ValueError("chunk_frames must be positive")
        ws = self._scratch("_ws_chunk", self._size("m2_vocoder_chunk_workspace_bytes", B, T, chunk_frames))
        st = stream_handle(self.device)
        for f0 in range(0, T, chunk_frames):
            f1 = min(T, f0 + chunk_frames)
            out = torch.empty(B, 1, 64 * (f1 - f0), device=self.device, dtype=torch.float32)
            _lib.call("m2_vocoder_chunk", self.handle, mel.data_ptr(), 1 if layout_btm else 0, B, T, f0, f1,
                      out.data_ptr(), ws.data_ptr(), ws.numel(), st)
            yield out

    # ------------------------------------------------------------------ stages
    def text_encoder(self, ids: Tensor, lengths: Optional[Tensor]):
        require_device(ids, lengths, what="TextEncoder")
        ids = ids.to(torch.int64).contiguous()
        B, S = ids.shape
        if S > self.cfg.max_positions:
            raise RuntimeError(f"sequence length {S} exceeds the positional table ({self.cfg.max_positions})")
        lens = lengths.to(torch.int64).contiguous() if lengths is not None else None
        enc = torch.empty(B, S, self.H, device=self.device, dtype=torch.float32)
        mask = torch.empty(B, S, device=self.device, dtype=torch.bool) if lens is not None else None
        ws = self.workspace(B, S, 0)
        _lib.call("m2_text_encoder", self.handle, ids.data_ptr(), None if lens is None else lens.data_ptr(), B, S,
                  enc.data_ptr(), None if mask is None else mask.data_ptr(), ws.data_ptr(), ws.numel(),
                  stream_handle(self.device))
        return enc, mask

    def duration(self, enc: Tensor) -> Tensor:
        enc = f32c(enc)
        B, S, _ = enc.shape
        dur = torch.empty(B, S, device=self.device, dtype=torch.float32)
        _lib.call("m2_duration_predictor", self.handle, enc.data_ptr(), B, S, dur.data_ptr(), None, 0,
                  stream_handle(self.device))
        return dur

    def decoder(self, x: Tensor) -> Tensor:
        x = f32c(x)
        B, T, _ = x.shape
        mel = torch.empty(B, T, self.M, device=self.device, dtype=torch.float32)
        ws = self.workspace(B, 0, T)
        _lib.call("m2_mel_decoder", self.handle, x.data_ptr(), B, T, mel.data_ptr(), ws.data_ptr(), ws.numel(),
                  stream_handle(self.device))
        return mel

    def vocoder(self, mel: Tensor, layout_btm: bool) -> Tensor:
        """mel [B,M,T] (layout_btm False) or [B,T,M] (True) -> audio [B,1,64T]."""
        mel = f32c(mel)
        B = mel.shape[0]
        T = mel.shape[1] if layout_btm else mel.shape[2]
        audio = torch.empty(B, 1, 64 * T, device=self.device, dtype=torch.float32)
        ws = self.workspace(B, 0, T)
        _lib.call("m2_vocoder", self.handle, mel.data_ptr(), 1 if layout_btm else 0, B, T, audio.data_ptr(),
                  ws.data_ptr(), ws.numel(), stream_handle(self.device))
        return audio

    def resblock(self, k: int, x: Tensor) -> Tensor:
        x = f32c(x)
        B, _, L = x.shape
        y = torch.empty_like(x)
        tmp = torch.empty_like(x)
        _lib.call("m2_vocoder_resblock", self.handle, k, x.data_ptr(), B, L, y.data_ptr(), tmp.data_ptr(),
                  stream_handle(self.device))
        return y

    def upsample(self, k: int, x: Tensor, rate: int) -> Tensor:
        x = f32c(x)
        B, C, L = x.shape
        y = torch.empty(B, C // 2, L * rate, device=self.device, dtype=torch.float32)
        _lib.call("m2_vocoder_upsample", self.handle, k, x.data_ptr(), B, L, y.data_ptr(), stream_handle(self.device))
        return y


RANGE_POLICIES = {"report": 0, "fallback": 1}


def default_range_policy() -> str:
    """The split-f16 range policy a new handle gets: "fallback" (never a
    non-finite result for finite inputs the exact-f32 path handles), unless
    M2_RANGE_POLICY names another one."""
    env = os.environ.get("M2_RANGE_POLICY")
    if env is None or env == "":
        return "fallback"
    if env not in RANGE_POLICIES:
        raise ValueError(f"M2_RANGE_POLICY={env!r}: expected one of {sorted(RANGE_POLICIES)}")
    return env


class HandleCache:
    """Per-device HipModel for one nn.Module, rebuilt when its weights change.
    ``lane`` > 0 gives further handles of the same weights (one per stream of a
    pipelined caller: a handle's device state is ordered on one stream)."""

    def __init__(self):
        self._entries: Dict[Tuple[torch.device, int], Tuple[Tuple, HipModel]] = {}

    def get(self, module: torch.nn.Module, cfg: _lib.M2Config, device: torch.device, lane: int = 0) -> HipModel:
        key = state_key(module)
        ent = self._entries.get((device, lane))
        if ent is not None and ent[0] == key:
            return ent[1]
        hm = HipModel(module.state_dict(), cfg, device)
        # per-model vocoder modes survive a rebuild (weights reloaded, .to())
        chunk = module.__dict__.get("_m2_chunk_frames", 0)
        if chunk:
            hm.set_chunking(chunk)
        path = module.__dict__.get("_m2_voc_path")
        if path:
            hm.vocoder_select(path)
        hm.set_range_policy(module.__dict__.get("_m2_range_policy") or default_range_policy())
        self._entries[(device, lane)] = (key, hm)
        return hm

    def handles(self):
        return [hm for _, hm in self._entries.values()]

    def clear(self):
        self._entries.clear()
