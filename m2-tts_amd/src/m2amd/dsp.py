"""Mel features and Griffin-Lim on the GPU (C ABI m2_dsp_*, csrc/audio_dsp.hip).

The reference's src/utils/audio.py:45-151 runs librosa on the CPU;
``Dsp`` runs the same algorithms on a ROCm device, batched over utterances
(tensors [B, L] of audio, [B, n_mels, T] of mel).  Like the rest of the
product path there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
import weakref
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from .ops import require_device, stream_handle

Tensor = torch.Tensor


class Dsp:
    """Tables for one (sample_rate, n_fft, hop, win_length, n_mels, fmin, fmax) on one device."""

    def __init__(self, sample_rate=22050, n_fft=1024, hop_length=256, win_length=1024, n_mels=64, fmin=0.0,
                 fmax=None, device=None):
        lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        fmax = sample_rate / 2.0 if fmax is None else float(fmax)
        self.sample_rate, self.n_fft, self.hop, self.win_length, self.n_mels = (sample_rate, n_fft, hop_length,
                                                                               win_length, n_mels)
        self.F = n_fft // 2 + 1
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.m2_dsp_create(sample_rate, n_fft, hop_length, win_length, n_mels, float(fmin), fmax,
                                         stream_handle(self.device), ctypes.byref(h)), "m2_dsp_create")
        self.handle = h
        self._ws: Optional[Tensor] = None
        self._finalizer = weakref.finalize(self, lib.m2_dsp_destroy, h)

    def frames(self, L: int) -> int:
        return 1 + L // self.hop

    def _audio(self, audio: Tensor) -> Tensor:
        require_device(audio, what="m2 dsp")
        if audio.dtype != torch.float32:
            audio = audio.float()
        return audio.reshape(-1, audio.shape[-1]).contiguous()

    def stft(self, audio: Tensor) -> Tensor:
        """librosa.stft(center=True, pad_mode='constant', window='hann') -> complex64 [B, F, T]."""
        y = self._audio(audio)
        B, L = y.shape
        out = torch.empty(B, self.frames(L), self.F, 2, device=y.device, dtype=torch.float32)
        _lib.call("m2_stft", self.handle, y.data_ptr(), B, L, out.data_ptr(), stream_handle(y.device))
        return torch.view_as_complex(out).transpose(1, 2)

    def mel_spectrogram(self, audio: Tensor) -> Tensor:
        """compute_mel_spectrogram (audio.py:45-98) per utterance -> [B, n_mels, T] in [-1, 1]."""
        y = self._audio(audio)
        B, L = y.shape
        out = torch.empty(B, self.n_mels, self.frames(L), device=y.device, dtype=torch.float32)
        _lib.call("m2_mel_spectrogram", self.handle, y.data_ptr(), B, L, out.data_ptr(), stream_handle(y.device))
        return out

    def mel_to_magnitude(self, mel: Tensor, nnls_iters: int = 200) -> Tensor:
        """librosa.feature.inverse.mel_to_stft of (mel + 1) / 2 in dB (audio.py:128-132)
        -> magnitudes [B, F, T]: librosa.util.nnls's result, its L-BFGS-B's
        start max(0, pinv(W) M) where its convergence test passes there (every
        mel in the normalised range); ``nnls_iters`` projected-gradient steps
        per frame for a block that would iterate (m2_mel_to_magnitude)."""
        require_device(mel, what="m2 mel_to_magnitude")
        m = mel.float().reshape(-1, self.n_mels, mel.shape[-1]).contiguous()
        B, T = m.shape[0], m.shape[2]
        out = torch.empty(B, T, self.F, device=m.device, dtype=torch.float32)
        n = int(_lib.load().m2_mel_to_magnitude_workspace_bytes(self.handle, B, T))
        ws = torch.empty(max(n, 1), dtype=torch.uint8, device=m.device)
        _lib.call("m2_mel_to_magnitude", self.handle, m.data_ptr(), B, T, int(nnls_iters), out.data_ptr(),
                  ws.data_ptr(), ws.numel(), stream_handle(m.device))
        return out.transpose(1, 2)

    def random_angles(self, B: int, T: int, seed: Optional[int] = None) -> Tensor:
        """librosa griffinlim(init='random'): unit phases exp(2 pi i U[0, 1)), [B, T, F] complex64."""
        g = torch.Generator(device=self.device)
        if seed is not None:
            g.manual_seed(seed)
        else:
            g.seed()
        ph = torch.rand(B, T, self.F, generator=g, device=self.device, dtype=torch.float64) * (2 * math.pi)
        return torch.polar(torch.ones_like(ph), ph).to(torch.complex64)

    def griffin_lim(self, mel: Optional[Tensor] = None, mag: Optional[Tensor] = None,
                    init_angles: Optional[Tensor] = None, n_iter: int = 32, momentum: float = 0.99,
                    nnls_iters: int = 200, seed: Optional[int] = None) -> Tensor:
        """mel_to_audio (audio.py:101-151) from mel [B, n_mels, T] (normalised dB), or
        the bare griffinlim from magnitudes mag [B, F, T]; -> audio [B, hop (T - 1)]."""
        src = mel if mel is not None else mag
        require_device(src, what="m2 griffin_lim")
        if mel is not None:
            m = mel.float().reshape(-1, self.n_mels, mel.shape[-1]).contiguous()
            B, T = m.shape[0], m.shape[2]
            mg = None
        else:
            mg = mag.float().reshape(-1, self.F, mag.shape[-1]).transpose(1, 2).contiguous()
            B, T = mg.shape[0], mg.shape[1]
            m = None
        if init_angles is None:
            init_angles = self.random_angles(B, T, seed)
        ang = torch.view_as_real(init_angles.to(torch.complex64).reshape(B, T, self.F).contiguous()).contiguous()
        out = torch.empty(B, self.hop * (T - 1), device=src.device, dtype=torch.float32)
        need = int(_lib.load().m2_griffin_lim_workspace_bytes(self.handle, B, T))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=src.device)
        _lib.call("m2_griffin_lim", self.handle, None if m is None else m.data_ptr(),
                  None if mg is None else mg.data_ptr(), ang.data_ptr(), B, T, int(n_iter), float(momentum),
                  int(nnls_iters), out.data_ptr(), self._ws.data_ptr(), self._ws.numel(), stream_handle(src.device))
        return out


_CACHE: Dict[Tuple, Dsp] = {}


def get_dsp(sample_rate=22050, n_fft=1024, hop_length=256, win_length=1024, n_mels=64, fmin=0.0, fmax=None,
            device=None) -> Dsp:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (sample_rate, n_fft, hop_length, win_length, n_mels, float(fmin), fmax, dev)
    d = _CACHE.get(key)
    if d is None:
        d = _CACHE[key] = Dsp(sample_rate, n_fft, hop_length, win_length, n_mels, fmin, fmax, dev)
    return d
