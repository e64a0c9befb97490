"""Audio I/O and features (reference src/utils/audio.py).

``save_audio`` replaces the reference's soundfile call (src/utils/audio.py:154-180,
``sf.write`` with the WAV default subtype PCM_16): mono 16-bit PCM RIFF/WAVE,
float samples converted as libsndfile does for normalised floats,
``lrintf(x * 32767)`` (round half to even), here with explicit clipping to the
int16 range.

``compute_mel_spectrogram`` / ``mel_to_audio`` / ``AudioProcessor``
(audio.py:45-151, 183-257) keep the reference's signatures and return numpy
float32 like it does, but compute on the GPU (m2amd.dsp: STFT, mel filters,
power_to_db, NNLS, Griffin-Lim kernels) instead of librosa, which this image
does not have.  ``mel_to_audio``'s random phase start (librosa
init='random') takes an optional ``seed``.
"""
from __future__ import annotations

import logging
import wave
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch

logger = logging.getLogger(__name__)


def _on_gpu(x) -> torch.Tensor:
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    if t.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("m2-tts_amd audio features run on a ROCm GPU; none is visible (no CPU path)")
        t = t.to("cuda")
    return t.float()


def compute_mel_spectrogram(audio, sample_rate: int = 22050, n_fft: int = 1024, hop_length: int = 256,
                            win_length: int = 1024, n_mels: int = 64, fmin: int = 0,
                            fmax: Optional[int] = None) -> np.ndarray:
    """Log mel spectrogram normalised to [-1, 1] (reference audio.py:45-98):
    [n_mels, frames] float32 for a 1-D signal, [B, n_mels, frames] for [B, L]."""
    from m2amd.dsp import get_dsp
    if fmax is None:
        fmax = sample_rate // 2
    y = _on_gpu(audio)
    d = get_dsp(sample_rate, n_fft, hop_length, win_length, n_mels, fmin, fmax, y.device)
    mel = d.mel_spectrogram(y)
    out = mel.cpu().numpy()
    return out[0] if y.dim() == 1 else out


def mel_to_audio(mel_spec, sample_rate: int = 22050, n_fft: int = 1024, hop_length: int = 256,
                 win_length: int = 1024, n_iter: int = 32, seed: Optional[int] = None,
                 init_angles: Optional[torch.Tensor] = None) -> np.ndarray:
    """Griffin-Lim reconstruction of a normalised log mel (reference
    audio.py:101-151): [n_mels, T] -> [hop (T - 1)] float32, peak-normalised."""
    from m2amd.dsp import get_dsp
    m = _on_gpu(mel_spec)
    single = m.dim() == 2
    m = m.reshape(-1, m.shape[-2], m.shape[-1])
    d = get_dsp(sample_rate, n_fft, hop_length, win_length, m.shape[1], 0.0, sample_rate / 2.0, m.device)
    audio = d.griffin_lim(mel=m, init_angles=init_angles, n_iter=n_iter, seed=seed).cpu().numpy()
    return audio[0] if single else audio


class AudioProcessor:
    """Reference audio.py:183-257: the feature settings of the trainers."""

    def __init__(self, sample_rate: int = 22050, n_fft: int = 1024, hop_length: int = 256, win_length: int = 1024,
                 n_mels: int = 64, fmin: int = 0, fmax: Optional[int] = None):
        self.sample_rate, self.n_fft, self.hop_length, self.win_length = sample_rate, n_fft, hop_length, win_length
        self.n_mels, self.fmin = n_mels, fmin
        self.fmax = fmax if fmax is not None else sample_rate // 2

    def compute_mel_spectrogram(self, audio) -> np.ndarray:
        return compute_mel_spectrogram(audio, self.sample_rate, self.n_fft, self.hop_length, self.win_length,
                                       self.n_mels, self.fmin, self.fmax)

    def process_file(self, audio_path: Union[str, Path]) -> Tuple[np.ndarray, np.ndarray]:
        audio, sr = load_audio_pcm16(audio_path)
        if sr != self.sample_rate:
            raise ValueError(f"{audio_path}: {sr} Hz, expected {self.sample_rate} (no resampler in this build)")
        m = np.max(np.abs(audio))
        audio = audio / m if m > 0 else audio  # load_audio(normalize=True), audio.py:36-37
        return audio, self.compute_mel_spectrogram(audio)

    def mel_to_audio(self, mel_spec, seed: Optional[int] = None) -> np.ndarray:
        return mel_to_audio(mel_spec, self.sample_rate, self.n_fft, self.hop_length, self.win_length, seed=seed)


def float_to_pcm16(audio: np.ndarray) -> np.ndarray:
    x = np.asarray(audio, dtype=np.float32) * np.float32(32767.0)
    return np.clip(np.rint(x), -32768, 32767).astype("<i2")


def save_audio(audio: Union[np.ndarray, torch.Tensor], output_path: Union[str, Path],
               sample_rate: int = 22050) -> None:
    if isinstance(audio, torch.Tensor):
        audio = audio.detach().cpu().numpy()
    audio = np.asarray(audio)
    if audio.ndim > 1:
        audio = audio.squeeze()
    pcm = float_to_pcm16(audio.reshape(-1))
    with wave.open(str(output_path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sample_rate))
        w.writeframes(pcm.tobytes())
    logger.debug(f"Saved audio to {output_path}")


def load_audio_pcm16(path: Union[str, Path]) -> Tuple[np.ndarray, int]:
    """Read a mono PCM16 WAV back as float32 in [-1, 1) (samples / 32768) and its rate."""
    with wave.open(str(path), "rb") as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1, "mono PCM16 only"
        data = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")
        return data.astype(np.float32) / 32768.0, w.getframerate()
