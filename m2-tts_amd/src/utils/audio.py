"""Audio output for the synthesis CLI.

``save_audio`` replaces the reference's soundfile call (src/utils/audio.py:154-180,
``sf.write`` with the WAV default subtype PCM_16): mono 16-bit PCM RIFF/WAVE,
float samples converted as libsndfile does for normalised floats,
``lrintf(x * 32767)`` (round half to even), here with explicit clipping to the
int16 range.  The reference's librosa feature extraction / Griffin-Lim
(audio.py:45-151) is training-side and out of scope.
"""
from __future__ import annotations

import logging
import wave
from pathlib import Path
from typing import Tuple, Union

import numpy as np
import torch

logger = logging.getLogger(__name__)


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
