"""ctypes binding of the gfx950 C-ABI library (include/m2tts_hip.h).

The library is built in-tree by ``make -C m2-tts_amd/csrc`` (or
``__graft_entry__.build()``) into ``m2amd/libm2tts_hip.so``.  There is no CPU
fallback: if the library is missing or cannot be loaded every call raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("M2TTS_HIP_LIB", _HERE / "libm2tts_hip.so"))

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_size = ctypes.c_size_t
c_vp = ctypes.c_void_p


class M2Config(ctypes.Structure):
    """Mirror of ``m2_config`` (the 8 M2TTSModel hyper-parameters that shape weights)."""
    _fields_ = [("vocab_size", c_i32), ("hidden_dim", c_i32), ("mel_channels", c_i32),
                ("text_encoder_layers", c_i32), ("decoder_layers", c_i32), ("num_heads", c_i32),
                ("vocoder_channels", c_i32), ("max_positions", c_i32)]


# name -> (restype, argtypes)
_SIGNATURES = {
    "m2_abi_version": (c_i32, []),
    "m2_last_error": (ctypes.c_char_p, []),
    "m2_weight_count": (c_i32, [ctypes.POINTER(M2Config)]),
    "m2_weight_name": (c_i32, [ctypes.POINTER(M2Config), c_i32, ctypes.c_char_p, c_i32]),
    "m2_weight_numel": (c_i64, [ctypes.POINTER(M2Config), c_i32]),
    "m2_model_create": (c_i32, [ctypes.POINTER(M2Config), ctypes.POINTER(c_vp), c_i32, c_vp, ctypes.POINTER(c_vp)]),
    "m2_model_destroy": (c_i32, [c_vp]),
    "m2_reload_switches": (None, []),
    "m2_model_config": (c_i32, [c_vp, ctypes.POINTER(M2Config)]),
    "m2_workspace_bytes": (c_size, [c_vp, c_i32, c_i32, c_i32]),
    "m2_text_encoder": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_size, c_vp]),
    "m2_duration_predictor": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_length_regulator_count": (c_i32, [c_vp, c_i32, c_f32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "m2_length_regulator_count_sync": (c_i32, [c_vp, c_i32, c_f32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "m2_length_regulator_expand": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_mel_decoder": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_vocoder": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_vocoder_set_chunking": (c_i32, [c_vp, c_i32]),
    "m2_vocoder_halo_frames": (c_i32, []),
    "m2_vocoder_chunk": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_vocoder_chunk_workspace_bytes": (c_size, [c_vp, c_i32, c_i32, c_i32]),
    "m2_vocoder_select": (c_i32, [c_vp, c_i32]),
    "m2_set_range_policy": (c_i32, [c_vp, c_i32]),
    "m2_model_check": (c_i32, [c_vp, c_vp, ctypes.POINTER(c_i32)]),
    "m2_vocoder_resblock": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "m2_vocoder_upsample": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "m2_conv1d": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_conv1d_ex": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                             c_i32, c_vp, c_vp]),
    "m2_conv_transpose1d": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_linear": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_layer_norm": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "m2_attention": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_embed_positional": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f32, c_vp, c_vp]),
    "m2_add_positional": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "m2_profile_enable": (c_i32, [c_vp, c_i32]),
    "m2_profile_read": (c_i32, [c_vp, ctypes.POINTER(c_f32), c_i32, ctypes.POINTER(c_i32)]),
    "m2_profile_disable": (c_i32, [c_vp]),
    "m2_profile_kernel_count": (c_i32, []),
    "m2_profile_kernel_name": (ctypes.c_char_p, [c_i32]),
    "m2_profile_kernel_name_for": (ctypes.c_char_p, [c_vp, c_i32]),
    "m2_profile_select": (c_i32, [c_vp, ctypes.c_uint32]),
    "m2_profile_stride": (c_i32, [c_vp, c_i32]),
    "m2_vocoder_path": (c_i32, [c_vp]),
    "m2_dsp_create": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_f32, c_vp, ctypes.POINTER(c_vp)]),
    "m2_dsp_destroy": (c_i32, [c_vp]),
    "m2_dsp_frames": (c_i32, [c_vp, c_i32]),
    "m2_stft": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "m2_mel_spectrogram": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "m2_griffin_lim_workspace_bytes": (c_size, [c_vp, c_i32, c_i32]),
    "m2_mel_to_magnitude_workspace_bytes": (c_size, [c_vp, c_i32, c_i32]),
    "m2_mel_to_magnitude": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_griffin_lim": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_f32, c_i32, c_vp, c_vp, c_size, c_vp]),
    "m2_transformer_path": (c_i32, [c_vp]),
    "m2_front_bytes": (c_size, [c_vp, c_i32, c_i32]),
    "m2_inference_workspace_bytes": (c_size, [c_vp, c_i32, c_i32, c_i32]),
    "m2_inference_front": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_size, c_vp, c_size, c_vp, c_vp]),
    "m2_inference": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_size, c_vp, c_size, c_vp, c_size, c_vp,
                             c_size, c_vp, c_vp, c_vp]),
    "m2_inference_back": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_size, c_vp, c_vp, c_vp, c_size, c_vp]),
    "m2_inference_dev_supported": (c_i32, [c_vp, c_i32]),
    "m2_frames_wait": (c_i32, [c_vp, c_vp, c_vp]),
    "m2_inference_front_dev": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i32, c_f32, c_vp, c_size, c_vp, c_size, c_vp,
                                       c_vp]),
    "m2_inference_back_dev": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_size, c_vp, c_vp, c_vp, c_size,
                                      c_vp]),
}

# act codes (m2_common.h Act)
ACT_NONE, ACT_LEAKY, ACT_TANH, ACT_RELU, ACT_SOFTPLUS = 0, 1, 2, 3, 4

_lib = None
_load_error = None


class M2Error(RuntimeError):
    pass


def load(path: Path = None):
    """Load (once) and return the library; raises M2Error if it cannot be loaded."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise M2Error(f"m2-tts_amd HIP library not found at {p}; build it with "
                      f"`make -C m2-tts_amd/csrc` (or __graft_entry__.build()). "
                      f"There is no CPU fallback.")
    try:
        lib = ctypes.CDLL(str(p))
    except OSError as e:  # pragma: no cover - depends on the ROCm install
        _load_error = e
        raise M2Error(f"cannot load {p}: {e}") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def reload_switches():
    """Re-read the M2_* developer switches into the library's table (it reads
    them at load and at every model-handle creation, never per call)."""
    load().m2_reload_switches()


def exported_symbols():
    return list(_SIGNATURES)


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = _lib.m2_last_error().decode(errors="replace") if _lib is not None else ""
        raise M2Error(f"{what or 'm2 call'} failed (status {rc}): {msg}")


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
