"""Drop-in ``models.tts_model`` for MI355X.

Same classes, constructor signatures, submodule/parameter names (so
reference checkpoints load unchanged), return types and shapes as the
reference ``src/models/tts_model.py``; the forward path runs on gfx950 HIP
kernels through the C ABI in ``include/m2tts_hip.h``:

* ``M2TTSModel.forward`` / ``inference`` use one packed model handle
  (``m2amd.runtime.HipModel``): one C call per stage, the length regulator as
  a GPU scan + gather with a single device->host read of the frame count.
* The stage modules (``text_encoder``, ``duration_predictor``,
  ``length_regulator``, ``decoder``, ``vocoder``) may be called directly, as
  the reference's callers do; inside an M2TTSModel they use the owner's
  handle, standalone they compose the per-op kernels of ``m2amd.ops``.

Differences from the reference that do not change results:
* ``inference`` runs the vocoder once (the reference runs it inside
  ``forward`` and again afterwards, tts_model.py:388-391 vs 435-436, on the
  same mel) and skips the unscaled decoder pass when duration_scale != 1.
* Eval-mode math only; see models/components.py.
"""
from __future__ import annotations

import logging
import weakref
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn as nn

from m2amd import ops, runtime
from m2amd.runtime import HandleCache, make_config

from .components import (LightweightResBlock, PositionalEncoding, TransformerEncoderLayer, VariancePredictor,
                         count_parameters, create_padding_mask, initialize_weights)

logger = logging.getLogger(__name__)
Tensor = torch.Tensor

UPSAMPLE_RATES = (4, 4, 2, 2)   # reference tts_model.py:244
VOCODER_HALO = 3                # receptive field of one audio sample, mel frames per side (m2_vocoder_halo_frames)
_HANDLES: "weakref.WeakKeyDictionary[nn.Module, HandleCache]" = weakref.WeakKeyDictionary()


def _owner_handle(stage: nn.Module, attr: str, device: torch.device):
    """The owning M2TTSModel's packed handle if `stage` is still its `attr`."""
    ref = getattr(stage, "_m2_owner", None)
    owner = ref() if ref is not None else None
    if owner is None or getattr(owner, attr, None) is not stage:
        return None
    return owner._hip(device)


class TextEncoder(nn.Module):
    """Embedding*sqrt(H) + positional table, pre-LN transformer layers with a
    key-padding mask, final LayerNorm (reference tts_model.py:19-89)."""

    def __init__(self, vocab_size: int = 256, hidden_dim: int = 64, num_layers: int = 2, num_heads: int = 2,
                 dropout: float = 0.1, max_seq_len: int = 1000):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.embedding = nn.Embedding(vocab_size, hidden_dim)
        self.pos_encoding = PositionalEncoding(hidden_dim, max_seq_len)
        self.layers = nn.ModuleList(
            [TransformerEncoderLayer(hidden_dim=hidden_dim, num_heads=num_heads, ffn_dim=hidden_dim * 2, dropout=dropout)
             for _ in range(num_layers)])
        self.norm = nn.LayerNorm(hidden_dim)
        self.dropout = nn.Dropout(dropout)
        self.apply(initialize_weights)

    def forward(self, phoneme_ids: Tensor, lengths: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
        hm = _owner_handle(self, "text_encoder", phoneme_ids.device)
        if hm is not None:
            return hm.text_encoder(phoneme_ids, lengths)
        ops.require_device(phoneme_ids, self.embedding.weight, what="TextEncoder")
        _, s = phoneme_ids.shape
        mask = create_padding_mask(lengths, s) if lengths is not None else None
        x = ops.embed_positional(phoneme_ids, self.embedding.weight, self.pos_encoding.pe[0, :s],
                                 ops.sqrt_hidden(self.hidden_dim))
        for layer in self.layers:
            x = layer(x, mask)
        return ops.layer_norm(x, self.norm.weight, self.norm.bias), mask


class DurationPredictor(nn.Module):
    """softplus(VariancePredictor(enc^T)) -> [B, S] (reference tts_model.py:92-117)."""

    def __init__(self, hidden_dim: int = 64, kernel_size: int = 3, dropout: float = 0.1):
        super().__init__()
        self.predictor = VariancePredictor(hidden_dim, kernel_size, dropout)

    def forward(self, encoder_output: Tensor) -> Tensor:
        hm = _owner_handle(self, "duration_predictor", encoder_output.device)
        if hm is not None:
            return hm.duration(encoder_output)
        x = encoder_output.transpose(1, 2).contiguous()
        return self.predictor(x, _act=ops.ACT_SOFTPLUS).squeeze(1)


class LengthRegulator(nn.Module):
    """Repeat each phoneme row int(duration) times, pad/truncate to the batch
    maximum or ``max_length`` (reference tts_model.py:120-178).  GPU scan +
    gather; truncation toward zero and the all-zero-durations case (one zero
    frame) follow the reference."""

    def forward(self, encoder_output: Tensor, durations: Tensor, max_length: Optional[int] = None) -> Tensor:
        return ops.regulate(encoder_output, durations, max_length)


class MelDecoder(nn.Module):
    """Unmasked pre-LN transformer over frames -> LayerNorm -> Linear(H, M)
    (reference tts_model.py:181-228)."""

    def __init__(self, hidden_dim: int = 64, mel_channels: int = 64, num_layers: int = 2, num_heads: int = 2,
                 dropout: float = 0.1):
        super().__init__()
        self.layers = nn.ModuleList(
            [TransformerEncoderLayer(hidden_dim=hidden_dim, num_heads=num_heads, ffn_dim=hidden_dim * 2, dropout=dropout)
             for _ in range(num_layers)])
        self.norm = nn.LayerNorm(hidden_dim)
        self.mel_projection = nn.Linear(hidden_dim, mel_channels)
        self.apply(initialize_weights)

    def forward(self, x: Tensor) -> Tensor:
        hm = _owner_handle(self, "decoder", x.device)
        if hm is not None:
            return hm.decoder(x)
        for layer in self.layers:
            x = layer(x)
        return ops.linear(x, self.mel_projection.weight, self.mel_projection.bias,
                          ln=(self.norm.weight, self.norm.bias))


class SimpleVocoder(nn.Module):
    """input_conv -> 4 x [ConvT(k=2r, s=r, p=r/2) -> leaky(0.1) -> resblock]
    -> output_conv -> tanh; 64 samples per mel frame (reference
    tts_model.py:231-297).  ``kernel_size``/``n_layers`` are accepted and, as
    in the reference, do not change the upsampling schedule."""

    def __init__(self, mel_channels: int = 64, hidden_channels: int = 128, kernel_size: int = 3, n_layers: int = 4):
        super().__init__()
        self.input_conv = nn.Conv1d(mel_channels, hidden_channels, kernel_size, padding=kernel_size // 2)
        self.upsamples = nn.ModuleList()
        self.resblocks = nn.ModuleList()
        ch = hidden_channels
        for r in UPSAMPLE_RATES:
            self.upsamples.append(nn.ConvTranspose1d(ch, ch // 2, kernel_size=2 * r, stride=r, padding=r // 2))
            ch //= 2
            self.resblocks.append(LightweightResBlock(ch, kernel_size))
        self.output_conv = nn.Conv1d(ch, 1, kernel_size, padding=kernel_size // 2)
        self.apply(initialize_weights)

    def forward(self, mel: Tensor) -> Tensor:
        hm = _owner_handle(self, "vocoder", mel.device)
        if hm is not None:
            return hm.vocoder(mel, layout_btm=False)
        # any kernel_size: input / output convs with padding k//2 and the
        # resblocks' general form (an even k changes lengths and the resblock
        # residual fails, as in the reference)
        x = ops.conv1d(mel, self.input_conv.weight, self.input_conv.bias, padding=self.input_conv.padding[0])
        for r, up, rb in zip(UPSAMPLE_RATES, self.upsamples, self.resblocks):
            x = ops.conv_transpose1d(x, up.weight, up.bias, r, act=ops.ACT_LEAKY)
            x = rb(x)
        return ops.conv1d(x, self.output_conv.weight, self.output_conv.bias, act=ops.ACT_TANH,
                          padding=self.output_conv.padding[0])

    def stream(self, mel: Tensor, chunk_frames: int = 256):
        """Yield the audio of mel [B, M, T] chunk by chunk ([B, 1, 64 n] for
        n <= chunk_frames frames each), for playback while later chunks are
        still being computed.  Each chunk is computed over its window widened
        by the vocoder's receptive field (VOCODER_HALO frames per side): the
        chunks concatenate to exactly forward(mel) (the reference's one-shot
        output, tts_model.py:279-297)."""
        if chunk_frames <= 0:
            raise ValueError("chunk_frames must be positive")
        hm = _owner_handle(self, "vocoder", mel.device)
        if hm is not None:
            yield from hm.vocoder_stream(mel, chunk_frames)
            return
        T = mel.shape[2]
        for f0 in range(0, T, chunk_frames):
            f1 = min(T, f0 + chunk_frames)
            w0, w1 = max(0, f0 - VOCODER_HALO), min(T, f1 + VOCODER_HALO)
            yield self.forward(mel[:, :, w0:w1])[:, :, 64 * (f0 - w0):64 * (f1 - w0)].contiguous()


class M2TTSModel(nn.Module):
    """Text encoder -> duration predictor -> length regulator -> mel decoder ->
    vocoder (reference tts_model.py:300-459)."""

    def __init__(self, vocab_size: int = 256, hidden_dim: int = 64, mel_channels: int = 64,
                 text_encoder_layers: int = 2, decoder_layers: int = 2, num_heads: int = 2, dropout: float = 0.1,
                 vocoder_channels: int = 128):
        super().__init__()
        self.text_encoder = TextEncoder(vocab_size=vocab_size, hidden_dim=hidden_dim, num_layers=text_encoder_layers,
                                        num_heads=num_heads, dropout=dropout)
        self.duration_predictor = DurationPredictor(hidden_dim=hidden_dim, dropout=dropout)
        self.length_regulator = LengthRegulator()
        self.decoder = MelDecoder(hidden_dim=hidden_dim, mel_channels=mel_channels, num_layers=decoder_layers,
                                  num_heads=num_heads, dropout=dropout)
        self.vocoder = SimpleVocoder(mel_channels=mel_channels, hidden_channels=vocoder_channels)
        self._m2_cfg = make_config(vocab_size, hidden_dim, mel_channels, text_encoder_layers, decoder_layers,
                                   num_heads, vocoder_channels, self.text_encoder.pos_encoding.pe.shape[1])
        me = weakref.ref(self)
        for stage in (self.text_encoder, self.duration_predictor, self.decoder, self.vocoder):
            object.__setattr__(stage, "_m2_owner", me)
        total, trainable = count_parameters(self)
        logger.info(f"M2TTSModel: {total:,} parameters ({trainable:,} trainable), "
                    f"{total * 4 / (1024 * 1024):.1f} MB fp32")

    # -------------------------------------------------------------- handle
    def _eval_if_training(self):
        """self.eval() (tts_model.py:404) without the recursive train(False)
        walk when every module is already in eval mode (~35 us of host time per
        call at stage1, more than the length regulator's GPU time)."""
        mods = self.__dict__.get("_m2_modules")
        if mods is None or mods[0] != runtime._GEN[0]:
            mods = (runtime._GEN[0], list(self.modules()))
            self.__dict__["_m2_modules"] = mods
        for mod in mods[1]:
            if mod.training:
                self.eval()
                return

    def _hip(self, device: torch.device, lane: int = 0):
        cache = _HANDLES.get(self)
        if cache is None:
            cache = HandleCache()
            _HANDLES[self] = cache
        return cache.get(self, self._m2_cfg, device, lane)

    def set_vocoder_chunking(self, chunk_frames: int = 256):
        """Stream the vocoder in chunks of ``chunk_frames`` mel frames inside
        forward/inference/vocoder (0 = whole utterance).  Each chunk is
        computed over a window widened by the vocoder's 3-frame receptive
        field, so the audio is bit-identical to the unchunked call; the
        workspace holds one window instead of the whole utterance."""
        self.__dict__["_m2_chunk_frames"] = int(chunk_frames)
        cache = _HANDLES.get(self)
        for hm in (cache.handles() if cache is not None else []):
            hm.set_chunking(chunk_frames)

    def set_range_policy(self, policy: str = "fallback"):
        """The split-f16 vocoder carries fp32 values as f16 hi/lo pairs; an
        input or activation of magnitude >= 65520 turns its audio non-finite
        (never silently wrong).  "fallback" (the default, also without this
        call; M2_RANGE_POLICY overrides it for new handles): the non-finite
        part of a vocoder call is recomputed in fp32 on the device before
        anything behind it on the stream runs, so a call never returns
        non-finite audio for an input the reference's fp32 path handles.  On
        the pipelined tails (the defaults) each strip whose split audio is not
        finite is recomputed inside the tail launch by direct fp32 convolution
        in the reference's layer order (within the reference-conditioned
        tolerance, not bit-equal to the exact-f32 kernels); M2_REDO_LAUNCH=1
        and the windowed tails use the guarded exact-f32 launch behind the
        split kernels instead (bit-equal to those kernels).  The per-call cost
        is bench.py's ``vocoder_report_policy`` difference.
        "report" (opt-in): asynchronous - the next call raises,
        check_numerics() reports it at once."""
        if policy not in runtime.RANGE_POLICIES:
            raise ValueError(f"range policy {policy!r}: expected one of {sorted(runtime.RANGE_POLICIES)}")
        self.__dict__["_m2_range_policy"] = policy
        cache = _HANDLES.get(self)
        for hm in (cache.handles() if cache is not None else []):
            hm.set_range_policy(policy)

    def check_numerics(self, device: Optional[torch.device] = None):
        """Synchronise and raise if a split-path vocoder call since the last
        check produced non-finite audio (M2_E_RANGE semantics)."""
        cache = _HANDLES.get(self)
        want = None
        if device is not None:
            want = torch.device(device)
            if want.type == "cuda" and want.index is None:
                want = torch.device("cuda", torch.cuda.current_device())
        for hm in (cache.handles() if cache is not None else []):
            if (want is None or hm.device == want) and hm.check():
                raise ops.M2Error(
                    "m2-tts_amd: a split-f16 vocoder call produced non-finite audio (an input or activation "
                    "of magnitude >= 65520); re-run with set_vocoder_precision('f32') or set_range_policy('fallback')")

    def set_vocoder_precision(self, precision: str = "split"):
        """"split" = split-f16 MFMA kernels (fp32 operands as f16 hi/lo pairs,
        the default), "f32" = exact-f32 MFMA kernels."""
        path = {"split": 2, "f32": 1}[precision]
        self.__dict__["_m2_voc_path"] = path
        cache = _HANDLES.get(self)
        for hm in (cache.handles() if cache is not None else []):
            hm.vocoder_select(path)

    # -------------------------------------------------------------- forward
    def forward(self, phoneme_ids: Tensor, phoneme_lengths: Optional[Tensor] = None,
                target_durations: Optional[Tensor] = None,
                max_target_length: Optional[int] = None) -> Dict[str, Optional[Tensor]]:
        """Reference tts_model.py:350-400: audio only when not training."""
        ops.require_device(phoneme_ids, what="M2TTSModel")
        with torch.no_grad():
            hm = self._hip(phoneme_ids.device)
            enc, mask = hm.text_encoder(phoneme_ids, phoneme_lengths)
            dur = hm.duration(enc)
            durations = target_durations if target_durations is not None else dur
            reg = ops.regulate(enc, durations, max_target_length)
            mel = hm.decoder(reg)
            audio = None if self.training else hm.vocoder(mel, layout_btm=True)
        return {"encoder_output": enc, "duration_pred": dur, "regulated_output": reg,
                "mel_output": mel, "audio_output": audio, "padding_mask": mask}

    def inference(self, phoneme_ids: Tensor, phoneme_lengths: Optional[Tensor] = None,
                  duration_scale: float = 1.0) -> Tuple[Tensor, Tensor]:
        """(mel [B,T,M], audio [B,1,64T]) - reference tts_model.py:402-438."""
        self._eval_if_training()
        ops.require_device(phoneme_ids, what="M2TTSModel")
        with torch.no_grad():
            mel, audio = self._hip(phoneme_ids.device).inference(phoneme_ids, phoneme_lengths, duration_scale)
        return mel, audio

    def get_model_size(self) -> Dict[str, Any]:
        """Parameter counts per component (reference tts_model.py:440-459)."""
        comps = {}
        for name, module in self.named_children():
            total, trainable = count_parameters(module)
            comps[name] = {"total": total, "trainable": trainable, "size_mb": total * 4 / (1024 * 1024)}
        total, trainable = count_parameters(self)
        return {"total_params": total, "trainable_params": trainable,
                "total_size_mb": total * 4 / (1024 * 1024), "components": comps}
