#!/usr/bin/env python3
"""Text -> WAV on MI355X.  Drop-in for the reference ``scripts/synthesize.py``
(same flags: --text --checkpoint --output --duration-scale --sample-rate;
same flow: load_model -> TextProcessor.process_text(max_length=256) ->
M2TTSModel.inference -> save_audio(audio[0, 0])).

Checkpoints: the trainer's dict ``{'model_state_dict', 'config', 'step', ...}``
(reference training/train.py:242-254) or a bare state_dict.  ``config`` may be
a plain dict or an OmegaConf DictConfig; only the 8 model keys are read.
torch.load runs with ``weights_only=True``; a checkpoint whose config is a
pickled DictConfig is refused by that loader, and is only unpickled with the
explicit ``--trust-checkpoint`` opt-in (trusted local files only), or its
config can be given with ``--config configs/stage1_poc.yaml`` instead.
"""
from __future__ import annotations

import argparse
import logging
import sys
from pathlib import Path
from typing import Any, Optional

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "src"))

from models.tts_model import M2TTSModel  # noqa: E402
from utils.audio import save_audio  # noqa: E402
from utils.device import setup_device  # noqa: E402
from utils.text import TextProcessor  # noqa: E402

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)


def _get(cfg: Any, dotted: str, default: Any = None) -> Any:
    """Attribute or key access through a DictConfig / dict / namespace."""
    cur = cfg
    for part in dotted.split("."):
        if cur is None:
            return default
        if isinstance(cur, dict):
            cur = cur.get(part, None)
        else:
            cur = getattr(cur, part, None)
    return default if cur is None else cur


def model_kwargs(config: Any) -> dict:
    """The 8 M2TTSModel arguments the reference reads from a config
    (scripts/synthesize.py:37-46)."""
    return dict(vocab_size=_get(config, "model.text_encoder.vocab_size"),
                hidden_dim=_get(config, "model.text_encoder.hidden_dim"),
                mel_channels=_get(config, "model.decoder.mel_channels"),
                text_encoder_layers=_get(config, "model.text_encoder.num_layers"),
                decoder_layers=_get(config, "model.decoder.num_layers", 2),
                num_heads=_get(config, "model.text_encoder.num_heads"),
                dropout=_get(config, "model.text_encoder.dropout"),
                vocoder_channels=_get(config, "model.vocoder.hidden_channels"))


def load_config(path: Optional[Path]) -> Optional[dict]:
    if path is None:
        return None
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def read_checkpoint(path: Path, device: torch.device, trust: bool = False) -> dict:
    try:
        ckpt = torch.load(path, map_location=device, weights_only=True)
    except Exception as e:  # noqa: BLE001 - the safe loader refuses pickled objects
        if not trust:
            raise RuntimeError(f"{path}: the weights-only loader refused this checkpoint ({e.__class__.__name__}); "
                               f"it probably carries a pickled OmegaConf config.  Pass --config <yaml> and a "
                               f"weights-only checkpoint, or --trust-checkpoint for a trusted local file.") from e
        ckpt = torch.load(path, map_location=device, weights_only=False)
    if isinstance(ckpt, dict) and "model_state_dict" not in ckpt and all(isinstance(v, torch.Tensor) for v in ckpt.values()):
        ckpt = {"model_state_dict": ckpt}
    return ckpt


def load_model(checkpoint_path: Path, device: torch.device, config_path: Optional[Path] = None,
               trust: bool = False) -> M2TTSModel:
    """Reference scripts/synthesize.py:24-55."""
    if not checkpoint_path.exists():
        raise FileNotFoundError(f"Checkpoint not found: {checkpoint_path}")
    ckpt = read_checkpoint(checkpoint_path, device, trust)
    config = load_config(config_path) if config_path else ckpt.get("config")
    if config is None:
        logger.warning("No config found in checkpoint, using default")
        model = M2TTSModel()
    else:
        model = M2TTSModel(**model_kwargs(config))
    model.load_state_dict(ckpt["model_state_dict"])
    model.to(device)
    model.eval()
    # one utterance per call and the audio goes to the host anyway: pay the
    # one synchronisation per vocoder call that guarantees a finite result
    # (split-f16 out of range -> recomputed on the exact-f32 kernels)
    model.set_range_policy("fallback")
    logger.info(f"Loaded model from {checkpoint_path}")
    logger.info(f"Training step: {ckpt.get('step', 'unknown')}")
    return model


def synthesize_text(text: str, model: M2TTSModel, text_processor: TextProcessor, device: torch.device,
                    duration_scale: float = 1.0) -> tuple:
    """Reference scripts/synthesize.py:58-88."""
    td = text_processor.process_text(text, max_length=256)
    ids = torch.LongTensor(td["phoneme_ids"]).unsqueeze(0).to(device)
    lens = torch.LongTensor([td["length"]]).to(device)
    logger.info(f"Synthesizing: '{text}'")
    logger.info(f"Phonemes: {' '.join(td['phonemes'][:20])}...")
    logger.info(f"Sequence length: {td['length']}")
    with torch.no_grad():
        mel, audio = model.inference(ids, lens, duration_scale=duration_scale)
    logger.info(f"Generated mel shape: {mel.shape}")
    logger.info(f"Generated audio shape: {audio.shape}")
    return mel, audio


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="M2 TTS Text Synthesis (MI355X)")
    p.add_argument("--text", type=str, required=True, help="Text to synthesize")
    p.add_argument("--checkpoint", type=str, required=True, help="Path to model checkpoint")
    p.add_argument("--output", type=str, default="output.wav", help="Output audio file path")
    p.add_argument("--duration-scale", type=float, default=1.0, help="Duration scaling factor (1.0 = normal speed)")
    p.add_argument("--sample-rate", type=int, default=22050, help="Audio sample rate")
    p.add_argument("--config", type=str, default=None, help="YAML config with the model section (overrides the checkpoint's)")
    p.add_argument("--trust-checkpoint", action="store_true",
                   help="allow full unpickling of a trusted local checkpoint (OmegaConf config objects)")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    device = setup_device()
    logger.info(f"Using device: {device}")
    model = load_model(Path(args.checkpoint), device, Path(args.config) if args.config else None,
                       args.trust_checkpoint)
    processor = TextProcessor()
    _, audio = synthesize_text(args.text, model, processor, device, args.duration_scale)
    if audio is not None and audio.size(0) > 0:
        audio_np = audio[0, 0].cpu().numpy()
        out = Path(args.output)
        out.parent.mkdir(parents=True, exist_ok=True)
        save_audio(audio_np, out, args.sample_rate)
        logger.info(f"Audio saved to: {out}")
        logger.info(f"Duration: {len(audio_np) / args.sample_rate:.2f} seconds")
    else:
        logger.error("No audio generated")


if __name__ == "__main__":
    main()
