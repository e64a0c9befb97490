"""Device selection for MI355X (replaces the reference's MPS/CPU logic in
src/utils/device.py:13-36).  One process per GPU: the device is the ROCm GPU
named by LOCAL_RANK (torchrun) or 0.  There is no CPU execution path."""
from __future__ import annotations

import logging
import os

import torch

logger = logging.getLogger(__name__)


def setup_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("m2-tts_amd needs a ROCm GPU (MI355X); none is visible")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    logger.info(f"Using {torch.cuda.get_device_name(dev)} ({dev})")
    return dev


def get_device_info() -> dict:
    info = {"rocm_available": torch.cuda.is_available(), "device_count": torch.cuda.device_count() if torch.cuda.is_available() else 0}
    if info["rocm_available"]:
        p = torch.cuda.get_device_properties(0)
        info.update(name=p.name, total_memory_gb=p.total_memory / 2**30, multi_processor_count=p.multi_processor_count)
    return info
