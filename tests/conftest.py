import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
for p in (ROOT / "m2-tts_amd" / "src", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

# Parity bar from BASELINE.json north_star.
MEL_MAXABS_TOL = 1e-3
AUDIO_RMS_TOL = 1e-4


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def golden(name):
    return np.load(GOLDEN / f"{name}.npz", allow_pickle=False)


def golden_state(stage: str, pinned: bool = True):
    w = golden(f"weights_{stage}")
    sd = {k: torch.from_numpy(w[k]) for k in w.files}
    if not pinned:
        u = golden(f"weights_{stage}_unpinned_proj")
        p = "duration_predictor.predictor.projection"
        sd[p + ".weight"] = torch.from_numpy(u["weight"])
        sd[p + ".bias"] = torch.from_numpy(u["bias"])
    return sd


def stage_config(stage: str):
    import m2tts_oracle as orc
    return orc.STAGE1 if stage == "s1" else orc.STAGE2


def rms(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float(((a - b) ** 2).mean().sqrt()) if a.numel() else 0.0


def maxabs(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max()) if a.numel() else 0.0


@pytest.fixture(scope="session")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    from m2amd import _lib
    _lib.load()
    return torch.device("cuda:0")


def _reload_switches():
    from m2amd import _lib
    if _lib._lib is not None:
        _lib.reload_switches()


@pytest.fixture
def monkeypatch():
    """pytest's monkeypatch, plus: setting or deleting an M2_* developer switch
    re-reads the library's switch table (m2_reload_switches; the library never
    reads the environment per call), and so does the undo at teardown."""
    mp = pytest.MonkeyPatch()
    set0, del0 = mp.setenv, mp.delenv

    def setenv(name, value, prepend=None):
        set0(name, value, prepend)
        if name.startswith("M2_"):
            _reload_switches()

    def delenv(name, raising=True):
        del0(name, raising)
        if name.startswith("M2_"):
            _reload_switches()

    mp.setenv, mp.delenv = setenv, delenv
    yield mp
    mp.undo()
    _reload_switches()
