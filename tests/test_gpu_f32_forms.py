"""GPU: the stage1 exact-f32 vocoder's tail / mid forms (the strict-fp32
path, M2_VOC_F32=1 / m2_vocoder_select(1)): the 8-channel ConvT4 and
ResBlock4 in the two-phase forms (M2_F32_PAIR=1, vocoder_fused.hip
lconvT2p / lconv3_2p), the 8-wave half-window mid / tail tilings
(M2_F32_MT) and the head's input conv composed into ConvT1 with its edge
terms (M2_F32_COMP=1, lconvT1c), each against the CPU oracle (reference
components.py:196-200, tts_model.py:243-297) at the waveform bound, at
ragged lengths whose
windows end inside a 16- / 32-column tile, and on both tilings the batch
size picks (the 16-wave one-per-CU form and the 8-wave form)."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def build_model(dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config("s1").as_dict())
    m.load_state_dict(golden_state("s1"))
    return m.to(dev).eval()


@pytest.mark.parametrize("comp", ["0", "1"])
@pytest.mark.parametrize("pair", ["0", "1"])
@pytest.mark.parametrize("mt", ["0", "1", "2", "3"])
@pytest.mark.parametrize("B,T,plan", [(3, 137, "-1"), (2, 61, "-1"), (5, 250, "1"), (1, 9, "2"), (2, 127, "2"),
                                       (1, 1, "-1"), (2, 2, "2"), (1, 64, "2")])
def test_exact_f32_tail_forms(gpu, monkeypatch, comp, pair, mt, B, T, plan):
    from m2amd import _lib
    lib = _lib.load()
    monkeypatch.setenv("M2_VOC_F32", "1")
    monkeypatch.setenv("M2_F32_COMP", comp)
    monkeypatch.setenv("M2_F32_PAIR", pair)
    monkeypatch.setenv("M2_F32_MT", mt)
    monkeypatch.setenv("M2_VOC_PLAN", plan)
    mel = torch.randn(B, 64, T, generator=torch.Generator().manual_seed(100 + B + T))
    ref = orc.vocoder(golden_state("s1"), mel)
    m = build_model(gpu)
    assert lib.m2_vocoder_path(m._hip(gpu).handle) == 1
    out = m.vocoder(mel.to(gpu)).cpu()
    assert out.shape == ref.shape
    assert torch.isfinite(out).all()
    assert rms(out, ref) <= AUDIO_RMS_TOL
    assert maxabs(out, ref) <= 1e-4


def test_exact_f32_forms_agree(gpu, monkeypatch):
    """Every form computes each sample with its own fixed summation order:
    the tilings (M2_F32_MT) agree bit for bit within one layer form, and the
    two-phase form differs from the phase-split one by fp32 reordering only."""
    monkeypatch.setenv("M2_VOC_F32", "1")
    mel = torch.randn(4, 64, 300, generator=torch.Generator().manual_seed(3)).to(gpu)
    outs = {}
    for comp in ("0", "1"):
        for pair in ("0", "1"):
            for mt in ("0", "3"):
                monkeypatch.setenv("M2_F32_COMP", comp)
                monkeypatch.setenv("M2_F32_PAIR", pair)
                monkeypatch.setenv("M2_F32_MT", mt)
                outs[(comp, pair, mt)] = build_model(gpu).vocoder(mel).cpu()
    for comp in ("0", "1"):
        assert torch.equal(outs[(comp, "0", "0")], outs[(comp, "0", "3")])
        assert torch.equal(outs[(comp, "1", "0")], outs[(comp, "1", "3")])
        assert maxabs(outs[(comp, "0", "0")], outs[(comp, "1", "0")]) <= 1e-5
    assert maxabs(outs[("0", "0", "0")], outs[("1", "0", "0")]) <= 2e-5


def test_exact_f32_composed_head_guarded_redo(gpu, monkeypatch):
    """The guarded exact-f32 launch (range policy "fallback" with
    M2_REDO_LAUNCH=1) runs the same head / tail forms as the exact-f32
    kernels, so its audio equals theirs bit for bit with the composed head."""
    monkeypatch.setenv("M2_F32_COMP", "1")
    monkeypatch.setenv("M2_REDO_LAUNCH", "1")
    mel = torch.randn(2, 64, 45, generator=torch.Generator().manual_seed(5)) * 1e5
    m = build_model(gpu)
    m.set_range_policy("fallback")
    out = m.vocoder(mel.to(gpu))
    m.set_vocoder_precision("f32")
    assert torch.equal(out, m.vocoder(mel.to(gpu)))


@pytest.mark.parametrize("comp", ["0", "1"])
@pytest.mark.parametrize("B,T", [(2, 61), (1, 1), (3, 25), (2, 12), (1, 13)])
def test_exact_f32_composed_head_stage2(gpu, monkeypatch, comp, B, T):
    """stage2's exact-f32 head (M = 80, C = 256, 12-frame windows) with the
    input conv composed into ConvT1 (M2_F32_COMP=1, the default) or as its own
    layer: against the oracle at lengths that put both utterance edges in one
    window, end a window exactly, or leave one frame in the last window."""
    from m2amd import _lib
    from models.tts_model import M2TTSModel
    lib = _lib.load()
    monkeypatch.setenv("M2_VOC_F32", "1")
    monkeypatch.setenv("M2_F32_COMP", comp)
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(200 + B + T))
    ref = orc.vocoder(golden_state("s2"), mel)
    m = M2TTSModel(**stage_config("s2").as_dict())
    m.load_state_dict(golden_state("s2"))
    m = m.to(gpu).eval()
    assert lib.m2_vocoder_path(m._hip(gpu).handle) == 1
    out = m.vocoder(mel.to(gpu)).cpu()
    assert out.shape == ref.shape and torch.isfinite(out).all()
    assert rms(out, ref) <= AUDIO_RMS_TOL
    assert maxabs(out, ref) <= 1e-4
