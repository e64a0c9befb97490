"""GPU: the stage1 vocoder head with input_conv composed into ConvT1
(vocoder_x3.hip, head_convT1c_planar: a 4-tap transposed conv straight from
the mel, with the outputs at t = 0, 1, 4T-2, 4T-1 corrected for the zeros the
reference's ConvT1 sees at input frames -1 and T) against the CPU oracle (the
reference's SimpleVocoder.forward, tts_model.py:279-297) and against the
two-layer head (M2_HEAD_INCONV=1), over lengths that put the utterance edges
in every window position, both mel layouts.
"""
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


@pytest.mark.parametrize("B,T", [(3, 1), (2, 2), (2, 5), (3, 63), (2, 64), (1, 127), (2, 137)])
def test_head_comp_vs_oracle(gpu, B, T):
    m = build_model(gpu)
    mel = torch.randn(B, stage_config("s1").mel_channels, T, generator=torch.Generator().manual_seed(400 + T))
    out = m.vocoder(mel.to(gpu)).cpu()
    ref = orc.vocoder(golden_state("s1"), mel)
    assert out.shape == ref.shape
    assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4
    # the samples the corrected head outputs feed (t = 0, 1 and 4T - 2, 4T - 1 at 16x)
    assert maxabs(out[..., :48], ref[..., :48]) <= 1e-5 and maxabs(out[..., -48:], ref[..., -48:]) <= 1e-5


@pytest.mark.parametrize("B,T", [(32, 500), (5, 333), (2, 2600), (4, 1)])
def test_head_comp_vs_two_layers(gpu, monkeypatch, B, T):
    """The composed layer reorders fp32 sums of the same products (and the
    composed weights are rounded once): agreement well inside the bound."""
    mel = torch.randn(B, stage_config("s1").mel_channels, T, generator=torch.Generator().manual_seed(B * T + 1))
    m = build_model(gpu)
    out = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_HEAD_INCONV", "1")
    ref = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 2e-5 and rms(out.cpu(), ref.cpu()) <= 2e-6


def test_head_comp_btm_layout(gpu):
    """The decoder hands the vocoder [B, T, M] mel (read transposed in place)."""
    m = build_model(gpu)
    mel = torch.randn(3, stage_config("s1").mel_channels, 70, generator=torch.Generator().manual_seed(9))
    a = m.vocoder(mel.to(gpu))
    hm = m._hip(gpu)
    b = hm.vocoder(mel.transpose(1, 2).contiguous().to(gpu), layout_btm=True)
    assert torch.equal(a, b)


def build_s2(dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config("s2").as_dict())
    m.load_state_dict(golden_state("s2"))
    return m.to(dev).eval()


@pytest.mark.parametrize("B,T", [(3, 1), (2, 2), (2, 15), (2, 16), (1, 17), (2, 47)])
def test_head_comp_s2_vs_oracle(gpu, B, T):
    """Stage2 (M = 80, C = 256): the composed layer on the generic item path,
    16-frame windows; the edge columns also appear as halo columns."""
    m = build_s2(gpu)
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(500 + T))
    out = m.vocoder(mel.to(gpu)).cpu()
    ref = orc.vocoder(golden_state("s2"), mel)
    assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4
    assert maxabs(out[..., :48], ref[..., :48]) <= 1e-5 and maxabs(out[..., -48:], ref[..., -48:]) <= 1e-5


@pytest.mark.parametrize("B,T", [(8, 500), (16, 2600), (3, 33)])
def test_head_comp_s2_vs_two_layers(gpu, monkeypatch, B, T):
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(B * T + 2))
    m = build_s2(gpu)
    out = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_HEAD_INCONV", "1")
    ref = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 2e-5 and rms(out.cpu(), ref.cpu()) <= 2e-6


@pytest.mark.parametrize("B,T", [(3, 33), (2, 263), (1, 54), (16, 262)])
def test_head_s2_windows_bit_identical(gpu, monkeypatch, B, T):
    """The stage2 head's four windows (16 / 19 frames, 8 waves; 24 / 27, 16
    waves; run<CfgS2> picks by rounds of workgroup slots, M2_S2_HEAD_TF
    forces) sum the same products in the same order: identical audio, and the
    27-frame one against the oracle."""
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(B * T + 3))
    m = build_s2(gpu)
    auto = m.vocoder(mel.to(gpu))
    for tf in (16, 19, 24, 27):
        monkeypatch.setenv("M2_S2_HEAD_TF", str(tf))
        assert torch.equal(m.vocoder(mel.to(gpu)), auto), tf
    if B * T <= 100:
        ref = orc.vocoder(golden_state("s2"), mel)
        out = auto.cpu()
        assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4


@pytest.mark.parametrize("B,T", [(3, 33), (8, 500), (16, 262)])
def test_mid_s2_windows_bit_identical(gpu, monkeypatch, B, T):
    """The stage2 mid's 30- and 33-position windows (M2_S2_MID_ALT forces
    either): identical audio."""
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(B * T + 4))
    m = build_s2(gpu)
    monkeypatch.setenv("M2_S2_MID_ALT", "0")
    a = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_S2_MID_ALT", "1")
    assert torch.equal(m.vocoder(mel.to(gpu)), a)
