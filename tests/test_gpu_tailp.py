"""GPU: the pipelined stage1 vocoder tail (vocoder_tailp.hip) in its six-layer
form, where ResBlock4's conv2 and output_conv run as one composed layer
(outc_role: a k5 conv on ResBlock4's intermediate plus a k3 conv on ConvT4's
output, with the two utterance-edge samples corrected for the reference's
zero padding of the resblock output), against the CPU oracle (the reference's
SimpleVocoder.forward, tts_model.py:279-297) and against the seven-layer form
(M2_TAILP_SEVEN=1), over lengths that put utterance ends in every position of a
16-column chunk and strips of every instantiated length.
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


def kernel_names(m, dev):
    from m2amd import _lib
    lib = _lib.load()
    h = m._hip(dev).handle
    return [lib.m2_profile_kernel_name_for(h, i).decode() for i in range(3)]


@pytest.mark.parametrize("B,T", [(3, 1), (2, 2), (2, 7), (3, 61), (1, 137)])
def test_tailp_outc_vs_oracle(gpu, B, T):
    m = build_model(gpu)
    assert kernel_names(m, gpu)[2].startswith("tailp_kernel")
    mel = torch.randn(B, stage_config("s1").mel_channels, T, generator=torch.Generator().manual_seed(200 + T))
    out = m.vocoder(mel.to(gpu)).cpu()
    ref = orc.vocoder(golden_state("s1"), mel)
    assert out.shape == ref.shape
    assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4
    # the corrected edge samples in particular
    assert maxabs(out[..., :4], ref[..., :4]) <= 1e-5 and maxabs(out[..., -4:], ref[..., -4:]) <= 1e-5


@pytest.mark.parametrize("B,T", [(32, 500), (8, 500), (2, 2600), (5, 333), (1, 3)])
def test_tailp_outc_vs_seven_layers(gpu, monkeypatch, B, T):
    """The composed layer reorders fp32 sums of the same products: agreement
    to fp32 rounding.  (32, 500) takes 21-chunk strips, (8, 500) 8, (2, 2600)
    8 (the grid model's choices)."""
    mel = torch.randn(B, stage_config("s1").mel_channels, T, generator=torch.Generator().manual_seed(B * T))
    m = build_model(gpu)
    out = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_TAILP_SEVEN", "1")
    ref = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 2e-6




@pytest.mark.parametrize("nch", [1, 5, 21, 77])
def test_tailp_strip_lengths(gpu, monkeypatch, nch):
    """The strip length is a launch argument (M2_TAILP_NCH forces one): every
    column's arithmetic is the same whatever strip holds it, so the audio is
    bit-identical to the default strips, with strip ends everywhere."""
    mel = torch.randn(3, stage_config("s1").mel_channels, 83, generator=torch.Generator().manual_seed(nch))
    m = build_model(gpu)
    ref = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_TAILP_NCH", str(nch))
    out = m.vocoder(mel.to(gpu))
    assert torch.equal(out, ref)


@pytest.mark.parametrize("nch", [1, 3, 16, 41])
def test_midp_strip_lengths(gpu, monkeypatch, nch):
    """The pipelined stage1 mid (vocoder_midp.hip) takes its strip length as a
    launch argument too (M2_MIDP_NCH forces one): bit-identical audio."""
    mel = torch.randn(2, stage_config("s1").mel_channels, 71, generator=torch.Generator().manual_seed(50 + nch))
    m = build_model(gpu)
    assert kernel_names(m, gpu)[1].startswith("midp_kernel")
    ref = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_MIDP_NCH", str(nch))
    out = m.vocoder(mel.to(gpu))
    assert torch.equal(out, ref)
