"""GPU: the pipelined stage2 vocoder tail (vocoder_tailp2.hip: ConvT3,
ResBlock3, ConvT4, ResBlock4 and output_conv at C = 256 in polyphase form,
two waves per layer) against the CPU oracle (the reference's
SimpleVocoder.forward, tts_model.py:279-297) and against the x3 tail kernel it
replaces (M2_VOC_TAIL_X3=1), over ragged lengths that put utterance ends in
every position of a 16-column chunk, and at forced strip lengths.
"""
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def build_model(dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config("s2").as_dict())
    m.load_state_dict(golden_state("s2"))
    return m.to(dev).eval()


def kernel_names(m, dev):
    from m2amd import _lib
    lib = _lib.load()
    h = m._hip(dev).handle
    return [lib.m2_profile_kernel_name_for(h, i).decode() for i in range(3)]


@pytest.mark.parametrize("B,T", [(3, 1), (2, 7), (3, 61), (1, 137)])
def test_tailp2_vs_oracle(gpu, B, T):
    m = build_model(gpu)
    assert kernel_names(m, gpu)[2].startswith("tailp2_kernel")
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(100 + T))
    out = m.vocoder(mel.to(gpu)).cpu()
    ref = orc.vocoder(golden_state("s2"), mel)
    assert out.shape == ref.shape
    assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4


@pytest.mark.parametrize("B,T", [(8, 500), (2, 2600), (16, 2600), (5, 333)])
def test_tailp2_vs_x3_tail(gpu, monkeypatch, B, T):
    """Same split-f16 products as the x3 tail in another summation order:
    agreement to fp32 rounding.  (16, 2600) takes 163-chunk strips (one
    round of 256 workgroups), (8, 500) 16-chunk strips."""
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(B * T))
    m = build_model(gpu)
    out = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_VOC_TAIL_X3", "1")
    mx = build_model(gpu)
    assert kernel_names(mx, gpu)[2].startswith("x3_tail")
    ref = mx.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 2e-6


@pytest.mark.parametrize("B,T", [(3, 1), (2, 2), (3, 61)])
def test_tailp2_outc_edges_vs_oracle(gpu, B, T):
    """The composed ResBlock4-conv2 + output_conv layer (the default six-layer
    form) corrects the two utterance-edge samples for the reference's zero
    padding of the resblock output."""
    m = build_model(gpu)
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(300 + T))
    out = m.vocoder(mel.to(gpu)).cpu()
    ref = orc.vocoder(golden_state("s2"), mel)
    assert maxabs(out[..., :4], ref[..., :4]) <= 1e-5 and maxabs(out[..., -4:], ref[..., -4:]) <= 1e-5
    assert rms(out, ref) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("B,T", [(8, 500), (16, 2600), (5, 333)])
def test_tailp2_outc_vs_seven_layers(gpu, monkeypatch, B, T):
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(B + T))
    m = build_model(gpu)
    out = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_TAILP2_SEVEN", "1")
    ref = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert float((out - ref).abs().max()) <= 2e-6


@pytest.mark.parametrize("nch", [1, 7, 13, 100])
def test_tailp2_strip_lengths(gpu, monkeypatch, nch):
    """The strip length is a launch argument (M2_TAILP2_NCH forces one): every
    column's arithmetic is the same whatever strip holds it, so the audio is
    bit-identical to the default strips, with strip ends everywhere."""
    mel = torch.randn(3, stage_config("s2").mel_channels, 97, generator=torch.Generator().manual_seed(nch))
    m = build_model(gpu)
    ref = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_TAILP2_NCH", str(nch))
    out = m.vocoder(mel.to(gpu))
    assert torch.equal(out, ref)
