"""GPU: the stage2 vocoder head as two launches (vocoder_x3.hip,
x3_ct1_kernel: the composed input_conv o ConvT1 for a window of frames and one
slice of ConvT1's output channels, rows to a scratch buffer; x3_rb1_kernel:
ResBlock1 on those rows) against the fused head (one launch) and the CPU
oracle (the reference's SimpleVocoder.forward, tts_model.py:279-297,
components.py:196-200).  Every output is the same operation sequence as the
fused head's, so the two are compared bit for bit, over lengths that put the
utterance edges in every position of the split windows, both mel layouts,
and the speculative (device frame count) inference path."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, MEL_MAXABS_TOL, golden, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def build_s2(dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config("s2").as_dict())
    m.load_state_dict(golden_state("s2"))
    return m.to(dev).eval()


@pytest.mark.parametrize("B,T", [(3, 1), (2, 15), (1, 16), (2, 63), (1, 64), (2, 65), (3, 129), (8, 500), (5, 333)])
def test_split_head_equals_fused_head(gpu, monkeypatch, B, T):
    mel = torch.randn(B, stage_config("s2").mel_channels, T, generator=torch.Generator().manual_seed(700 + B * T))
    m = build_s2(gpu)
    monkeypatch.setenv("M2_S2_HEAD_SPLIT", "0")
    fused = m.vocoder(mel.to(gpu))
    monkeypatch.setenv("M2_S2_HEAD_SPLIT", "1")
    split = m.vocoder(mel.to(gpu))
    assert torch.equal(split, fused)
    hm = m._hip(gpu)
    btm = hm.vocoder(mel.transpose(1, 2).contiguous().to(gpu), layout_btm=True)
    assert torch.equal(btm, fused)
    if B * T <= 1000:
        ref = orc.vocoder(golden_state("s2"), mel)
        assert rms(split, ref) <= AUDIO_RMS_TOL and maxabs(split, ref) <= 1e-4


def test_split_head_inference_and_speculative(gpu, monkeypatch):
    """inference() twice (the second call launches the back half for a
    frame capacity, T from the device): both equal to the fused head's."""
    g = golden("s2_small")
    ids, lens = torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu)
    m = build_s2(gpu)
    monkeypatch.setenv("M2_S2_HEAD_SPLIT", "0")
    mel0, audio0 = m.inference(ids, lens)
    monkeypatch.setenv("M2_S2_HEAD_SPLIT", "1")
    for _ in range(2):
        mel1, audio1 = m.inference(ids, lens)
        assert torch.equal(mel1, mel0) and torch.equal(audio1, audio0)
    assert maxabs(mel1, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio1, torch.from_numpy(g["audio"])) <= AUDIO_RMS_TOL
