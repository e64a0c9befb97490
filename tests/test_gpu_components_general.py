"""GPU: the standalone components' general geometries (reference
components.py:42-90, 143-223, tts_model.py:231-297) - what the drop-in
accepts beyond the shapes M2TTSModel itself uses: LightweightResBlock with
any odd kernel size and dilation, ConvBlock / VariancePredictor with any
kernel size, SimpleVocoder(kernel_size=...), and MultiHeadAttention with a
head_dim outside the MFMA instances (16/32/48/64) - each against the CPU
oracle's functional restatement of the same module on the same weights."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import maxabs, rms

pytestmark = pytest.mark.gpu


def _sd(module, prefix):
    return {f"{prefix}.{k}": v.detach().cpu() for k, v in module.state_dict().items()}


@pytest.mark.parametrize("k,d", [(3, 1), (3, 2), (5, 1), (5, 3), (7, 2), (1, 1)])
def test_resblock_kernel_dilation(gpu, k, d):
    from models.components import LightweightResBlock
    torch.manual_seed(k * 10 + d)
    blk = LightweightResBlock(24, kernel_size=k, dilation=d)
    x = torch.randn(3, 24, 301)
    ref = orc.resblock(_sd(blk, "rb"), "rb", x, dilation=d)
    out = blk.to(gpu)(x.to(gpu))
    assert out.shape == ref.shape
    assert maxabs(out, ref) <= 1e-5


def test_resblock_even_kernel_fails_like_the_reference(gpu):
    from models.components import LightweightResBlock
    blk = LightweightResBlock(8, kernel_size=4).to(gpu)
    with pytest.raises(RuntimeError):
        blk(torch.randn(1, 8, 50, device=gpu))


@pytest.mark.parametrize("k", [1, 3, 4, 5, 7])
def test_conv_block_and_variance_predictor_kernel_size(gpu, k):
    from models.components import ConvBlock, VariancePredictor
    torch.manual_seed(k)
    cb = ConvBlock(16, 24, kernel_size=k).eval()
    with torch.no_grad():  # non-trivial BatchNorm running statistics
        cb.norm.running_mean.uniform_(-0.5, 0.5)
        cb.norm.running_var.uniform_(0.5, 2.0)
        cb.norm.weight.uniform_(0.5, 1.5)
        cb.norm.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2, 16, 77)
    ref = orc.conv_block(_sd(cb, "cb"), "cb", x)
    out = cb.to(gpu)(x.to(gpu))
    assert out.shape == ref.shape  # even k: L + 1 frames, as nn.Conv1d(padding=k//2)
    assert maxabs(out, ref) <= 1e-5
    if k % 2 == 1:
        vp = VariancePredictor(16, kernel_size=k).eval()
        sd = _sd(vp, "vp.predictor")
        y = orc.conv_block(sd, "vp.predictor.conv_layers.0", x)
        y = orc.conv_block(sd, "vp.predictor.conv_layers.1", y)
        ref = torch.nn.functional.conv1d(y, sd["vp.predictor.projection.weight"], sd["vp.predictor.projection.bias"])
        out = vp.to(gpu)(x.to(gpu))
        assert maxabs(out, ref) <= 1e-5


@pytest.mark.parametrize("ks", [5, 7])
def test_simple_vocoder_kernel_size(gpu, ks):
    from models.tts_model import SimpleVocoder
    torch.manual_seed(ks)
    voc = SimpleVocoder(mel_channels=16, hidden_channels=64, kernel_size=ks).eval()
    mel = torch.randn(2, 16, 23)
    ref = orc.vocoder(_sd(voc, "vocoder"), mel)
    out = voc.to(gpu)(mel.to(gpu))
    assert out.shape == ref.shape == (2, 1, 64 * 23)
    assert rms(out, ref) <= 1e-4 and maxabs(out, ref) <= 1e-4


@pytest.mark.parametrize("H,heads", [(40, 2), (96, 4), (72, 3), (40, 5), (256, 2), (24, 1)])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_any_head_dim(gpu, H, heads, masked):
    from models.components import MultiHeadAttention
    torch.manual_seed(H + heads)
    mha = MultiHeadAttention(H, heads).eval()
    B, N = 3, 70
    x = torch.randn(B, N, H)
    mask = None
    if masked:
        lens = torch.tensor([70, 33, 0])
        mask = torch.arange(N).expand(B, N) < lens.unsqueeze(1)
    ref = orc.attention(_sd(mha, "a"), "a", x, heads, mask)
    out = mha.to(gpu)(x.to(gpu), None if mask is None else mask.to(gpu))
    assert maxabs(out, ref) <= 2e-5


def test_model_with_generic_head_dim(gpu):
    """M2TTSModel(hidden 96, 4 heads: head_dim 24) runs its attention on the
    generic kernel and matches the oracle end to end."""
    from models.tts_model import M2TTSModel
    torch.manual_seed(3)
    m = M2TTSModel(hidden_dim=96, mel_channels=80, text_encoder_layers=2, decoder_layers=2, num_heads=4,
                   vocoder_channels=64).eval()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    sd = orc.pin_durations(sd)
    m.load_state_dict(sd)
    cfg = orc.OracleConfig(hidden_dim=96, mel_channels=80, text_encoder_layers=2, decoder_layers=2, num_heads=4,
                           vocoder_channels=64)
    ids = torch.randint(0, 42, (2, 19), generator=torch.Generator().manual_seed(1))
    lens = torch.tensor([19, 12])
    m = m.to(gpu)
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    ref_mel, ref_audio = orc.inference(sd, cfg, ids, lens, as_written=False)
    assert mel.shape == ref_mel.shape
    assert maxabs(mel, ref_mel) <= 1e-3
    assert rms(audio, ref_audio) <= 1e-4
