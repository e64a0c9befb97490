"""GPU: the one-launch-per-layer transformer kernels (csrc/transformer_layer.hip)
against the CPU oracle (reference components.py:59-140, tts_model.py:57-89,
211-228) and against the three-launch layers (M2_TF_LAYER=0).

Edge cases of the tiling: N around the 16-row tile and 32-key chunk edges
(1, 15, 16, 17, 31, 32, 33, ...), tiles wholly past an utterance's end (their
K / V rows must be written as zeros), batches that are not a multiple of the
8 XCDs, key-padding masks with lengths 0 (every key masked: uniform weights
over the N keys, the -1e9 fill), 1, ragged and past S."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import MEL_MAXABS_TOL, golden, golden_state, maxabs, stage_config

pytestmark = pytest.mark.gpu

STAGES = ["s1", "s2"]
# fp32 reorder noise of the split-f16 layers against the oracle (observed ~2e-6)
ENC_TOL = 2e-5
DEC_TOL = 2e-5


def build_model(stage, dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config(stage).as_dict())
    m.load_state_dict(golden_state(stage))
    return m.to(dev).eval()


@pytest.fixture(params=["auto", "1", "2", "4", "4q3", "4q12", "f4"])
def rows_per_tile(request, monkeypatch):
    """The tile forms a default can pick: 16- and 32-row workgroup tiles with
    key-quarter attention, 64-row tiles with query-split attention (K / V
    staged in LDS; M2_TFL_RB) - the key-quarter form on unmasked layers
    (eight computing waves, fragments straight from L2), on masked ones the
    lean one-block form at head_dim 32 and the lean two-block form at
    head_dim 48 - and the per-call choice; "4q3": the lean
    two-block form on the unmasked layers too (M2_TFL_QS2=3: what a layer
    whose scores may leave the f16 range runs, m2_layer_w::wide_scores);
    "4q12": M2_TFL_QS2=12 forced (the masked layers still fall back);
    "f4": 64-row tiles for the first (LN1 -> QKV) launch (M2_TFL_FIRST_RB,
    the default for very large grids)."""
    if request.param == "f4":
        monkeypatch.setenv("M2_TFL_FIRST_RB", "4")
    elif request.param != "auto":
        monkeypatch.setenv("M2_TFL_RB", request.param[0])
    if request.param.startswith("4q"):
        monkeypatch.setenv("M2_TFL_QS2", request.param[2:])
    return request.param


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("B,S", [(1, 1), (2, 15), (3, 16), (1, 17), (9, 31), (2, 32), (5, 33), (17, 47), (4, 100)])
def test_text_encoder_edges(gpu, stage, B, S, rows_per_tile):
    cfg = stage_config(stage)
    sd = golden_state(stage)
    m = build_model(stage, gpu)
    g = torch.Generator().manual_seed(B * 1000 + S)
    ids = torch.randint(0, 42, (B, S), generator=g)
    lens = torch.randint(0, S + 3, (B,), generator=g)
    lens[0] = S
    if B > 2:
        lens[1] = 0  # every key masked: the -1e9 fill gives uniform weights
        lens[2] = 1
    for lengths in (lens, None):
        enc, mask = m.text_encoder(ids.to(gpu), None if lengths is None else lengths.to(gpu))
        ref, ref_mask = orc.text_encoder(sd, cfg, ids, lengths)
        assert maxabs(enc, ref) <= ENC_TOL, (lengths is None, maxabs(enc, ref))
        if lengths is not None:
            assert torch.equal(mask.cpu(), ref_mask)


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("B,T", [(1, 1), (2, 16), (3, 17), (1, 31), (9, 32), (2, 33), (5, 63), (1, 64), (2, 65),
                                 (1, 500), (3, 257)])
def test_mel_decoder_edges(gpu, stage, B, T, rows_per_tile):
    cfg = stage_config(stage)
    sd = golden_state(stage)
    m = build_model(stage, gpu)
    x = torch.randn(B, T, cfg.hidden_dim, generator=torch.Generator().manual_seed(7 * T + B))
    mel = m.decoder(x.to(gpu))
    ref = orc.mel_decoder(sd, cfg, x)
    assert mel.shape == ref.shape
    assert maxabs(mel, ref) <= DEC_TOL, maxabs(mel, ref)


@pytest.mark.parametrize("stage", STAGES)
def test_one_launch_layers_match_three_launch_layers(gpu, stage, monkeypatch):
    """inference() on the one-launch layers and on the three-launch layers
    (ln_gemm / attention / post_attn): both parity-green, and within fp32
    reordering noise of each other (the frame counts identical)."""
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("M2_TF_LAYER", v)
        out[v] = m.inference(ids, lens)
        assert maxabs(out[v][0], g["mel"]) <= MEL_MAXABS_TOL
    assert out["1"][0].shape == out["0"][0].shape
    assert maxabs(out["1"][0], out["0"][0]) <= 2e-5
    assert maxabs(out["1"][1], out["0"][1]) <= 2e-5


@pytest.mark.parametrize("stage", STAGES)
def test_inference_ragged_batch_not_multiple_of_8(gpu, stage):
    """11 utterances, ragged lengths (some masked keys, one length 0), the
    whole path against the oracle."""
    cfg = stage_config(stage)
    sd = golden_state(stage)
    m = build_model(stage, gpu)
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, 42, (11, 37), generator=g)
    lens = torch.randint(1, 38, (11,), generator=g)
    lens[3] = 0
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    ref_mel, ref_audio = orc.inference(sd, cfg, ids, lens, as_written=False)
    assert mel.shape == ref_mel.shape
    assert maxabs(mel, ref_mel) <= MEL_MAXABS_TOL
    assert float(((audio.cpu().double() - ref_audio.double()) ** 2).mean().sqrt()) <= 1e-4


@pytest.mark.parametrize("stage", STAGES)
def test_large_grid_query_split_auto(gpu, stage):
    """Grids of >= 1024 16-row tiles pick the 64-row query-split attention by
    themselves: the decoder (unmasked, B=64 T=250) and the text encoder
    (masked, ragged, B=128 S=130) against the oracle."""
    cfg = stage_config(stage)
    sd = golden_state(stage)
    m = build_model(stage, gpu)
    x = torch.randn(64, 250, cfg.hidden_dim, generator=torch.Generator().manual_seed(5))
    mel = m.decoder(x.to(gpu))
    assert maxabs(mel, orc.mel_decoder(sd, cfg, x)) <= DEC_TOL
    g = torch.Generator().manual_seed(6)
    ids = torch.randint(0, 42, (128, 130), generator=g)
    lens = torch.randint(0, 131, (128,), generator=g)
    enc, mask = m.text_encoder(ids.to(gpu), lens.to(gpu))
    ref, ref_mask = orc.text_encoder(sd, cfg, ids, lens)
    assert maxabs(enc, ref) <= ENC_TOL
    assert torch.equal(mask.cpu(), ref_mask)
