"""GPU parity: the HIP path vs the reference's outputs (golden fixtures made
by importing the reference, tests/golden/make_golden.py) and vs the CPU
oracle (oracle/m2tts_oracle.py, bit-identical to the reference on CPU).

Tolerances (BASELINE.json north_star): mel max-abs <= 1e-3, waveform RMS
<= 1e-4.  Integer outputs (frame counts, masks) must match exactly.
"""
import numpy as np
import pytest
import torch

import m2tts_oracle as orc
from conftest import (AUDIO_RMS_TOL, MEL_MAXABS_TOL, golden, golden_state, maxabs, rms, stage_config)

pytestmark = pytest.mark.gpu
STAGES = ["s1", "s2"]
# Intermediate fp32 tensors: reordering noise only.
ENC_TOL = 1e-4


def build_model(stage, dev, pinned=True):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config(stage).as_dict())
    m.load_state_dict(golden_state(stage, pinned))
    return m.to(dev).eval()


def _ids(g, dev):
    return torch.from_numpy(g["ids"]).to(dev), torch.from_numpy(g["lengths"]).to(dev)


@pytest.mark.parametrize("stage", STAGES)
def test_forward_small(gpu, stage):
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    out = m(ids, lens)
    assert maxabs(out["encoder_output"], g["encoder_output"]) <= ENC_TOL
    assert maxabs(out["duration_pred"], g["duration_pred"]) <= ENC_TOL
    assert torch.equal(out["padding_mask"].cpu(), torch.from_numpy(g["padding_mask"]))
    assert out["regulated_output"].shape == tuple(g["regulated_output"].shape)
    assert maxabs(out["regulated_output"], g["regulated_output"]) <= ENC_TOL
    assert out["mel_output"].shape == tuple(g["mel"].shape)
    assert maxabs(out["mel_output"], g["mel"]) <= MEL_MAXABS_TOL
    assert out["audio_output"].shape == tuple(g["audio"].shape)
    assert rms(out["audio_output"], g["audio"]) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", STAGES)
def test_inference_small(gpu, stage):
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    mel, audio = m.inference(ids, lens)
    assert mel.shape == tuple(g["mel"].shape) and audio.shape == tuple(g["audio"].shape)
    assert maxabs(mel, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio, g["audio"]) <= AUDIO_RMS_TOL
    assert maxabs(audio, g["audio"]) <= 1e-3


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("sub", ["free", "pad", "trunc"])
def test_teacher_forced(gpu, stage, sub):
    g = golden(f"{stage}_target_{sub}")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    mtl = int(g["max_target_length"])
    out = m(ids, lens, target_durations=torch.from_numpy(g["target_durations"]).to(gpu),
            max_target_length=None if mtl < 0 else mtl)
    assert out["regulated_output"].shape == tuple(g["regulated_output"].shape)
    assert maxabs(out["regulated_output"], g["regulated_output"]) <= ENC_TOL
    assert maxabs(out["mel_output"], g["mel"]) <= MEL_MAXABS_TOL
    assert rms(out["audio_output"], g["audio"]) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", STAGES)
def test_duration_scale(gpu, stage):
    g = golden(f"{stage}_scale")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    mel, audio = m.inference(ids, lens, duration_scale=float(g["duration_scale"]))
    assert mel.shape == tuple(g["mel"].shape)
    assert maxabs(mel, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio, g["audio"]) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", STAGES)
def test_untrained_durations_give_one_zero_frame(gpu, stage):
    g = golden(f"{stage}_untrained")
    m = build_model(stage, gpu, pinned=False)
    ids, lens = _ids(g, gpu)
    mel, audio = m.inference(ids, lens)
    assert mel.shape == tuple(g["mel"].shape) == (2, 1, stage_config(stage).mel_channels)
    assert maxabs(mel, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio, g["audio"]) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", STAGES)
def test_vocoder_layers(gpu, stage):
    """Every vocoder layer, through the model handle and the standalone kernels."""
    m = build_model(stage, gpu)
    voc = m.vocoder
    hm = m._hip(gpu)
    g = golden(f"{stage}_input_conv")
    from m2amd import ops
    y = ops.conv1d(torch.from_numpy(g["x"]).to(gpu), voc.input_conv.weight, voc.input_conv.bias)
    assert maxabs(y, g["y"]) <= 1e-4
    for k in range(4):
        g = golden(f"{stage}_convT{k}")
        x = torch.from_numpy(g["x"]).to(gpu)
        assert maxabs(hm.upsample(k, x, int(g["rate"])), g["y"]) <= 1e-4
        assert maxabs(ops.conv_transpose1d(x, voc.upsamples[k].weight, voc.upsamples[k].bias, int(g["rate"]),
                                           act=ops.ACT_LEAKY), g["y"]) <= 1e-4
        g = golden(f"{stage}_resblock{k}")
        x = torch.from_numpy(g["x"]).to(gpu)
        assert maxabs(hm.resblock(k, x), g["y"]) <= 1e-4
        assert maxabs(voc.resblocks[k](x), g["y"]) <= 1e-4
    g = golden(f"{stage}_output_conv")
    y = ops.conv1d(torch.from_numpy(g["x"]).to(gpu), voc.output_conv.weight, voc.output_conv.bias, act=ops.ACT_TANH)
    assert maxabs(y, g["y"]) <= 1e-5


@pytest.mark.parametrize("stage", STAGES)
def test_stage_modules_called_directly(gpu, stage):
    """Callers use model.text_encoder / duration_predictor / length_regulator /
    decoder / vocoder directly (train_stage2.py:258); standalone copies of the
    stage modules take the per-op path.  Both must agree with the reference."""
    from models.tts_model import DurationPredictor, MelDecoder, SimpleVocoder, TextEncoder
    cfg = stage_config(stage)
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    sd = golden_state(stage)
    standalone = {
        "text_encoder": TextEncoder(cfg.vocab_size, cfg.hidden_dim, cfg.text_encoder_layers, cfg.num_heads),
        "duration_predictor": DurationPredictor(cfg.hidden_dim),
        "decoder": MelDecoder(cfg.hidden_dim, cfg.mel_channels, cfg.decoder_layers, cfg.num_heads),
        "vocoder": SimpleVocoder(cfg.mel_channels, cfg.vocoder_channels),
    }
    for name, mod in standalone.items():
        mod.load_state_dict({k[len(name) + 1:]: v for k, v in sd.items() if k.startswith(name + ".")})
        mod.to(gpu).eval()
    for te in (m.text_encoder, standalone["text_encoder"]):
        enc, mask = te(ids, lens)
        assert maxabs(enc, g["encoder_output"]) <= ENC_TOL
        assert torch.equal(mask.cpu(), torch.from_numpy(g["padding_mask"]))
    enc = torch.from_numpy(g["encoder_output"]).to(gpu)
    for dp in (m.duration_predictor, standalone["duration_predictor"]):
        assert maxabs(dp(enc), g["duration_pred"]) <= ENC_TOL
    reg = m.length_regulator(enc, torch.from_numpy(g["duration_pred"]).to(gpu))
    assert torch.equal(reg.cpu(), torch.from_numpy(g["regulated_output"]))  # pure copy: exact
    for dec in (m.decoder, standalone["decoder"]):
        assert maxabs(dec(reg), g["mel"]) <= MEL_MAXABS_TOL
    mel_bmt = torch.from_numpy(g["mel"]).to(gpu).transpose(1, 2).contiguous()
    for voc in (m.vocoder, standalone["vocoder"]):
        assert rms(voc(mel_bmt), g["audio"]) <= AUDIO_RMS_TOL


def test_components_api(gpu):
    """models.components used on their own (test_simple.py:49-63 pattern)."""
    from models.components import (FeedForward, MultiHeadAttention, PositionalEncoding, TransformerEncoderLayer,
                                   create_padding_mask)
    torch.manual_seed(0)
    H, heads, B, N = 64, 2, 2, 37
    pe = PositionalEncoding(H).to(gpu)
    x = torch.randn(B, N, H)
    assert maxabs(pe(x.to(gpu)), x + pe.pe[:, :N].cpu()) <= 1e-6
    mha = MultiHeadAttention(H, heads).eval()
    lens = torch.tensor([N, 20])
    mask = create_padding_mask(lens, N)
    sd = {f"a.{k}": v for k, v in mha.state_dict().items()}
    ref = orc.attention(sd, "a", x, heads, mask)
    got = mha.to(gpu)(x.to(gpu), mask.to(gpu))
    assert maxabs(got, ref) <= 1e-4
    ffn = FeedForward(H, 2 * H).eval()
    sd = {f"f.{k}": v for k, v in ffn.state_dict().items()}
    assert maxabs(ffn.to(gpu)(x.to(gpu)), orc.feed_forward(sd, "f", x)) <= 1e-4
    layer = TransformerEncoderLayer(H, heads, 2 * H).eval()
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    sd = {f"l.{k}": v.clone() for k, v in layer.state_dict().items()}
    assert maxabs(layer.to(gpu)(x.to(gpu), mask.to(gpu)), orc.encoder_layer(sd, "l", x, heads, mask)) <= 1e-4


def test_all_keys_masked_is_uniform(gpu):
    """Length-0 utterances: every key -1e9 -> softmax is uniform (reference behaviour)."""
    from models.components import MultiHeadAttention
    torch.manual_seed(1)
    mha = MultiHeadAttention(32, 2).eval()
    x = torch.randn(2, 9, 32)
    mask = torch.tensor([[False] * 9, [True] * 4 + [False] * 5])
    sd = {f"a.{k}": v for k, v in mha.state_dict().items()}
    assert maxabs(mha.to(gpu)(x.to(gpu), mask.to(gpu)), orc.attention(sd, "a", x, 2, mask)) <= 1e-5


def test_tiny_model_api(gpu):
    """test_simple.py:70-98 shape checks: hidden 32, heads 2 (hd 16), voc 64, max_target_length 30."""
    from models.tts_model import M2TTSModel
    torch.manual_seed(3)
    m = M2TTSModel(vocab_size=100, hidden_dim=32, mel_channels=32, text_encoder_layers=1, decoder_layers=1,
                   num_heads=2, vocoder_channels=64).eval()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    cfg = orc.OracleConfig(vocab_size=100, hidden_dim=32, mel_channels=32, text_encoder_layers=1,
                           decoder_layers=1, num_heads=2, vocoder_channels=64)
    ids = torch.randint(0, 100, (2, 10))
    lens = torch.tensor([8, 6])
    dur = torch.rand(2, 10) * 2 + 1
    ref = orc.forward(sd, cfg, ids, lens, dur, 30)
    out = m.to(gpu)(phoneme_ids=ids.to(gpu), phoneme_lengths=lens.to(gpu), target_durations=dur.to(gpu),
                    max_target_length=30)
    assert set(out) == set(ref)
    for k in ("encoder_output", "duration_pred", "regulated_output", "mel_output", "audio_output"):
        assert out[k].shape == ref[k].shape, k
    assert maxabs(out["mel_output"], ref["mel_output"]) <= MEL_MAXABS_TOL
    assert rms(out["audio_output"], ref["audio_output"]) <= AUDIO_RMS_TOL
    info = m.get_model_size()
    assert info["total_params"] == sum(p.numel() for p in m.parameters())


def test_cli_sentence_stage1(gpu):
    g = golden("cli_stage1")
    m = build_model("s1", gpu)
    ids, lens = _ids(g, gpu)
    mel, audio = m.inference(ids, lens)
    assert mel.shape == tuple(g["mel"].shape) == (1, 1280, 64)
    assert maxabs(mel, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio, g["audio"]) <= AUDIO_RMS_TOL


# ---------------------------------------------------------------------------
# Benchmark shapes: full tensors vs the oracle where it is quick
# on the host, fingerprints from the reference everywhere.
def _check_fingerprint(fp, mel, audio):
    B = audio.shape[0]
    a = audio[:, 0].double().cpu()
    assert mel.shape[1] == int(fp["T"][0])
    assert maxabs(audio[:, 0, :256], fp["audio_head"]) <= 1e-3
    assert maxabs(audio[:, 0, -256:], fp["audio_tail"]) <= 1e-3
    assert rms(audio[:, 0, :256], fp["audio_head"]) <= AUDIO_RMS_TOL
    n = a.shape[1]
    # sum of squares: |d(sumsq)| <= 2*sqrt(sumsq)*||err|| ~ 2*sqrt(n*ms)*sqrt(n)*rms_tol
    np.testing.assert_allclose(a.pow(2).sum(1).numpy(), fp["audio_sumsq"], rtol=2e-3, atol=n * 1e-6)
    np.testing.assert_allclose(a.abs().amax(1).numpy(), fp["audio_maxabs"], atol=1e-3)
    np.testing.assert_allclose(a.sum(1).numpy(), fp["audio_sum"], rtol=1e-4, atol=n * 1e-6)
    if "mel_head" in fp.files:
        assert maxabs(mel[:, :4], fp["mel_head"]) <= MEL_MAXABS_TOL
        assert maxabs(mel[:, -4:], fp["mel_tail"]) <= MEL_MAXABS_TOL
        m = mel.double().cpu().flatten(1)
        nm = m.shape[1]
        # whole-tensor mel statistics: a per-value error e moves the sum by <= nm*e
        # and the sum of squares by <= 2*sum|m|*e (observed e ~ 2e-6; bound at 1e-5)
        np.testing.assert_allclose(m.sum(1).numpy(), fp["mel_sum"], rtol=0, atol=nm * 1e-5)
        d_sq = np.abs(m.pow(2).sum(1).numpy() - fp["mel_sumsq"])
        assert np.all(d_sq <= (2 * m.abs().sum(1) * 1e-5).numpy()), d_sq.max()
        np.testing.assert_allclose(m.abs().amax(1).numpy(), fp["mel_maxabs"], rtol=0, atol=MEL_MAXABS_TOL)
    assert B == fp["audio_head"].shape[0]


def test_vocoder_stage1_b32_full(gpu):
    fp = golden("fp_s1_vocoder_B32_T500")
    m = build_model("s1", gpu)
    mel = torch.randn(32, 64, 500, generator=torch.Generator().manual_seed(int(fp["seed"])))
    audio = m.vocoder(mel.to(gpu))
    ref = orc.vocoder(golden_state("s1"), mel)
    assert audio.shape == (32, 1, 32000)
    assert rms(audio, ref) <= AUDIO_RMS_TOL
    assert maxabs(audio, ref) <= 1e-3
    assert maxabs(audio[:, 0, :256], fp["audio_head"]) <= 1e-3


@pytest.mark.parametrize("stage,B,S", [("s1", 32, 100), ("s2", 64, 100)])
def test_pipeline_bench_shapes(gpu, stage, B, S):
    fp = golden(f"fp_{stage}_B{B}_S{S}")
    m = build_model(stage, gpu)
    ids = torch.from_numpy(fp["ids"])
    lens = torch.from_numpy(fp["lengths"])
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    _check_fingerprint(fp, mel, audio)
    ref_mel, ref_audio = orc.inference(golden_state(stage), stage_config(stage), ids, lens, as_written=False)
    assert maxabs(mel, ref_mel) <= MEL_MAXABS_TOL
    assert rms(audio, ref_audio) <= AUDIO_RMS_TOL


def test_pipeline_longform_stage2(gpu):
    """B=128, S=520 -> T=2600 (30.2 s of mel at hop 256): fingerprints of all
    128 utterances, and full tensors of the first and last utterance against
    the oracle run on those two (every utterance has T=2600, so the two-row
    batch pads to the same global T as the 128-row one)."""
    fp = golden("fp_s2_B128_S520")
    m = build_model("s2", gpu)
    ids, lens = torch.from_numpy(fp["ids"]), torch.from_numpy(fp["lengths"])
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    assert audio.shape == (128, 1, 64 * 2600)
    _check_fingerprint(fp, mel, audio)
    rows = [0, 127]
    assert all(int(fp["T"][r]) == 2600 for r in rows)
    ref_mel, ref_audio = orc.inference(golden_state("s2"), stage_config("s2"), ids[rows], lens[rows], as_written=False)
    assert ref_mel.shape == (2, 2600, 80)
    assert maxabs(mel[rows], ref_mel) <= MEL_MAXABS_TOL
    assert rms(audio[rows], ref_audio) <= AUDIO_RMS_TOL
    assert maxabs(audio[rows], ref_audio) <= 1e-3


def test_repeatable_and_stream_ordered(gpu):
    """Same inputs twice -> bitwise identical outputs (no atomics in the data path)."""
    g = golden("s1_small")
    m = build_model("s1", gpu)
    ids, lens = _ids(g, gpu)
    a = m.inference(ids, lens)
    b = m.inference(ids, lens)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_weights_reload_invalidates_handle(gpu):
    g = golden("s1_small")
    m = build_model("s1", gpu)
    ids, lens = _ids(g, gpu)
    mel1, _ = m.inference(ids, lens)
    with torch.no_grad():
        m.decoder.mel_projection.bias.add_(1.0)
    mel2, _ = m.inference(ids, lens)
    assert maxabs(mel2 - 1.0, mel1) <= 1e-5


def test_cli_end_to_end_wav(gpu, tmp_path):
    """scripts/synthesize.py main(): checkpoint (trainer dict format) -> WAV.
    The PCM16 samples must equal the reference audio for the same sentence
    quantised the same way, up to 1 LSB where fp32 noise straddles a rounding
    boundary."""
    import sys
    from conftest import ROOT
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "scripts"))
    import synthesize
    from utils.audio import float_to_pcm16, load_audio_pcm16
    g = golden("cli_stage1")
    ck = tmp_path / "stage1.pt"
    cfg = {"model": {"text_encoder": {"vocab_size": 256, "hidden_dim": 64, "num_layers": 2, "num_heads": 2,
                                      "dropout": 0.1}, "decoder": {"mel_channels": 64, "num_layers": 2},
                     "vocoder": {"hidden_channels": 128}}}
    torch.save({"model_state_dict": golden_state("s1"), "config": cfg, "step": 1}, ck)
    out = tmp_path / "out.wav"
    synthesize.main(["--text", str(g["text"]), "--checkpoint", str(ck), "--output", str(out)])
    y, sr = load_audio_pcm16(out)
    want = float_to_pcm16(g["audio"][0, 0]).astype(np.int32)
    got = np.rint(y * 32768).astype(np.int32)
    assert sr == 22050 and got.shape == want.shape == (81920,)
    assert int(np.abs(got - want).max()) <= 1


@pytest.mark.parametrize("stage", STAGES)
def test_vocoder_arithmetic_paths(gpu, stage, monkeypatch):
    """Default = split-f16 MFMA (path 2); M2_VOC_F32=1 = exact-f32 MFMA (path 1).
    Both within the waveform bound of the CPU oracle, and close to each other."""
    from m2amd import _lib
    lib = _lib.load()
    mel = torch.randn(3, stage_config(stage).mel_channels, 137, generator=torch.Generator().manual_seed(7))
    ref = orc.vocoder(golden_state(stage), mel)
    out = {}
    for path, env in ((2, None), (1, "1")):
        if env is None:
            monkeypatch.delenv("M2_VOC_F32", raising=False)
        else:
            monkeypatch.setenv("M2_VOC_F32", env)
        m = build_model(stage, gpu)
        assert lib.m2_vocoder_path(m._hip(gpu).handle) == path
        out[path] = m.vocoder(mel.to(gpu)).cpu()
        assert rms(out[path], ref) <= AUDIO_RMS_TOL
        assert maxabs(out[path], ref) <= 1e-4
    assert maxabs(out[1], out[2]) <= 1e-4


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("env", ["M2_TF_UNFUSED", "M2_VOCODER_PERLAYER", "M2_VOC_TAIL_X3", "M2_VOC_MID_X3",
                                 "M2_ATT_F32"])
def test_alternate_kernel_paths(gpu, stage, env, monkeypatch):
    """The unfused transformer layer (five linears), the per-layer vocoder
    kernels, the x3 tail / mid kernels (instead of the pipelined stage1 ones)
    and the exact-f32 attention stay parity-green: inference vs the
    reference's fixture."""
    monkeypatch.setenv(env, "1")
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = _ids(g, gpu)
    mel, audio = m.inference(ids, lens)
    assert maxabs(mel, g["mel"]) <= MEL_MAXABS_TOL
    assert rms(audio, g["audio"]) <= AUDIO_RMS_TOL


def test_profile_events_strided(gpu):
    """bench.py's roofline events: a stride-k sample of the m2_vocoder calls
    records one event pair per selected kernel on every k-th call only."""
    import ctypes
    from m2amd import _lib
    lib = _lib.load()
    m = build_model("s1", gpu)
    mel = torch.randn(2, 64, 40, device=gpu)
    h = m._hip(gpu).handle
    nk = lib.m2_profile_kernel_count()
    _lib.check(lib.m2_profile_select(h, 1 << 2), "select")
    _lib.check(lib.m2_profile_stride(h, 3), "stride")
    _lib.check(lib.m2_profile_enable(h, 3), "enable")
    for _ in range(7):  # calls 0, 3, 6 record
        m.vocoder(mel)
    buf = (ctypes.c_float * (3 * nk))()
    n = ctypes.c_int32(0)
    _lib.check(lib.m2_profile_read(h, buf, 3 * nk, ctypes.byref(n)), "read")
    lib.m2_profile_disable(h)
    _lib.check(lib.m2_profile_stride(h, 1), "stride")
    ms = list(buf[: n.value])
    assert n.value == 3 * nk
    assert all(v > 0 for v in ms[2::nk]) and all(v < 0 for i, v in enumerate(ms) if i % nk != 2)
    assert lib.m2_profile_stride(h, 0) != 0  # bad stride is an error, not a crash


@pytest.mark.parametrize("B,S", [(1, 7), (3, 100), (300, 40)])
def test_frame_counts_sync_mailbox(gpu, B, S):
    """m2_length_regulator_count_sync (the host-mapped T_max mailbox) against
    the plain count kernel and the reference's int(d.item()) loop (oracle),
    over repeated calls (the mailbox sequence and the ticket reset), B > 256
    (the last workgroup's reduction loop), zero / negative / fractional
    durations and a duration scale."""
    from m2amd import ops
    g = torch.Generator().manual_seed(B * 1000 + S)
    for it in range(3):
        d = (torch.rand(B, S, generator=g) * 12 - 2).to(torch.float32)
        if it == 1:
            d[0] = 0.0  # an utterance with no frames
        scale = 1.0 if it < 2 else 1.3
        dg = d.to(gpu)
        cum, tot, tmax, t_host = ops.frame_counts_sync(dg, scale)
        cum0, tot0, tmax0 = ops.frame_counts(dg, scale)
        assert torch.equal(cum, cum0) and torch.equal(tot, tot0)
        assert int(tmax.item()) == int(tmax0.item()) == t_host
        n = [[max(0, int(float(np.float32(v) * np.float32(scale)))) for v in row] for row in d.numpy()]
        assert t_host == max(sum(r) for r in n)
        enc = torch.randn(B, S, 8, generator=g)
        ref = orc.length_regulator(enc, d * scale if scale != 1.0 else d)
        out = ops.regulate(enc.to(gpu), dg, None, scale=scale)
        assert out.shape == ref.shape and torch.equal(out.cpu(), ref)


def test_frame_counts_sync_empty_batch(gpu):
    from m2amd import ops
    cum, tot, tmax, t_host = ops.frame_counts_sync(torch.zeros(0, 5, device=gpu), 1.0)
    assert t_host == 0 and int(tmax.item()) == 0


@pytest.mark.parametrize("stage", STAGES)
def test_inference_single_call_capacity(gpu, stage):
    """M2TTSModel.inference through m2_inference: the first call for a (B, S)
    has no frame capacity (front call + m2_inference_back), later calls with
    the same or fewer frames run in one call into capacity-sized buffers, a
    longer request (duration_scale) overflows the capacity and falls back.
    Every result matches the fixtures and the staged six-call path bit for bit,
    and earlier results are not overwritten by later calls."""
    from m2amd import ops
    gs, gc = golden(f"{stage}_small"), golden(f"{stage}_scale")
    m = build_model(stage, gpu)
    g = gs
    ids, lens = _ids(g, gpu)
    hm = m._hip(gpu)

    def staged(scale):
        enc, _ = hm.text_encoder(ids, lens)
        reg = ops.regulate(enc, hm.duration(enc), None, scale=scale)
        mel = hm.decoder(reg)
        return mel, hm.vocoder(mel, layout_btm=True)

    plan = [(g, 1.0), (g, 1.0), (gc, float(gc["duration_scale"])), (g, 1.0), (gc, float(gc["duration_scale"]))]
    kept = []
    for fx, scale in plan:
        fids, flens = _ids(fx, gpu)
        assert torch.equal(fids, ids) and torch.equal(flens, lens)
        mel, audio = m.inference(ids, lens, duration_scale=scale)
        assert mel.is_contiguous() and audio.is_contiguous()
        assert mel.shape == tuple(fx["mel"].shape) and audio.shape == tuple(fx["audio"].shape)
        assert maxabs(mel, fx["mel"]) <= MEL_MAXABS_TOL
        assert rms(audio, fx["audio"]) <= AUDIO_RMS_TOL
        smel, saudio = staged(scale)
        assert torch.equal(mel, smel) and torch.equal(audio, saudio)
        kept.append((mel, audio, mel.clone(), audio.clone()))
    for mel, audio, mel0, audio0 in kept:
        assert torch.equal(mel, mel0) and torch.equal(audio, audio0)
    caps = hm._tcap[tuple(ids.shape)]
    assert caps >= max(k[0].shape[1] for k in kept)


def test_inference_single_call_empty(gpu):
    """B = 0 and all-zero durations (one zero frame) through m2_inference."""
    m = build_model("s1", gpu)
    mel, audio = m.inference(torch.zeros(0, 7, dtype=torch.long, device=gpu))
    assert mel.shape == (0, 1, stage_config("s1").mel_channels) and audio.shape == (0, 1, 64)


def test_inference_many_utterances(gpu):
    """m2_inference against the staged six-call path, bit for bit, for B > 256
    (several count workgroups per ticket round, 14-phoneme duration tiles with
    a ragged last tile), repeated calls, ragged lengths, a duration scale."""
    from m2amd import ops
    m = build_model("s1", gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(7)
    for B, S, scale in ((300, 20, 1.0), (300, 20, 1.7), (5, 37, 1.0), (300, 20, 1.0)):
        ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
        lens = torch.randint(1, S + 1, (B,), generator=g).to(gpu)
        mel, audio = m.inference(ids, lens, duration_scale=scale)
        enc, _ = hm.text_encoder(ids, lens)
        reg = ops.regulate(enc, hm.duration(enc), None, scale=scale)
        smel = hm.decoder(reg)
        assert torch.equal(mel, smel)
        assert torch.equal(audio, hm.vocoder(smel, layout_btm=True))


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("T", [1, 37, 500])
def test_vocoder_mel_layouts_identical(gpu, stage, T):
    """The vocoder reading the decoder's [B,T,M] mel in place (inference path)
    and the module's own [B,M,T] input give identical audio, including ragged
    tiles (T not a multiple of the head's frame window) and T = 1."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(T)
    mel_btm = torch.randn(3, T, stage_config(stage).mel_channels, generator=g).to(gpu)
    a = hm.vocoder(mel_btm, layout_btm=True)
    b = hm.vocoder(mel_btm.transpose(1, 2).contiguous(), layout_btm=False)
    assert torch.equal(a, b)
