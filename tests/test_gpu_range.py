"""GPU: the split-f16 range guard.  Values of magnitude >= 65520 (mel input or
any vocoder activation) make the split path's audio non-finite, which its last
kernel flags; the "fallback" policy recomputes such a call on the exact-f32
kernels, "report" raises on the next call / check_numerics().  Tiny inputs
(f16-subnormal lo halves) stay within the waveform bound.  Transformer
activations are bounded by the weights and checked at model creation."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, MEL_MAXABS_TOL, golden, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def build_model(stage, dev, sd=None):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config(stage).as_dict())
    m.load_state_dict(sd if sd is not None else golden_state(stage))
    return m.to(dev).eval()


def _mel(stage, T, scale, seed=5):
    return torch.randn(2, stage_config(stage).mel_channels, T, generator=torch.Generator().manual_seed(seed)) * scale


# The fallback's recomputation: the pipelined tails (stage1 tailp, stage2
# tailp2) redo their own non-finite strips in fp32 inside the launch
# (vocoder_redo.h; direct convolutions, another fp32 summation order than the
# exact-f32 kernels); the guarded exact-f32 launch (M2_REDO_LAUNCH=1, or a
# model without a pipelined tail) is bit-equal to those kernels.  Inputs that
# overflow the split range are far outside the reference's normalised mel
# range, and there the audio is ill-conditioned: activations of ~1e5 stored
# in fp32 carry ~1e-2 of rounding each, which reaches the audio near tanh's
# zero crossings.  So such outputs are checked against a float64 evaluation
# of the reference's op sequence, within the distance the reference's own
# fp32 CPU path (the oracle) lands from it on the same input (at least the
# 1e-4 waveform bound).
def _assert_like_reference(out, sd, mel_bmt):
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    ref64 = orc.vocoder(sd64, mel_bmt.double())
    cond = rms(orc.vocoder(sd, mel_bmt), ref64)  # the reference's fp32 path on this input
    assert rms(out, ref64) <= max(AUDIO_RMS_TOL, 2 * cond), (rms(out, ref64), cond)


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_huge_mel_fallback_matches_exact_f32_and_oracle(gpu, stage):
    mel = _mel(stage, 45, 1e5)
    assert float(mel.abs().max()) > 65520
    m = build_model(stage, gpu)
    m.set_range_policy("fallback")
    out = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    _assert_like_reference(out, golden_state(stage), mel)
    m.set_vocoder_precision("f32")
    _assert_like_reference(m.vocoder(mel.to(gpu)), golden_state(stage), mel)  # the exact-f32 kernels alike


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_local_redo_only_touches_non_finite_strips(gpu, stage):
    """One utterance with an out-of-range stretch (frames 30-33 of
    70): the other utterance's audio is the split path's, bit for bit; the
    overflowing one matches the reference's op sequence (float64) as closely
    as the reference's own fp32 path does."""
    mel = _mel(stage, 70, 1.0)
    clean = mel.clone()
    mel[0, :, 30:34] *= 1e6
    m = build_model(stage, gpu)
    m.set_range_policy("report")
    split_clean = m.vocoder(clean.to(gpu))
    m.set_range_policy("fallback")
    out = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    assert torch.equal(out[1], split_clean[1])
    _assert_like_reference(out, golden_state(stage), mel)
    m.check_numerics()


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_guarded_launch_still_available(gpu, monkeypatch, stage):
    """M2_REDO_LAUNCH=1 keeps the guarded exact-f32 launch behind the split
    kernels (no local redo): the fallback equals the exact-f32 audio."""
    monkeypatch.setenv("M2_REDO_LAUNCH", "1")
    mel = _mel(stage, 45, 1e5)
    m = build_model(stage, gpu)
    m.set_range_policy("fallback")
    out = m.vocoder(mel.to(gpu))
    m.set_vocoder_precision("f32")
    assert torch.equal(out, m.vocoder(mel.to(gpu)))


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_huge_mel_report_raises(gpu, stage):
    from m2amd._lib import M2Error
    m = build_model(stage, gpu)
    m.set_range_policy("report")  # opt-in (the default is "fallback")
    ok = _mel(stage, 30, 1.0)
    base = m.vocoder(ok.to(gpu))
    bad = m.vocoder(_mel(stage, 30, 1e6).to(gpu))
    with pytest.raises(M2Error, match="non-finite"):
        m.check_numerics("cuda")  # an unindexed device names the current one
    m.check_numerics()  # cleared
    assert torch.equal(m.vocoder(ok.to(gpu)), base)
    m.vocoder(_mel(stage, 30, 1e6).to(gpu))
    torch.cuda.synchronize()
    with pytest.raises(M2Error, match="status -6"):  # M2_E_RANGE on the next call
        m.vocoder(ok.to(gpu))
    assert torch.equal(m.vocoder(ok.to(gpu)), base)
    del bad


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_huge_activation_inside_the_vocoder(gpu, stage):
    """A finite mel, but input_conv's bias puts its activations near 1e5: the
    split path flags it and the fallback's fp32 recomputation matches the
    reference's op sequence (as closely as the reference's fp32 path does)."""
    sd = golden_state(stage)
    sd["vocoder.input_conv.bias"] = sd["vocoder.input_conv.bias"] + 1e5
    m = build_model(stage, gpu, sd)
    assert m._hip(gpu).vocoder_path() == 2  # weights themselves stay in the f16 range
    mel = _mel(stage, 33, 1.0)
    m.set_range_policy("fallback")
    out = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    _assert_like_reference(out, sd, mel)


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_default_policy_inference_never_nan(gpu, stage):
    """Without any policy call, inference() on weights whose vocoder
    activations overflow the split-f16 range returns the exact-f32 result
    (the reference's), in the same call - never non-finite audio."""
    sd = golden_state(stage)
    sd["vocoder.input_conv.bias"] = sd["vocoder.input_conv.bias"] + 1e5
    m = build_model(stage, gpu, sd)
    g = golden(f"{stage}_small")
    ids, lens = torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"])
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    assert torch.isfinite(audio).all()
    ref_mel, _ = orc.inference(sd, stage_config(stage), ids, lens, as_written=False)
    assert maxabs(mel, ref_mel) <= MEL_MAXABS_TOL
    # the second call of the shape runs the speculative back half (T from the
    # device, the redo kernels sized for the capacity): the same audio
    mel2, audio2 = m.inference(ids.to(gpu), lens.to(gpu))
    assert torch.equal(mel2, mel) and torch.equal(audio2, audio)
    _assert_like_reference(audio, sd, mel.transpose(1, 2).cpu())
    m.check_numerics()  # nothing left pending


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_fallback_on_device_alternating_calls(gpu, stage):
    """The "fallback" policy's on-device redo (two flag words used by
    alternate calls, the next call's head kernel zeroing the other): any
    sequence of overflowing and ordinary calls gives, call by call, the
    exact-f32 audio for the former and the split-path audio for the latter,
    with nothing left pending."""
    ok, bad = _mel(stage, 30, 1.0).to(gpu), _mel(stage, 30, 1e6, seed=6).to(gpu)
    ref = build_model(stage, gpu)
    ref.set_range_policy("report")
    split_ok = ref.vocoder(ok)
    m = build_model(stage, gpu)
    m.set_range_policy("fallback")
    first_bad = None
    for x in ("bad", "ok", "bad", "bad", "ok", "ok", "bad", "ok"):
        out = m.vocoder(bad if x == "bad" else ok)
        if x == "ok":
            assert torch.equal(out, split_ok), x
        elif first_bad is None:
            _assert_like_reference(out, golden_state(stage), bad.cpu())
            first_bad = out
        else:
            assert torch.equal(out, first_bad)  # deterministic
    torch.cuda.synchronize()
    m.check_numerics()


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_fallback_on_device_chunked(gpu, stage):
    """Streamed (chunked) vocoding with an overflowing stretch in one window:
    finite audio within the waveform bound of the oracle."""
    mel = _mel(stage, 70, 1.0)
    mel[:, :, 30:34] *= 1e6
    m = build_model(stage, gpu)
    m.set_range_policy("fallback")
    m.set_vocoder_chunking(16)
    out = m.vocoder(mel.to(gpu))
    assert torch.isfinite(out).all()
    _assert_like_reference(out, golden_state(stage), mel)
    m.check_numerics()


@pytest.mark.parametrize("stage", ["s1", "s2"])
@pytest.mark.parametrize("scale", [1e-3, 1e-6])
def test_tiny_mel_within_bound(gpu, stage, scale):
    """Mel values whose lo halves are f16 subnormals (or zero): the absolute
    error stays far inside the waveform bound and nothing is flagged."""
    m = build_model(stage, gpu)
    mel = _mel(stage, 64, scale)
    out = m.vocoder(mel.to(gpu))
    ref = orc.vocoder(golden_state(stage), mel)
    assert rms(out, ref) <= AUDIO_RMS_TOL and maxabs(out, ref) <= 1e-4
    m.check_numerics()


def test_transformer_range_bound_selects_f32(gpu):
    """Decoder LayerNorm gains of 1e3 push q/k/v past half the f16 range: the
    model is created on the fp32 transformer path and still matches the oracle."""
    from m2amd import _lib
    lib = _lib.load()
    sd = golden_state("s1")
    assert lib.m2_transformer_path(build_model("s1", gpu, sd)._hip(gpu).handle) == 1
    sd["decoder.layers.0.norm1.weight"] = sd["decoder.layers.0.norm1.weight"] * 1e3
    m = build_model("s1", gpu, sd)
    assert lib.m2_transformer_path(m._hip(gpu).handle) == 0
    g = golden("s1_small")
    ids, lens = torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"])
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    ref_mel, ref_audio = orc.inference(sd, orc.STAGE1, ids, lens, as_written=False)
    assert maxabs(mel, ref_mel) <= MEL_MAXABS_TOL
    assert rms(audio, ref_audio) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", ["s1", "s2"])
@pytest.mark.parametrize("scale", [0.3, 10.0])
@pytest.mark.parametrize("rb,form", [("1", "auto"), ("2", "auto"), ("4", "auto"), ("4", "3"), ("4", "4"),
                                     ("4", "12")])
def test_attention_scores_large(gpu, monkeypatch, stage, scale, rb, form):
    """Decoder layer 0 with every q and k row = scale u (q_d = k_d = scale
    u.LN1(x)): attention scores spread over > 128 log2 units (scale 0.3) or
    past the f16 maximum (scale 10, with q / k still inside the split range,
    so the creation-time activation bound passes).  The 64-row query-split
    forms (M2_TFL_RB=4) keep an unnormalised base and move it only when a
    weight's f16 hi half exceeds 2^8 - a later chunk scoring more than 16
    above the base makes that hi half +inf, which the move must catch (a
    float compare of packed f16 maxima missed it: NaN output).  At scale 10
    the head_dim-48 default form, whose base is an f16 pair, gives way to
    the f32-base form (m2_transformer_path 2).  "auto" is the
    default (12 on unmasked layers at both head dims), "3" / "4" the lean two- /
    one-block forms, "12" the key-quarter form (base an f16 pair at
    head_dim 48).  M2_TFL_RB=1 / 2 run the same layer on the 16- / 32-row
    tile forms (attention_tile), whose softmax base is fp32 in every form
    (the wide-score claim is checked on every tile form)."""
    from m2amd import _lib
    import torch.nn.functional as F
    lib = _lib.load()
    monkeypatch.setenv("M2_TFL_RB", rb)  # 16- / 32-row tiles, or 64-row query-split tiles
    if form != "auto":
        monkeypatch.setenv("M2_TFL_QS2", form)
    cfg = stage_config(stage)
    H, hd = cfg.hidden_dim, cfg.hidden_dim // 2
    sd = golden_state(stage)
    w = sd["decoder.layers.0.self_attn.qkv.weight"].clone()
    u = torch.randn(H, generator=torch.Generator().manual_seed(3))
    w[: 2 * H] = scale * u
    sd["decoder.layers.0.self_attn.qkv.weight"] = w
    x = torch.randn(2, 300, H, generator=torch.Generator().manual_seed(4))
    xn = F.layer_norm(x, (H,), sd["decoder.layers.0.norm1.weight"], sd["decoder.layers.0.norm1.bias"])
    q = xn @ w[:hd].T
    sc = (q @ q.transpose(1, 2)) / hd ** 0.5 * 1.4426950408889634  # log2 units, as the kernels see them
    assert float((sc.amax(-1) - sc.amin(-1)).amax()) > 128
    m = build_model(stage, gpu, sd)
    if scale > 1:
        assert float(sc.amax()) > 65520
        assert lib.m2_transformer_path(m._hip(gpu).handle) == 2
        assert lib.m2_transformer_path(build_model(stage, gpu)._hip(gpu).handle) == 1
    mel = m.decoder(x.to(gpu))
    assert torch.isfinite(mel).all()
    assert maxabs(mel, orc.mel_decoder(sd, cfg, x)) <= MEL_MAXABS_TOL


def test_frame_count_overflow_is_an_error(gpu):
    """Per-phoneme counts clamp at 2^30 and the sums are 64-bit and saturating:
    a total past the 2^24-frame limit is M2_E_SHAPE, never a wrapped int32."""
    from m2amd import ops
    from m2amd._lib import M2Error
    d = torch.full((2, 100), 1e9, device=gpu)
    cum, tot, tmax = ops.frame_counts(d)
    assert int(tot.min()) == 2**31 - 1 and int(tmax.item()) == 2**31 - 1  # saturated, not wrapped
    assert int(cum[0, 2]) == 2_000_000_000 and int(cum[0, -1]) == 2**31 - 1
    with pytest.raises(M2Error, match="status -2"):
        ops.regulate(torch.zeros(2, 100, 8, device=gpu), d)
    m = build_model("s1", gpu)
    g = golden("s1_small")
    with pytest.raises(M2Error, match="status -2"):
        m.inference(torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu), duration_scale=1e7)
    mel, _ = m.inference(torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu))
    assert mel.shape == tuple(g["mel"].shape)  # the mailbox protocol is intact after the error
    # with a capacity learnt the back half is launched before the count is
    # known: the overflowing call still raises (its launches did nothing) and
    # the next call is intact
    with pytest.raises(M2Error, match="status -2"):
        m.inference(torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu), duration_scale=1e7)
    mel2, _ = m.inference(torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu))
    assert torch.equal(mel2, mel)
