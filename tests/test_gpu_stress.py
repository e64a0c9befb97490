"""GPU: inference() with every linear / conv weight of the seeded model scaled
up (trained checkpoints carry larger weights than the seeded init, and none
exists in the reference to test with), against the CPU oracle (the
reference's op sequence, tts_model.py:350-438).  Larger weights sharpen the
attention (score ranges of hundreds of log2 units: the lean softmax's base
moves past +inf weights), push activations toward and past the split-f16
range (the creation-time bounds move the transformer to its fp32 path, the
vocoder's range policy recomputes non-finite strips in fp32), and the
result must stay finite and match the oracle.  The duration projection is
zeroed (every duration softplus(5.5), 0.49 from an integer) so the frame
counts cannot flip between the two paths.

Tolerances: mel max-abs 1e-3 relative to the oracle mel's magnitude (the
north-star bound is absolute at the reference's unit-scale outputs; scaled
weights scale the mel); audio against a float64 evaluation of the
reference's vocoder on the oracle mel, within the distance the reference's
own fp32 path lands from it (at least 1e-4 RMS).

Samples more than 1e-2 from float64 (a tanh sign flip) are accounted for,
not tolerated (tools/probe/stress_flips.py,
profiles/r06/r06h_flips_x{2,4}.txt): their number per case is asserted exactly,
and each must sit where fp32 itself is ill-conditioned - its float64
pre-tanh value within 8x the error the reference's own fp32 path makes in
the pre-tanh signal near it.  At x4 the vocoder's activations reach ~3e8,
far past the split-f16 range (65520): every strip of the split path is
non-finite and the default range policy recomputes all of it in fp32 inside
the tail launch (vocoder_redo.h).  stage1 x4 has exactly one such sample,
[3, 0, 6547]: float64 pre-tanh 64.1 where the fp32 oracle's own pre-tanh
error is 13.7; the redo and the exact-f32 kernels both flip it, the fp32
oracle (another summation order) does not.  stage2 x4 and both x2 cases
have none."""
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, MEL_MAXABS_TOL, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def scaled_state(stage, f):
    sd = dict(golden_state(stage))
    for k, v in sd.items():
        if k.endswith(".weight") and v.dim() >= 2:  # Linear / Conv / ConvT (not norms, not embeddings' rows)
            sd[k] = v * f
    p = "duration_predictor.predictor.projection"
    sd[p + ".weight"] = torch.zeros_like(sd[p + ".weight"])
    sd[p + ".bias"] = torch.full_like(sd[p + ".bias"], 5.5)
    return sd


# samples that land > 1e-2 from float64 (tanh sign flips at ill-conditioned
# zero crossings), per (stage, weight scale): see the module docstring
FAR_SAMPLES = {("s1", 2.0): 0, ("s2", 2.0): 0, ("s1", 4.0): 1, ("s2", 4.0): 0}


@pytest.mark.parametrize("stage", ["s1", "s2"])
@pytest.mark.parametrize("f", [2.0, 4.0])
def test_scaled_weights_inference(gpu, stage, f):
    from models.tts_model import M2TTSModel
    cfg = stage_config(stage)
    sd = scaled_state(stage, f)
    m = M2TTSModel(**cfg.as_dict())
    m.load_state_dict(sd)
    m = m.to(gpu).eval()
    g = torch.Generator().manual_seed(int(11 * f) + (0 if stage == "s1" else 1))
    ids = torch.randint(0, 42, (5, 70), generator=g)
    lens = torch.randint(20, 71, (5,), generator=g)
    lens[0] = 70
    mel, audio = m.inference(ids.to(gpu), lens.to(gpu))
    ref_mel, _ = orc.inference(sd, cfg, ids, lens, as_written=False)
    assert mel.shape == ref_mel.shape
    assert torch.isfinite(mel).all() and torch.isfinite(audio).all()
    scale = max(1.0, float(ref_mel.abs().max()))
    assert maxabs(mel, ref_mel) <= MEL_MAXABS_TOL * scale, (maxabs(mel, ref_mel), scale)
    mel_bmt = ref_mel.transpose(1, 2)
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    ref64 = orc.vocoder(sd64, mel_bmt.double())
    cond = rms(orc.vocoder(sd, mel_bmt), ref64)
    # the GPU vocoder on the oracle's mel (so mel differences do not enter)
    out = m.vocoder(mel_bmt.to(gpu)).cpu().double()
    assert torch.isfinite(out).all()
    far = (out - ref64).abs() > 1e-2
    assert int(far.sum()) == FAR_SAMPLES[(stage, f)], far.nonzero().tolist()
    if far.any():
        pre64 = orc.vocoder_pre_tanh(sd64, mel_bmt.double())
        err32 = (orc.vocoder_pre_tanh(sd, mel_bmt).double() - pre64).abs()
        err32 = torch.nn.functional.max_pool1d(err32, 65, stride=1, padding=32)  # fp32's error near each sample
        assert (pre64.abs()[far] <= 8 * err32[far]).all(), (pre64[far], err32[far])
    assert rms(out[~far], ref64[~far]) <= max(AUDIO_RMS_TOL, 2 * cond), (rms(out[~far], ref64[~far]), cond)
    # inference()'s audio is the same vocoder on the GPU's own mel
    assert torch.equal(audio, m.vocoder(mel.transpose(1, 2).contiguous()))
