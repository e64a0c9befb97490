"""CPU oracle vs the reference's golden fixtures (tests/golden/make_golden.py).

The oracle restates the reference forward with the same ATen ops; on the
build container it matched the reference bit for bit (manifest.json).  Here
it is checked against the committed outputs with a small tolerance, since a
different host CPU may reorder fp32 sums in MKL/oneDNN.
"""
import json

import numpy as np
import pytest
import torch

import m2tts_oracle as orc
from conftest import GOLDEN, golden, golden_state, maxabs, stage_config

TOL = 2e-5
STAGES = ["s1", "s2"]


def test_manifest_records_bitwise_agreement():
    man = json.loads((GOLDEN / "manifest.json").read_text())
    for case in man["cases"].values():
        for v in case.get("oracle_vs_ref_maxabs", {}).values():
            assert v == 0.0


@pytest.mark.parametrize("stage", STAGES)
def test_small_forward_and_inference(stage):
    g = golden(f"{stage}_small")
    sd, cfg = golden_state(stage), stage_config(stage)
    ids, lens = torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"])
    out = orc.forward(sd, cfg, ids, lens)
    for k, gk in (("encoder_output", "encoder_output"), ("duration_pred", "duration_pred"),
                  ("regulated_output", "regulated_output"), ("mel_output", "mel"), ("audio_output", "audio")):
        assert tuple(out[k].shape) == g[gk].shape
        assert maxabs(out[k], g[gk]) <= TOL, k
    assert torch.equal(out["padding_mask"], torch.from_numpy(g["padding_mask"]))
    mel, audio = orc.inference(sd, cfg, ids, lens)
    assert maxabs(mel, g["mel"]) <= TOL and maxabs(audio, g["audio"]) <= TOL
    # the pinned durations stay far from the int() discontinuity
    d = out["duration_pred"]
    assert float((d - d.round()).abs().min()) > 0.4


@pytest.mark.parametrize("stage", STAGES)
@pytest.mark.parametrize("sub", ["free", "pad", "trunc"])
def test_teacher_forced(stage, sub):
    g = golden(f"{stage}_target_{sub}")
    mtl = int(g["max_target_length"])
    out = orc.forward(golden_state(stage), stage_config(stage), torch.from_numpy(g["ids"]),
                      torch.from_numpy(g["lengths"]), torch.from_numpy(g["target_durations"]),
                      None if mtl < 0 else mtl)
    assert torch.equal(out["regulated_output"], torch.from_numpy(g["regulated_output"])) or \
        maxabs(out["regulated_output"], g["regulated_output"]) <= TOL
    assert maxabs(out["mel_output"], g["mel"]) <= TOL
    assert maxabs(out["audio_output"], g["audio"]) <= TOL


@pytest.mark.parametrize("stage", STAGES)
def test_duration_scale_and_untrained(stage):
    g = golden(f"{stage}_scale")
    mel, audio = orc.inference(golden_state(stage), stage_config(stage), torch.from_numpy(g["ids"]),
                               torch.from_numpy(g["lengths"]), duration_scale=float(g["duration_scale"]))
    assert mel.shape == g["mel"].shape and maxabs(mel, g["mel"]) <= TOL and maxabs(audio, g["audio"]) <= TOL
    g = golden(f"{stage}_untrained")
    mel, audio = orc.inference(golden_state(stage, pinned=False), stage_config(stage), torch.from_numpy(g["ids"]),
                               torch.from_numpy(g["lengths"]))
    assert mel.shape[1] == 1  # every int(duration) == 0 -> one zero frame
    assert maxabs(mel, g["mel"]) <= TOL and maxabs(audio, g["audio"]) <= TOL


@pytest.mark.parametrize("stage", STAGES)
def test_vocoder_layers(stage):
    sd = golden_state(stage)
    g = golden(f"{stage}_input_conv")
    y = torch.nn.functional.conv1d(torch.from_numpy(g["x"]), sd["vocoder.input_conv.weight"], sd["vocoder.input_conv.bias"], padding=1)
    assert maxabs(y, g["y"]) <= TOL
    for k in range(4):
        g = golden(f"{stage}_convT{k}")
        y = torch.nn.functional.leaky_relu(orc.conv_transpose(sd, f"vocoder.upsamples.{k}", torch.from_numpy(g["x"]),
                                                              int(g["rate"])), 0.1)
        assert maxabs(y, g["y"]) <= TOL
        g = golden(f"{stage}_resblock{k}")
        assert maxabs(orc.resblock(sd, f"vocoder.resblocks.{k}", torch.from_numpy(g["x"])), g["y"]) <= TOL


def test_fingerprint_stage1_b32():
    fp = golden("fp_s1_B32_S100")
    mel, audio = orc.inference(golden_state("s1"), orc.STAGE1, torch.from_numpy(fp["ids"]),
                               torch.from_numpy(fp["lengths"]), as_written=False)
    assert mel.shape[1] == int(fp["T"][0]) == 500
    assert maxabs(audio[:, 0, :256], fp["audio_head"]) <= TOL
    assert maxabs(audio[:, 0, -256:], fp["audio_tail"]) <= TOL
    np.testing.assert_allclose(audio[:, 0].double().pow(2).sum(1).numpy(), fp["audio_sumsq"], rtol=1e-5)


def test_fingerprint_stage1_vocoder_b32():
    fp = golden("fp_s1_vocoder_B32_T500")
    mel = torch.randn(32, 64, 500, generator=torch.Generator().manual_seed(int(fp["seed"])))
    audio = orc.vocoder(golden_state("s1"), mel)
    assert maxabs(audio[:, 0, :256], fp["audio_head"]) <= TOL
    np.testing.assert_allclose(audio[:, 0].double().sum(1).numpy(), fp["audio_sum"], rtol=1e-4, atol=1e-3)


def test_cli_sentence_fixture():
    g = golden("cli_stage1")
    mel, audio = orc.inference(golden_state("s1"), orc.STAGE1, torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"]))
    assert mel.shape == (1, 1280, 64) and audio.shape == (1, 1, 81920)
    assert maxabs(audio, g["audio"]) <= TOL


def test_length_regulator_edge_cases():
    enc = torch.arange(2 * 3 * 2, dtype=torch.float32).reshape(2, 3, 2)
    dur = torch.tensor([[0.9, 2.7, -1.0], [0.0, 0.0, 0.0]])
    out = orc.length_regulator(enc, dur)
    assert out.shape == (2, 2, 2)                       # max(2, 1 zero frame)
    assert torch.equal(out[0], enc[0, 1].repeat(2, 1))  # int(0.9)=0, int(2.7)=2, negative skipped
    assert torch.equal(out[1], torch.zeros(2, 2))
    assert orc.length_regulator(enc, dur, max_length=1).shape == (2, 1, 2)
