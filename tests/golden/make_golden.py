#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference implementation.

Run in the survey/build container only (it imports the read-only reference
at /root/reference, which does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does
  1. builds the reference ``M2TTSModel`` for stage1/stage2 with
     ``torch.manual_seed(1234)`` (SURVEY.md 8c recipe) and pins durations to
     5.5 (projection weight *0.01, bias 5.5) -> T = 5*S;
  2. checks the oracle (oracle/m2tts_oracle.py) against the reference on every
     case below and records the max-abs difference (expected: 0, same ATen ops);
  3. writes inputs + reference outputs as npz/json fixtures into this
     directory.  Only data is written - no reference source.
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF_SRC = Path("/root/reference/src")
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REF_SRC))

import m2tts_oracle as orc  # noqa: E402
from models.tts_model import M2TTSModel as RefModel  # noqa: E402  (reference)
from utils.text import TextProcessor as RefTextProcessor  # noqa: E402  (reference)

torch.set_num_threads(8)
MANIFEST = {"torch": torch.__version__, "cases": {}}


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def build(cfg: orc.OracleConfig):
    torch.manual_seed(1234)
    m = RefModel(**cfg.as_dict())
    m.eval()
    sd_raw = {k: v.detach().clone() for k, v in m.state_dict().items()}
    sd = orc.pin_durations(sd_raw)
    m.load_state_dict(sd)
    return m, sd, sd_raw


def maxdiff(a, b):
    if a is None and b is None:
        return 0.0
    return float((a.float() - b.float()).abs().max()) if a.numel() else 0.0


def save(name, **arrays):
    np.savez_compressed(HERE / f"{name}.npz", **{k: (v if isinstance(v, np.ndarray) else np.asarray(v)) for k, v in arrays.items()})


def fingerprint(mel, audio, t_per_utt):
    """Size-independent per-utterance summaries (SURVEY.md 8c fingerprints)."""
    a = audio[:, 0].double()
    m = mel.double()
    return dict(
        T=np.asarray(t_per_utt, np.int32),
        mel_sum=m.sum(dim=(1, 2)).numpy(), mel_sumsq=(m * m).sum(dim=(1, 2)).numpy(),
        mel_maxabs=m.abs().amax(dim=(1, 2)).numpy(),
        audio_sum=a.sum(dim=1).numpy(), audio_sumsq=(a * a).sum(dim=1).numpy(),
        audio_maxabs=a.abs().amax(dim=1).numpy(),
        audio_head=np32(audio[:, 0, :256]), audio_tail=np32(audio[:, 0, -256:]),
        mel_head=np32(mel[:, :4, :]), mel_tail=np32(mel[:, -4:, :]),
    )


def stage_cases(tag, cfg):
    m, sd, sd_raw = build(cfg)
    save(f"weights_{tag}", **{k: v.numpy() for k, v in sd.items()})
    # unpinned duration projection (untrained: durations 0.6-0.8 -> T = 1 edge case)
    p = "duration_predictor.predictor.projection"
    save(f"weights_{tag}_unpinned_proj", weight=sd_raw[p + ".weight"].numpy(), bias=sd_raw[p + ".bias"].numpy())

    g = torch.Generator().manual_seed(0)
    B, S = 2, 24
    ids = torch.randint(0, 42, (B, S), generator=g)
    lens = torch.tensor([24, 17])

    # --- small inference case -------------------------------------------------
    with torch.no_grad():
        ref_fwd = m(ids, lens)
        ref_mel, ref_audio = m.inference(ids, lens)
    o = orc.forward(sd, cfg, ids, lens)
    o_mel, o_audio = orc.inference(sd, cfg, ids, lens)
    d = {k: maxdiff(ref_fwd[k], o[k]) for k in ("encoder_output", "duration_pred", "regulated_output", "mel_output", "audio_output")}
    d["inference_mel"] = maxdiff(ref_mel, o_mel)
    d["inference_audio"] = maxdiff(ref_audio, o_audio)
    dur = ref_fwd["duration_pred"]
    MANIFEST["cases"][f"{tag}_small"] = {"oracle_vs_ref_maxabs": d,
                                          "min_dist_to_int": float((dur - dur.round()).abs().min()),
                                          "T": int(ref_mel.shape[1])}
    save(f"{tag}_small", ids=ids.numpy(), lengths=lens.numpy(),
         encoder_output=np32(ref_fwd["encoder_output"]), duration_pred=np32(ref_fwd["duration_pred"]),
         regulated_output=np32(ref_fwd["regulated_output"]), mel=np32(ref_mel), audio=np32(ref_audio),
         padding_mask=ref_fwd["padding_mask"].numpy())

    # --- teacher-forced durations (half-integers), free length / pad / truncate -
    tdur = torch.randint(3, 9, (B, S), generator=g).float() + 0.5
    for sub, mtl in (("free", None), ("pad", int(tdur.trunc().sum(1).max()) + 7), ("trunc", 60)):
        with torch.no_grad():
            r = m(ids, lens, target_durations=tdur, max_target_length=mtl)
        oo = orc.forward(sd, cfg, ids, lens, target_durations=tdur, max_target_length=mtl)
        MANIFEST["cases"][f"{tag}_target_{sub}"] = {"oracle_vs_ref_maxabs": {k: maxdiff(r[k], oo[k]) for k in ("regulated_output", "mel_output", "audio_output")},
                                                     "T": int(r["mel_output"].shape[1])}
        save(f"{tag}_target_{sub}", ids=ids.numpy(), lengths=lens.numpy(), target_durations=tdur.numpy(),
             max_target_length=np.int64(-1 if mtl is None else mtl),
             regulated_output=np32(r["regulated_output"]), mel=np32(r["mel_output"]), audio=np32(r["audio_output"]))

    # --- duration_scale --------------------------------------------------------
    with torch.no_grad():
        rm, ra = m.inference(ids, lens, duration_scale=1.3)
    om, oa = orc.inference(sd, cfg, ids, lens, duration_scale=1.3)
    MANIFEST["cases"][f"{tag}_scale"] = {"oracle_vs_ref_maxabs": {"mel": maxdiff(rm, om), "audio": maxdiff(ra, oa)}, "T": int(rm.shape[1])}
    save(f"{tag}_scale", ids=ids.numpy(), lengths=lens.numpy(), duration_scale=np.float64(1.3), mel=np32(rm), audio=np32(ra))

    # --- untrained durations: every int(d) == 0 -> regulator emits zeros(1,H) ----
    m_un, _, _ = build(cfg)
    m_un.load_state_dict(sd_raw)
    with torch.no_grad():
        um, ua = m_un.inference(ids, lens)
    om, oa = orc.inference(sd_raw, cfg, ids, lens)
    MANIFEST["cases"][f"{tag}_untrained"] = {"oracle_vs_ref_maxabs": {"mel": maxdiff(um, om), "audio": maxdiff(ua, oa)}, "T": int(um.shape[1])}
    save(f"{tag}_untrained", ids=ids.numpy(), lengths=lens.numpy(), mel=np32(um), audio=np32(ua))

    # --- kernel-level cases: every resblock width and every upsample ------------
    voc = m.vocoder
    with torch.no_grad():
        x = torch.randn(2, voc.input_conv.in_channels, 37, generator=g)
        y = voc.input_conv(x)
        save(f"{tag}_input_conv", x=np32(x), y=np32(y))
        for k, (up, rb) in enumerate(zip(voc.upsamples, voc.resblocks)):
            x = torch.randn(2, up.in_channels, 50, generator=g)
            y = torch.nn.functional.leaky_relu(up(x), 0.1)
            save(f"{tag}_convT{k}", x=np32(x), y=np32(y), rate=np.int32(orc.UPSAMPLE_RATES[k]))
            x = torch.randn(2, rb.conv1.in_channels, 203, generator=g)
            y = rb(x)
            save(f"{tag}_resblock{k}", x=np32(x), y=np32(y))
        x = torch.randn(2, voc.output_conv.in_channels, 301, generator=g)
        y = torch.tanh(voc.output_conv(x))
        save(f"{tag}_output_conv", x=np32(x), y=np32(y))
    return m, sd


def bench_fingerprints(tag, m, sd, cfg, B, S, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, 42, (B, S), generator=g)
    lens = torch.full((B,), S, dtype=torch.long)
    t0 = time.time()
    with torch.no_grad():
        mel, audio = m.inference(ids, lens)
    dt = time.time() - t0
    fp = fingerprint(mel, audio, [mel.shape[1]] * B)
    save(f"fp_{tag}_B{B}_S{S}", ids=ids.numpy(), lengths=lens.numpy(), **fp)
    MANIFEST["cases"][f"fp_{tag}_B{B}_S{S}"] = {"T": int(mel.shape[1]), "ref_inference_s": dt}


def vocoder_fingerprint(tag, m, B, M, T, seed=0):
    g = torch.Generator().manual_seed(seed)
    mel = torch.randn(B, M, T, generator=g)
    with torch.no_grad():
        audio = m.vocoder(mel)
    a = audio[:, 0].double()
    save(f"fp_{tag}_vocoder_B{B}_T{T}", seed=np.int64(seed),
         audio_sum=a.sum(1).numpy(), audio_sumsq=(a * a).sum(1).numpy(), audio_maxabs=a.abs().amax(1).numpy(),
         audio_head=np32(audio[:, 0, :256]), audio_tail=np32(audio[:, 0, -256:]))


SENTENCES = [
    "printing in the only sense with which we are at present concerned differs from most if not from all the arts",
    "Hello world", "Hello world, this is a test.", "The first test.", "Dr. Smith met Mr. Jones on St. James st.",
    "I have 3 apples and 20 pears, vs. 21 plums.", "e.g. this & that i.e. the other etc.",
    "It was the best of times, it was the worst of times.", "  Multiple   spaces\tand\ttabs  ",
    "Numbers: 0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18 19 20", "", "!!!", "café naïve résumé",
    "Quick brown fox jumps over the lazy dog", "What would you like to do today?", "ms. mrs. first. last.",
    "One two three; four (five) [six] {seven}", "a" * 300, "WHEN WILL THEY COME DOWN", "zzz xyz qqq",
]


def text_fixtures():
    tp = RefTextProcessor()
    out = []
    for s in SENTENCES:
        r256 = tp.process_text(s, max_length=256)
        r50 = tp.process_text(s, max_length=50)
        rn = tp.process_text(s)
        out.append({"text": s, "phonemes": rn["phonemes"], "ids": rn["phoneme_ids"], "length": rn["length"],
                    "ids256": r256["phoneme_ids"], "length256": r256["length"],
                    "ids50": r50["phoneme_ids"], "length50": r50["length"]})
    (HERE / "text_ids.json").write_text(json.dumps(out, indent=0, ensure_ascii=True))


def cli_case(m, sd):
    tp = RefTextProcessor()
    text = SENTENCES[0]
    td = tp.process_text(text, max_length=256)
    ids = torch.LongTensor(td["phoneme_ids"]).unsqueeze(0)
    lens = torch.LongTensor([td["length"]])
    with torch.no_grad():
        mel, audio = m.inference(ids, lens)
    save("cli_stage1", text=np.asarray(text), ids=ids.numpy(), lengths=lens.numpy(), mel=np32(mel), audio=np32(audio))
    MANIFEST["cases"]["cli_stage1"] = {"T": int(mel.shape[1]), "n_samples": int(audio.shape[-1]), "length": td["length"]}


def main():
    text_fixtures()
    m1, sd1 = stage_cases("s1", orc.STAGE1)
    m2, sd2 = stage_cases("s2", orc.STAGE2)
    cli_case(m1, sd1)
    bench_fingerprints("s1", m1, sd1, orc.STAGE1, 32, 100)
    vocoder_fingerprint("s1", m1, 32, 64, 500)
    bench_fingerprints("s2", m2, sd2, orc.STAGE2, 64, 100)
    if os.environ.get("M2_GOLDEN_LONGFORM", "1") == "1":
        bench_fingerprints("s2", m2, sd2, orc.STAGE2, 128, 520)
    (HERE / "manifest.json").write_text(json.dumps(MANIFEST, indent=1))
    worst = max((v for c in MANIFEST["cases"].values() for v in c.get("oracle_vs_ref_maxabs", {}).values()), default=0.0)
    print("oracle vs reference worst max-abs:", worst)
    assert worst == 0.0, "oracle must reproduce the reference bit for bit on CPU"


if __name__ == "__main__":
    main()
