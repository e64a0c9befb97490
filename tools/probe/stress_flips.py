#!/usr/bin/env python3
"""which vocoder path writes the samples of
tests/test_gpu_stress.py::test_scaled_weights_inference[4.0-*] that land more
than 1e-2 from a float64 evaluation of the reference.  For each stage at
weights x4: the GPU vocoder on the oracle's mel under the default policy
(split-f16 + in-launch fp32 redo of non-finite strips), under "report" (the
split path's own output: NaN where a strip overflowed the split range, i.e.
where the default redo writes), on the exact-f32 kernels, and the oracle's
fp32 path; per far sample its float64 pre-tanh value and the fp32 oracle's
pre-tanh error there.
    python3 tools/probe/stress_flips.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent


def main():
    import torch
    sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import m2tts_oracle as orc
    from conftest import golden_state, stage_config  # noqa: F401
    from test_gpu_stress import scaled_state
    from models.tts_model import M2TTSModel
    gpu = torch.device("cuda", 0)
    f = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    for stage in ("s1", "s2"):
        cfg = stage_config(stage)
        sd = scaled_state(stage, f)
        m = M2TTSModel(**cfg.as_dict())
        m.load_state_dict(sd)
        m = m.to(gpu).eval()
        g = torch.Generator().manual_seed(int(11 * f) + (0 if stage == "s1" else 1))
        ids = torch.randint(0, 42, (5, 70), generator=g)
        lens = torch.randint(20, 71, (5,), generator=g)
        lens[0] = 70
        ref_mel, _ = orc.inference(sd, cfg, ids, lens, as_written=False)
        mel_bmt = ref_mel.transpose(1, 2).contiguous()
        sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
        tanh = torch.tanh
        torch.tanh = lambda x: x  # the oracle's pre-tanh output
        try:
            pre64 = orc.vocoder(sd64, mel_bmt.double())
            pre32 = orc.vocoder(sd, mel_bmt).double()
        finally:
            torch.tanh = tanh
        ref64 = torch.tanh(pre64)
        o32 = orc.vocoder(sd, mel_bmt).double()
        outs = {}
        mg = mel_bmt.to(gpu)
        outs["default"] = m.vocoder(mg).cpu().double()
        m.set_range_policy("report")
        outs["report"] = m.vocoder(mg).cpu().double()
        try:
            m.check_numerics()
            flagged = False
        except Exception:
            flagged = True
        m.set_range_policy("fallback")
        m.set_vocoder_precision("f32")
        outs["exact_f32"] = m.vocoder(mg).cpu().double()
        m.set_vocoder_precision("split")
        outs["oracle_fp32"] = o32
        nan = ~torch.isfinite(outs["report"])
        print(f"== {stage} x{f}: {ref64.numel()} samples, |pre64| max {float(pre64.abs().max()):.3g}, "
              f"split path non-finite samples {int(nan.sum())} (flagged {flagged}); fp32 oracle pre-tanh err max "
              f"{float((pre32 - pre64).abs().max()):.3g}", flush=True)
        for k, o in outs.items():
            far = (o - ref64).abs() > 1e-2
            n = int(far.sum())
            line = f"  {k:12s} far {n:5d} ({n / far.numel():.2e})"
            if n:
                idx = far.nonzero()
                in_redo = int(nan[far].sum())
                p = pre64[far]
                e = (pre32 - pre64)[far].abs()
                line += (f"  in redone strips {in_redo}  |pre64| at far: max {float(p.abs().max()):.3g} "
                         f"median {float(p.abs().median()):.3g}; fp32-oracle pre err there max {float(e.max()):.3g}")
                line += f"  first {idx[:3].tolist()}"
            fin = ~far & torch.isfinite(o)
            line += f"  rms(rest) {float((o[fin] - ref64[fin]).pow(2).mean().sqrt()):.3g}"
            print(line, flush=True)
        # how close to zero the float64 pre-tanh values get, against fp32's resolution there
        small = pre64.abs() < 1.0
        print(f"  samples with |pre64| < 1: {int(small.sum())}; < 0.01: {int((pre64.abs() < 0.01).sum())}", flush=True)


if __name__ == "__main__":
    main()
