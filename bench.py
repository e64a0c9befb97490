#!/usr/bin/env python3
"""Benchmark: audio samples/s (22.05 kHz) + real-time factor of the m2-tts
mel-synthesis + vocoder path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload vocoder|pipeline]

One process per GPU (torchrun for N>1, RCCL backend); every rank processes
its own batch of B utterances (weak scaling: utterances are independent, no
collective in the data path).  Timed region: barrier + synchronize, K steps,
synchronize + barrier; the max elapsed over ranks is the job time.

Workloads:
  vocoder  (default, BASELINE.json configs[1]) stage1_poc SimpleVocoder, B=32,
           mel [32, 64, 500] ~ N(0,1) resident in HBM -> audio [32, 1, 32000]
  pipeline (configs[2]) stage1_poc M2TTSModel.inference, B=32, 100 phonemes,
           fixture weights with durations pinned to 5 frames -> T=500

Extra fields: ``roofline`` for the dominant kernel (HIP events on its launch
stream, around every launch of the timed region), ``cpu_baseline`` (the CPU
oracle = the reference's op sequence, timed on this host, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))

SAMPLE_RATE = 22050
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 vector = f32 MFMA peak
F16_PEAK_TFLOPS = 2516.8     # MI355X_MICROARCH.md: f16/bf16 dense MFMA = 16 x the f32 MFMA rate
# Vocoder arithmetic paths (m2_vocoder_path): peak for ALGORITHMIC fp32 FLOP/s and what it means.
VOC_PATHS = {
    0: ("f32", FP32_PEAK_TFLOPS, "per-layer fp32 kernels; fp32 peak 157.3 TF"),
    1: ("f32", FP32_PEAK_TFLOPS, "fp32: v_mfma_f32_16x16x4_f32 = f32 VALU peak 157.3 TF (no xf32 on gfx950)"),
    2: ("f32 (split 3xf16 MFMA, fp32 accumulate)", F16_PEAK_TFLOPS / 3,
        "fp32 operands as f16 hi/lo pairs, 3 v_mfma_f32_16x16x32_f16 per fp32 product: "
        "effective fp32 peak = 2516.8 / 3 = 838.9 TF"),
}
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec
METRIC = "audio samples/sec (22.05 kHz) + RTF, stage1_poc batch=32 @1/2/4/8 MI355X"

STAGE1 = dict(vocab_size=256, hidden_dim=64, mel_channels=64, text_encoder_layers=2, decoder_layers=2,
              num_heads=2, dropout=0.1, vocoder_channels=128)


# Event sampling in the timed region: one event pair around the dominant
# kernel every PROF_STRIDE steps (each pair costs a few us of pipeline drain).
PROF_STRIDE = 8

def vocoder_flops_per_sample(C: int, M: int) -> float:
    """Algorithmic FLOPs per output audio sample of SimpleVocoder.

    Per mel frame: input conv 2*M*C*3; stage k (rate r, c -> c/2, L -> rL):
    ConvT 2*2*c*(c/2) per output, resblock 2*(2*(c/2)^2*3) per output;
    output conv 2*c_last*3 per sample.  Divided by 64 samples per frame."""
    f = 2 * M * C * 3
    c, n = C, 1
    for r in (4, 4, 2, 2):
        n *= r
        co = c // 2
        f += n * (2 * 2 * c * co + 2 * 2 * co * co * 3)
        c = co
    f += n * 2 * c * 3
    return f / n


def vocoder_kernel_flops_per_frame(C: int, M: int):
    """Algorithmic FLOPs per mel frame of the three fused vocoder kernels
    (head: input_conv+ConvT1+RB1, mid: ConvT2+RB2, tail: ConvT3+RB3+ConvT4+RB4+out)."""
    def stage(c, n):  # ConvT c -> c/2 then resblock(c/2), n output positions per frame
        co = c // 2
        return n * (2 * 2 * c * co + 2 * 2 * co * co * 3)
    head = 2 * M * C * 3 + stage(C, 4)
    mid = stage(C // 2, 16)
    tail = stage(C // 4, 32) + stage(C // 8, 64) + 64 * 2 * (C // 16) * 3
    return [head, mid, tail]


def fixture_model(dev):
    """Random-init stage1 weights (seed 1234) with durations pinned
    to 5 frames/phoneme: projection weight * 0.01, bias 5.5."""
    from models.tts_model import M2TTSModel
    torch.manual_seed(1234)
    m = M2TTSModel(**STAGE1)
    with torch.no_grad():
        p = m.duration_predictor.predictor.projection
        p.weight.mul_(0.01)
        p.bias.fill_(5.5)
    return m.to(dev).eval()


def cpu_baseline(workload: str, B: int, S: int, T: int, budget_s: float):
    """Time the CPU oracle (reference op order) on a bounded sample of the workload."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import m2tts_oracle as orc
    threads = torch.get_num_threads()
    torch.manual_seed(1234)
    from models.tts_model import M2TTSModel  # only for the seeded init (module construction on CPU)
    m = M2TTSModel(**STAGE1)
    sd = orc.pin_durations({k: v.detach().clone() for k, v in m.state_dict().items()})
    cfg = orc.STAGE1
    g = torch.Generator().manual_seed(0)
    if workload == "vocoder":
        mel = torch.randn(B, cfg.mel_channels, T, generator=g)
        run = lambda: orc.vocoder(sd, mel)  # noqa: E731
        desc = f"oracle SimpleVocoder single pass, B={B} mel [{B},{cfg.mel_channels},{T}]"
    else:
        ids = torch.randint(0, 42, (B, S), generator=g)
        lens = torch.full((B,), S, dtype=torch.long)
        run = lambda: orc.inference(sd, cfg, ids, lens, as_written=True)  # noqa: E731
        desc = f"oracle M2TTSModel.inference as written (2 vocoder passes), B={B} S={S}"
    with torch.no_grad():
        run()  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            run()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 200:
                break
    samples = n * B * 64 * T
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": samples / el, "unit": "audio samples/s", "cores": threads, "kind": "port",
            "sample": f"{desc}; {n} runs in {el:.1f} s; torch {torch.__version__} CPU, {threads} threads, {cpu_model}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Defaults: the GPU clocks take tens of ms of load to settle (a first
    # 30 ms loop runs ~7 % slow: tools/probe/timing_order.py), so the default
    # warm-up is a few hundred steps (~40 ms); both finish in well under a second.
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--workload", choices=["vocoder", "pipeline"], default="vocoder")
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    ap.add_argument("--phonemes", type=int, default=100)
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline-extra", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        td.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from m2amd import _lib
    lib = _lib.load()
    model = fixture_model(dev)
    B, S, T = args.batch, args.phonemes, 5 * args.phonemes
    g = torch.Generator().manual_seed(1000 + rank)
    mel = torch.randn(B, STAGE1["mel_channels"], T, generator=g).to(dev)
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    hm = model._hip(dev)
    voc_dtype, voc_peak, voc_note = VOC_PATHS[lib.m2_vocoder_path(hm.handle)]

    def step_vocoder():
        return model.vocoder(mel)

    def step_pipeline():
        return model.inference(ids, lens)

    step = step_vocoder if args.workload == "vocoder" else step_pipeline

    nk = lib.m2_profile_kernel_count()

    def timed(fn, steps, warmup, kernel_mask=0, stride=1):
        """Run `steps` of fn between barriers + syncs; with kernel_mask, HIP
        events (fence-free, on the launch stream inside m2_vocoder) around
        the selected fused vocoder kernels of every `stride`-th step."""
        for _ in range(warmup):
            fn()
        if kernel_mask:
            _lib.check(lib.m2_profile_select(hm.handle, kernel_mask), "m2_profile_select")
            _lib.check(lib.m2_profile_stride(hm.handle, stride), "m2_profile_stride")
            _lib.check(lib.m2_profile_enable(hm.handle, (steps + stride - 1) // stride), "m2_profile_enable")
        torch.cuda.synchronize(dev)
        if dist:
            td.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        if dist:
            td.barrier()
        el = time.perf_counter() - t0
        ms = []
        if kernel_mask:
            import ctypes
            cap = (steps + stride - 1) // stride * nk
            buf = (ctypes.c_float * cap)()
            n = ctypes.c_int32(0)
            _lib.check(lib.m2_profile_read(hm.handle, buf, cap, ctypes.byref(n)), "m2_profile_read")
            ms = list(buf[: n.value])
            lib.m2_profile_disable(hm.handle)
            _lib.check(lib.m2_profile_stride(hm.handle, 1), "m2_profile_stride")
        if dist:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            td.all_reduce(t, op=td.ReduceOp.MAX)
            el = float(t.item())
        return el, ms

    C, M = STAGE1["vocoder_channels"], STAGE1["mel_channels"]
    fl = vocoder_kernel_flops_per_frame(C, M)

    def kernel_table(kern_ms):
        rows = []
        for i in range(nk):
            vals = [v for v in kern_ms[i::nk] if v >= 0]
            if not vals:
                continue
            avg = sum(vals) / len(vals)
            flops = fl[i] * B * T
            rows.append({"index": i, "kernel": lib.m2_profile_kernel_name_for(hm.handle, i).decode(),
                         "avg_ms": round(avg, 5), "launches": len(vals), "algorithmic_flop_per_launch": flops,
                         "tflops": round(flops / (avg * 1e-3) / 1e12, 3)})
        return rows

    # 1) Untimed pass with events on all three kernels: per-kernel table and
    #    which kernel dominates.  Events drain the pipeline between kernels
    #    (a few us each), so 2) the timed region carries events around the
    #    dominant kernel of every PROF_STRIDE-th step only: its average
    #    duration over those launches of the timed region is the roofline's
    #    denominator.  3) the same loop with no events at all, for the record.
    _, all_ms = timed(step, min(args.steps, 20), args.warmup, kernel_mask=(1 << nk) - 1)
    per_kernel = kernel_table(all_ms)
    dom_i = max(per_kernel, key=lambda d: d["avg_ms"])["index"] if per_kernel else 0
    elapsed, kern_ms = timed(step, args.steps, 2, kernel_mask=1 << dom_i, stride=PROF_STRIDE)
    el_ne, _ = timed(step, args.steps, 2)
    samples_per_step = B * 64 * T
    total_samples = samples_per_step * args.steps * world
    value = total_samples / elapsed

    roofline = None
    live = kernel_table(kern_ms)
    if live:
        dom = live[0]
        achieved = dom["tflops"]
        roofline = {"bound": "mfma", "achieved": achieved, "peak": round(voc_peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / voc_peak, 4), "traffic": None, "kernel": dom["kernel"],
                    "avg_kernel_ms": dom["avg_ms"], "launches": dom["launches"],
                    "algorithmic_flop_per_launch": dom["algorithmic_flop_per_launch"],
                    "dtype_peak_note": voc_note}
        tf = ROOT / "profiles" / "traffic.json"
        if tf.exists():
            try:
                roofline["traffic"] = json.loads(tf.read_text()).get(dom["kernel"].split()[0])
            except ValueError:
                pass

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "audio samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": voc_dtype,
        "data": "synthetic (seeded N(0,1) mel / U{0..41} phoneme ids; random-init stage1 weights, seed 1234)",
        "config": {"workload": "stage1_poc SimpleVocoder B=32 (configs[1])" if args.workload == "vocoder"
                   else "stage1_poc M2TTSModel.inference B=32 S=100 (configs[2])",
                   "stage": "stage1_poc", "per_gpu_batch": B, "global_batch": B * world, "mel_frames": T,
                   "audio_samples_per_utt": 64 * T, "parallelism": f"utterance-sharded x{world} (dp{world})"},
        "ms_per_step_without_kernel_events": round(el_ne / args.steps * 1e3, 4),
        "rtf_x_realtime": round(value / SAMPLE_RATE, 1),
        "rtf_x_realtime_per_gpu": round(value / SAMPLE_RATE / world, 1),
        "roofline": roofline,
        "vocoder_kernels": per_kernel,  # untimed pass, events on every kernel
    }
    if args.workload == "vocoder":
        out["vocoder_flop_per_sample"] = vocoder_flops_per_sample(STAGE1["vocoder_channels"], STAGE1["mel_channels"])
        out["vocoder_tflops"] = round(value * out["vocoder_flop_per_sample"] / 1e12, 3)

    if not args.no_pipeline_extra:
        other = step_pipeline if args.workload == "vocoder" else step_vocoder
        el2, _ = timed(other, max(5, args.steps // 2), 3)
        n2 = max(5, args.steps // 2)
        out["other_workload"] = {"workload": "pipeline" if args.workload == "vocoder" else "vocoder",
                                 "value": round(samples_per_step * n2 * world / el2, 1),
                                 "ms_per_step": round(el2 / n2 * 1e3, 4)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.workload, B, S, T, args.cpu_budget)
        out["cpu_baseline"]["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        if not args.no_pipeline_extra:
            other = "pipeline" if args.workload == "vocoder" else "vocoder"
            out["cpu_baseline_other"] = cpu_baseline(other, B, S, T, args.cpu_budget / 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
