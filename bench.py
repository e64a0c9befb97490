#!/usr/bin/env python3
"""Benchmark: audio samples/s (22.05 kHz) + real-time factor of the m2-tts
mel-synthesis + vocoder path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

One process per GPU, RCCL (torch.distributed "nccl") between them.  With
``--gpus N > 1`` and no WORLD_SIZE in the environment, this process starts N
fresh rank processes (spawn, before anything touches the GPU) and waits for
them; under ``torch.distributed.run`` the ranks come from the environment.
Timed region of every line: barrier + synchronize, K steps, synchronize +
barrier; the job time is the max over ranks.  Before the first timed region
every rank runs the workload untimed for ``--settle-ms`` (the GPU clocks need
tens of ms of load to settle; a 1.6 ms timed loop right after launch runs
~20 % slow, tools/probe/timing_order.py).

Workloads (BASELINE.json configs):
  vocoder      configs[1] (headline): stage1 SimpleVocoder, B=32 utterances
               PER GPU, mel [32, 64, 500] ~ N(0,1) resident in HBM -> audio
               [32, 1, 32000]; weak scaling (independent replicas, no collective)
  pipeline     configs[2]: stage1 M2TTSModel.inference, B=32 per GPU, 100
               phonemes, fixture weights (durations pinned to 5 frames) -> T=500
  s2_b64       configs[3]: stage2 M2TTSModel.inference over a GLOBAL batch of 64
               utterances (100 phonemes -> T=500) sharded by utterance across
               the N ranks (m2amd.parallel.sharded_inference: RCCL all_reduce(MAX)
               of the frame count + gather of mel/audio to rank 0); strong scaling
  s2_longform  configs[4]: the same with a global batch of 128 utterances of
               520 phonemes -> T=2600 mel frames (30.2 s at hop 256), vocoder
               streamed in 256-frame chunks (3-frame halo)
  s2_vocoder   stage2 SimpleVocoder at the per-GPU shape of configs[3] on 8
               GPUs: B=8, T=500 (per-kernel roofline table)
The default run measures ``vocoder`` as the headline ``value`` and adds the
other workloads, the exact-f32 vocoder, and (rank 0, N=1) the CPU oracle as
sub-objects of the same JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path


def _cpu_child_pin():
    """CPU-baseline child (``bench.py --cpu-child SPEC``): pin this process to
    the CPUs SPEC lists (one logical CPU per physical core) and bind one
    OpenMP thread to each, before torch (and its OpenMP runtime) loads."""
    spec = json.loads(sys.argv[sys.argv.index("--cpu-child") + 1])
    os.sched_setaffinity(0, spec["cpus"])
    n = str(len(spec["cpus"]))
    os.environ.update(OMP_NUM_THREADS=n, MKL_NUM_THREADS=n, OMP_PROC_BIND="close", OMP_PLACES="threads",
                      OMP_WAIT_POLICY="PASSIVE")


if __name__ == "__main__" and "--cpu-child" in sys.argv:
    _cpu_child_pin()

import torch  # noqa: E402

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))

SAMPLE_RATE = 22050
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 vector = f32 MFMA peak
F16_PEAK_TFLOPS = 2516.8     # MI355X_MICROARCH.md: f16/bf16 dense MFMA = 16 x the f32 MFMA rate
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E
# Vocoder arithmetic paths (m2_vocoder_path): peak for ALGORITHMIC fp32 FLOP/s and what it means.
VOC_PATHS = {
    0: ("f32", FP32_PEAK_TFLOPS, "per-layer fp32 kernels; fp32 peak 157.3 TF"),
    1: ("f32", FP32_PEAK_TFLOPS, "fp32: v_mfma_f32_16x16x4_f32 = f32 VALU peak 157.3 TF (no xf32 on gfx950)"),
    2: ("f32 (split 3xf16 MFMA, fp32 accumulate)", F16_PEAK_TFLOPS / 3,
        "fp32 operands as f16 hi/lo pairs, 3 v_mfma_f32_16x16x32_f16 per fp32 product: "
        "effective fp32 peak = 2516.8 / 3 = 838.9 TF"),
}
METRIC = "audio samples/sec (22.05 kHz) + RTF, stage1_poc batch=32 @1/2/4/8 MI355X"

STAGE1 = dict(vocab_size=256, hidden_dim=64, mel_channels=64, text_encoder_layers=2, decoder_layers=2,
              num_heads=2, dropout=0.1, vocoder_channels=128)
STAGE2 = dict(vocab_size=256, hidden_dim=96, mel_channels=80, text_encoder_layers=3, decoder_layers=3,
              num_heads=2, dropout=0.1, vocoder_channels=256)
RATES = (4, 4, 2, 2)


# ---------------------------------------------------------------------------- work models
def vocoder_flops_per_sample(C: int, M: int) -> float:
    """Algorithmic FLOPs per output audio sample of SimpleVocoder.

    Per mel frame: input conv 2*M*C*3; stage k (rate r, c -> c/2, L -> rL):
    ConvT 2*2*c*(c/2) per output, resblock 2*(2*(c/2)^2*3) per output;
    output conv 2*c_last*3 per sample.  Divided by 64 samples per frame."""
    f = 2 * M * C * 3
    c, n = C, 1
    for r in RATES:
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


def mrf_bytes(C: int, B: int, T: int) -> float:
    """SURVEY.md 8d per-kernel bytes of the four LightweightResBlocks ("MRF"):
    each reads its input once and writes its output once (8*c*L per
    utterance) plus its weights once (4*(6c^2+2c))."""
    tot, c, L = 0.0, C, T
    for r in RATES:
        c //= 2
        L *= r
        tot += B * 8.0 * c * L + 4.0 * (6 * c * c + 2 * c)
    return tot


def fixture_model(cfg: dict, dev):
    """Random-init weights (seed 1234) with durations pinned to 5
    frames/phoneme: projection weight * 0.01, bias 5.5."""
    from models.tts_model import M2TTSModel
    torch.manual_seed(1234)
    m = M2TTSModel(**cfg)
    with torch.no_grad():
        p = m.duration_predictor.predictor.projection
        p.weight.mul_(0.01)
        p.bias.fill_(5.5)
    return m.to(dev).eval()


# ---------------------------------------------------------------------------- host / CPU baseline
def host_info():
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return cpu_model, os.cpu_count(), affinity


def physical_cores():
    """One logical CPU per physical core of this process's affinity mask, and
    the sockets they sit on (sysfs topology)."""
    chosen = {}
    for c in sorted(os.sched_getaffinity(0)):
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            key = (int(open(base + "physical_package_id").read()), int(open(base + "core_id").read()))
        except (OSError, ValueError):
            key = (0, c)
        chosen.setdefault(key, c)
    return sorted(chosen.values()), len({k[0] for k in chosen})


def cpu_quota():
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max or
    v1 cfs quota / period), or None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def _cg_throttled_s():
    """Seconds this cgroup has been throttled by its CPU quota so far (cgroup
    v2 cpu.stat throttled_usec, v1 throttled_time), or None."""
    for path, key, scale in (("/sys/fs/cgroup/cpu.stat", "throttled_usec", 1e-6),
                             ("/sys/fs/cgroup/cpu/cpu.stat", "throttled_time", 1e-9)):
        try:
            for line in open(path):
                k, v = line.split()[:2]
                if k == key:
                    return int(v) * scale
        except (OSError, ValueError):
            pass
    return None


def _steal_s():
    """Steal time so far, summed over this process's CPUs (the cpuN lines of
    /proc/stat, USER_HZ ticks) and divided by their number: wall seconds the
    hypervisor took from a thread pinned there, on average."""
    try:
        mine = {f"cpu{c}" for c in os.sched_getaffinity(0)}
        tot = 0
        for line in open("/proc/stat"):
            f = line.split()
            if f and f[0] in mine and len(f) > 8:
                tot += int(f[8])
        return tot / os.sysconf("SC_CLK_TCK") / max(1, len(mine))
    except (OSError, ValueError, IndexError):
        return None


def cpu_measure(run, runs: int, min_s: float, threads: int):
    """`runs` measurements of run()'s rate (calls/s), each timing whole calls
    for at least min_s seconds, with what each run got of the CPUs: busy =
    this process's CPU seconds / (wall seconds x threads), and the cgroup
    throttle / host steal seconds that fell inside it.  A run that another
    tenant's load slowed down shows a busy fraction well under the best run's
    (its threads were descheduled) or throttle / steal time: it is dropped
    (kept: busy >= 0.85 x the best run's, throttle + steal <= 5 % of the wall
    time), and the statistics are over the kept runs."""
    recs = []
    with torch.no_grad():
        run()  # warm-up
        for _ in range(runs):
            n, th0, st0 = 0, _cg_throttled_s(), _steal_s()
            c0, t0 = time.process_time(), time.perf_counter()
            while True:
                run()
                n += 1
                el = time.perf_counter() - t0
                if el >= min_s:
                    break
            cpu = time.process_time() - c0
            th1, st1 = _cg_throttled_s(), _steal_s()
            thr = th1 - th0 if th0 is not None and th1 is not None else 0.0
            stl = st1 - st0 if st0 is not None and st1 is not None else 0.0
            recs.append({"rate": n / el, "busy": round(cpu / (el * max(1, threads)), 3), "throttled_s": round(thr, 3),
                         "steal_s": round(stl, 3), "wall_s": round(el, 3)})
    best_busy = max(r["busy"] for r in recs)
    kept = [r for r in recs
            if r["busy"] >= 0.85 * best_busy and r["throttled_s"] + r["steal_s"] <= 0.05 * r["wall_s"]]
    if len(kept) < 3:  # too few clean runs: keep them all and say so
        kept = recs
    rates = sorted(r["rate"] for r in kept)
    return rates[len(rates) // 2], rates[0], rates[-1], recs, len(kept)


def cpu_child_main(spec):
    """Runs in the pinned child: the CPU oracle (the reference's op sequence)
    on both workloads of the headline configuration."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import m2tts_oracle as orc
    torch.set_num_threads(len(spec["cpus"]))
    B, S, T = spec["B"], spec["S"], spec["T"]
    torch.manual_seed(1234)
    from models.tts_model import M2TTSModel  # only for the seeded init (module construction on CPU)
    m = M2TTSModel(**STAGE1)
    sd = orc.pin_durations({k: v.detach().clone() for k, v in m.state_dict().items()})
    cfg = orc.STAGE1
    g = torch.Generator().manual_seed(0)
    mel = torch.randn(B, cfg.mel_channels, T, generator=g)
    ids = torch.randint(0, 42, (B, S), generator=g)
    lens = torch.full((B,), S, dtype=torch.long)
    out = {"torch_threads": torch.get_num_threads()}
    if spec.get("ids_seed") is not None:
        # the CPU path's frame counts for the pipeline line's batch (T equality)
        pids = torch.randint(0, 42, (B, S), generator=torch.Generator().manual_seed(spec["ids_seed"]))
        with torch.no_grad():
            enc, _ = orc.text_encoder(sd, cfg, pids, lens)
            dur = orc.duration_predictor(sd, enc).double()
        out["frames"] = {"cpu_T_per_utt": torch.trunc(dur).clamp(min=0).sum(1).to(torch.int64).tolist(),
                         "min_duration_dist_to_int": float((dur - dur.round()).abs().min())}
    for name, run in (("vocoder", lambda: orc.vocoder(sd, mel)),
                      ("inference_as_written", lambda: orc.inference(sd, cfg, ids, lens, as_written=True))):
        med, lo, hi, recs, nkept = cpu_measure(run, spec["runs"], spec["min_s"], len(spec["cpus"]))
        out[name] = {"median": med * B * 64 * T, "min": lo * B * 64 * T, "max": hi * B * 64 * T,
                     "calls_per_s": [round(r["rate"], 3) for r in recs], "runs": recs, "kept": nkept}
    print(json.dumps(out), flush=True)


def cpu_baseline(B: int, S: int, T: int, runs: int = 7, min_s: float = 1.5, ids_seed=None):
    """Time the CPU oracle (the reference's op sequence) on the
    node's host cores: a child process pinned to one logical CPU per physical
    core of this process's affinity mask, one OpenMP thread per core
    (torch.set_num_threads(physical cores)), median of the clean runs among
    `runs` measurements (cpu_measure drops runs another tenant's load slowed
    down), with their spread; `unstable` when the kept runs still spread by
    20 % or more (value = the median run).  Two figures for the headline configuration: the
    vocoder single pass (configs[1], the `value`) and M2TTSModel.inference as
    written (2 vocoder passes, Python length-regulator loop)."""
    phys, sockets = physical_cores()
    quota = cpu_quota()
    # threads beyond the job's CPU quota only queue behind the throttle (and
    # make the figure swing with the neighbours' load): one per physical core,
    # capped at the quota
    cpus = phys[:max(1, int(quota))] if quota is not None else phys
    spec = {"cpus": cpus, "B": B, "S": S, "T": T, "runs": runs, "min_s": min_s, "ids_seed": ids_seed}
    env = dict(os.environ)
    env.pop("HIP_VISIBLE_DEVICES", None)
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--cpu-child", json.dumps(spec)], env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": f"cpu baseline child failed (rc {r.returncode}): {r.stderr[-400:]}"}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    cpu_model, ncpu, aff = host_info()
    voc, inf = res["vocoder"], res["inference_as_written"]
    spread = lambda d: round((d["max"] - d["min"]) / d["median"], 3)  # noqa: E731
    unstable = lambda d: spread(d) >= 0.2  # noqa: E731
    # value = the median of the runs; the best run (other tenants' load on the
    # shared host only slows a run down) and the spread are reported beside it
    busy = sorted(r["busy"] for r in voc["runs"])
    return {"value": voc["median"], "best": voc["max"], "unit": "audio samples/s", "cores": len(cpus),
            "effective_cores": round(busy[len(busy) // 2] * len(cpus), 2),
            "effective_cores_def": "median over the runs of busy (process CPU s / (wall s x threads)) x threads: "
                                   "the cores the reference's op sequence actually kept busy",
            "kind": "port",
            "sockets": sockets, "host_logical_cpus": ncpu, "affinity_cpus": aff,
            "physical_cores_in_affinity": len(phys), "cgroup_cpu_quota": quota,
            "torch_threads": res["torch_threads"], "pinned": "one OpenMP thread per physical core "
            "(OMP_PROC_BIND=close on one logical CPU per core)", "cpu_model": cpu_model,
            "stat": f"median of the {voc['kept']} clean runs of {runs} of >= {min_s} s (best, min, max "
                    f"beside it; a run is dropped when its threads got < 0.85 x the best run's CPU time or the "
                    f"cgroup throttle / host steal took > 5 % of it)", "min": voc["min"],
            "max": voc["max"],
            "spread": spread(voc), "unstable": unstable(voc), "runs": voc["runs"],
            "sample": f"oracle SimpleVocoder single pass (the reference's ATen op sequence), B={B} mel [{B},64,{T}] "
                      f"(configs[1]); torch {torch.__version__} CPU ops on {len(cpus)} physical cores "
                      f"(of {len(phys)} on {sockets} sockets; job CPU quota {quota}) of {cpu_model}",
            "inference_as_written": {"value": inf["median"], "best": inf["max"], "min": inf["min"],
                                     "max": inf["max"],
                                     "spread": spread(inf), "unstable": unstable(inf),
                                     "kept": inf["kept"], "unit": "audio samples/s",
                                     "sample": f"oracle M2TTSModel.inference as written (2 vocoder passes, "
                                               f"Python length-regulator loop), B={B} S={S} -> T={T}"},
            "frames": res.get("frames"), "wall_s": round(time.perf_counter() - t0, 1)}


def samples_per(B: int, T: int) -> int:
    return B * 64 * T


# ---------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(rank: int, world: int, port: int, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse_args(argv))


def launch_ranks(args, argv):
    """Start args.gpus fresh rank processes (this process has not touched the GPU)."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_entry, args=(args.gpus, _free_port(), argv), nprocs=args.gpus, join=True,
                       start_method="spawn")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=400.0,
                    help="untimed, time-based run of the workload before the first timed region")
    ap.add_argument("--workload", choices=["vocoder", "pipeline", "s2_b64", "s2_longform", "s2_vocoder"],
                    default="vocoder")
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU (vocoder / pipeline)")
    ap.add_argument("--phonemes", type=int, default=100)
    ap.add_argument("--s2-shape", default="8x500", help="BxT of the s2_vocoder workload")
    ap.add_argument("--cpu-runs", type=int, default=7, help="CPU baseline: measurements per workload (median of the clean ones)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline line only")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL (default); gloo only to rehearse N ranks sharing one GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group, all-reduce, print one line")
    return ap.parse_args(argv)


def dry_run(args):
    """CPU check of the launch path (tests/test_bench_launcher.py): every rank
    joins a gloo group with the rendezvous the launcher set up and
    all-reduces its rank; rank 0 prints n_gpus = world size seen."""
    import torch.distributed as td
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        td.init_process_group("gloo", rank=rank, world_size=world)
        t = torch.tensor([rank + 1.0])
        td.all_reduce(t)
        total = float(t.item())
        td.destroy_process_group()
    else:
        total = 1.0
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "rank_sum": total, "gpus_flag": args.gpus}), flush=True)


# ---------------------------------------------------------------------------- measurement
class Ctx:
    def __init__(self, dev, world, rank, dist):
        self.dev, self.world, self.rank, self.dist = dev, world, rank, dist
        from m2amd import _lib
        self.lib = _lib.load()
        self._lib = _lib
        self.nk = self.lib.m2_profile_kernel_count()
        self.models = {}
        self.backend = "RCCL"

    def model(self, stage: str):
        if stage not in self.models:
            # the public default range policy ("fallback": a call whose split-f16
            # audio came out non-finite is re-run on the exact-f32 kernels, on the
            # device); the "report" policy is its own side line
            # (vocoder_report_policy)
            m = fixture_model(STAGE1 if stage == "s1" else STAGE2, self.dev)
            self.models[stage] = m
        return self.models[stage]

    def barrier(self):
        if self.dist:
            import torch.distributed as td
            td.barrier()

    def max_over_ranks(self, v: float) -> float:
        if not self.dist:
            return v
        import torch.distributed as td
        t = torch.tensor([v], device=self.dev if self.backend == "RCCL" else "cpu", dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        return float(t.item())

    def settle(self, fn, ms: float) -> float:
        """Run fn untimed for about `ms` milliseconds of wall time (clock settling).
        With several ranks the ranks agree on every further iteration (fn may
        hold collectives: a rank that stopped alone would leave the others
        waiting in one)."""
        t0 = time.perf_counter()
        while True:
            go = (time.perf_counter() - t0) * 1e3 < ms
            if self.dist:
                go = self.max_over_ranks(1.0 if go else 0.0) > 0.5
            if not go:
                break
            fn()
            torch.cuda.synchronize(self.dev)
        return (time.perf_counter() - t0) * 1e3

    def timed(self, fn, steps: int, warmup: int, hm=None, kernel_mask: int = 0, stride: int = 1):
        """Run `steps` of fn between barriers + syncs (max over ranks); with
        kernel_mask, fence-free HIP events on the launch stream inside
        m2_vocoder around the selected vocoder kernels of every stride-th call."""
        lib, chk = self.lib, self._lib.check
        for _ in range(warmup):
            fn()
        if kernel_mask:
            chk(lib.m2_profile_select(hm.handle, kernel_mask), "m2_profile_select")
            chk(lib.m2_profile_stride(hm.handle, stride), "m2_profile_stride")
            chk(lib.m2_profile_enable(hm.handle, (steps + stride - 1) // stride), "m2_profile_enable")
        torch.cuda.synchronize(self.dev)
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(self.dev)
        self.barrier()
        el = time.perf_counter() - t0
        ms = []
        if kernel_mask:
            cap = (steps + stride - 1) // stride * self.nk
            buf = (ctypes.c_float * cap)()
            n = ctypes.c_int32(0)
            chk(lib.m2_profile_read(hm.handle, buf, cap, ctypes.byref(n)), "m2_profile_read")
            ms = list(buf[: n.value])
            lib.m2_profile_disable(hm.handle)
            chk(lib.m2_profile_stride(hm.handle, 1), "m2_profile_stride")
        return self.max_over_ranks(el), ms

    def kernel_table(self, hm, kern_ms, C, M, B, T):
        fl = vocoder_kernel_flops_per_frame(C, M)
        _, peak, _ = VOC_PATHS[self.lib.m2_vocoder_path(hm.handle)]
        rows = []
        for i in range(self.nk):
            vals = [v for v in kern_ms[i::self.nk] if v >= 0]
            if not vals:
                continue
            avg = sum(vals) / len(vals)
            flops = fl[i] * B * T
            tf = flops / (avg * 1e-3) / 1e12
            rows.append({"index": i, "kernel": self.lib.m2_profile_kernel_name_for(hm.handle, i).decode(),
                         "avg_ms": round(avg, 5), "launches": len(vals), "algorithmic_flop_per_launch": flops,
                         "tflops": round(tf, 3), "frac_of_peak": round(tf / peak, 4)})
        return rows


def traffic_for(kernel_name: str):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (not measured in this run)."""
    tf = ROOT / "profiles" / "traffic.json"
    if not tf.exists():
        return None, None
    try:
        d = json.loads(tf.read_text())
    except ValueError:
        return None, None
    v = d.get(kernel_name.split()[0])
    return v, d.get("_source", "profiles/traffic.json")


def vocoder_line(cx: Ctx, stage: str, B: int, T: int, args, settle_ms: float, seed: int, f32: bool = False):
    """SimpleVocoder throughput on mel [B, M, T] per rank (weak scaling), the
    per-kernel HIP-event table, and the dominant kernel's roofline sampled
    live inside the timed region."""
    cfg = STAGE1 if stage == "s1" else STAGE2
    m = cx.model(stage)
    hm = m._hip(cx.dev)
    hm.vocoder_select(1 if f32 else 2)
    try:
        g = torch.Generator().manual_seed(seed + cx.rank)
        mel = torch.randn(B, cfg["mel_channels"], T, generator=g).to(cx.dev)
        step = lambda: m.vocoder(mel)  # noqa: E731
        settled = cx.settle(step, settle_ms)
        # untimed pass with events on all three kernels -> per-kernel table + dominant kernel
        _, all_ms = cx.timed(step, min(args.steps, 20), 2, hm, kernel_mask=(1 << cx.nk) - 1)
        per_kernel = cx.kernel_table(hm, all_ms, cfg["vocoder_channels"], cfg["mel_channels"], B, T)
        dom_i = max(per_kernel, key=lambda d: d["avg_ms"])["index"] if per_kernel else 0
        # every stride-th call carries the events (at least every 4th: 5 of the
        # driver's 20 steps): a sampled call pays ~4.5 us before and after its
        # timed kernel (profiles/r05/r05o_gaps.txt), unsampled none; every call
        # sampled cost the driver-form line ~3 % (profiles/r06/r06as_bench*.json)
        stride = max(4, args.steps // 16)
        elapsed, kern_ms = cx.timed(step, args.steps, args.warmup, hm, kernel_mask=1 << dom_i, stride=stride)
        path = cx.lib.m2_vocoder_path(hm.handle)
        # (before the path is restored: the table's kernel names and peak are this path's)
        live = cx.kernel_table(hm, kern_ms, cfg["vocoder_channels"], cfg["mel_channels"], B, T)
    finally:
        hm.vocoder_select(2)
    dtype, peak, note = VOC_PATHS[path]
    value = samples_per(B, T) * args.steps * cx.world / elapsed
    ms = elapsed / args.steps * 1e3
    roof = None
    if live:
        d = live[0]
        traffic, src = traffic_for(d["kernel"]) if (stage == "s1" and path == 2) else (None, None)
        roof = {"bound": "mfma", "achieved": d["tflops"], "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(d["tflops"] / peak, 4), "traffic": traffic,
                "traffic_source": (f"static: {src} (rocprofv3 PMC passes, 2*FETCH_SIZE + WRITE_SIZE per launch); "
                                   "not measured in this run") if traffic is not None else None,
                "kernel": d["kernel"], "avg_kernel_ms": d["avg_ms"], "launches": d["launches"],
                "event_stride": stride, "algorithmic_flop_per_launch": d["algorithmic_flop_per_launch"],
                "dtype_peak_note": note}
    flop_s = vocoder_flops_per_sample(cfg["vocoder_channels"], cfg["mel_channels"])
    voc_s = ms * 1e-3
    # north_star "rocprof GB/s vs peak" for the whole vocoder step: the three
    # kernels' PMC bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950
    # correction, profiles/traffic.json) / this run's step time
    hbm = None
    if stage == "s1" and path == 2 and B == 32 and T == 500:
        per = [traffic_for(d["kernel"])[0] for d in per_kernel]
        if per and all(v is not None for v in per):
            gbs = sum(per) / voc_s / 1e9
            hbm = {"hbm_gbs": round(gbs, 1), "frac_of_8tbs": round(gbs / HBM_PEAK_GBS, 4),
                   "bytes_per_step": sum(per),
                   "def": "sum over the 3 vocoder kernels of PMC bytes per launch (2*FETCH_SIZE + WRITE_SIZE, "
                          "static: " + (traffic_for("_source")[0] or "profiles/traffic.json") + ") / this run's "
                          "ms_per_step, against 8 TB/s"}
    out = {"value": round(value, 1), "ms_per_step": round(ms, 5), "dtype": dtype, "settle_ms": round(settled, 1),
           "config": {"stage": stage, "per_gpu_batch": B, "mel_frames": T, "audio_samples_per_utt": 64 * T},
           "roofline": roof, "vocoder_kernels": per_kernel,
           "vocoder_flop_per_sample": flop_s, "vocoder_hbm": hbm,
           "vocoder_tflops": round(value / cx.world * flop_s / 1e12, 3),
           # SURVEY.md 8d "MRF HBM fraction": sum of the 4 resblocks' per-kernel algorithmic
           # bytes / the whole fused vocoder's time per step / 8 TB/s (the resblocks are fused
           # with the ConvTs, so their own time is not separable: this is a lower bound)
           "mrf_hbm_fraction": round(mrf_bytes(cfg["vocoder_channels"], B, T) / voc_s / (HBM_PEAK_GBS * 1e9), 4),
           "mrf_hbm_fraction_def": "sum(resblock bytes 8cL + weights, SURVEY 8d) / whole-vocoder step time / 8 TB/s",
           "fp32_valu_fraction": round(value / cx.world * flop_s / (FP32_PEAK_TFLOPS * 1e12), 4),
           "fp32_valu_fraction_def": "algorithmic vocoder FLOP/s / 157.3 TF (MI355X fp32 vector peak)"}
    return out


def report_policy_line(cx: Ctx, B: int, T: int, args, head: dict):
    """The headline vocoder workload on the opt-in "report" range policy (a
    non-finite split-f16 result raises on the next call) - what the default
    "fallback" policy of the headline costs per call: the pipelined tail's
    workgroup-local non-finite word and the barrier before its in-launch fp32
    redo, which runs only for a strip whose audio is not finite (round 5; a
    guarded exact-f32 launch behind the tail with M2_REDO_LAUNCH=1).  Measured like for
    like: both policies timed exactly as the headline is (same steps, the
    same fence-free events on the dominant kernel every stride-th call),
    alternated three times in this process; the cost is the difference of
    the medians.  (Comparing this line with the headline's own figure mixes
    in the clock drift between two separate runs.)"""
    m = cx.model("s1")
    hm = m._hip(cx.dev)
    g = torch.Generator().manual_seed(1000 + cx.rank)
    mel = torch.randn(B, STAGE1["mel_channels"], T, generator=g).to(cx.dev)
    roof = head.get("roofline") or {}
    dom = [d["index"] for d in head.get("vocoder_kernels", []) if d["kernel"] == roof.get("kernel")]
    mask = 1 << dom[0] if dom else 0
    stride = roof.get("event_stride", 1)
    step = lambda: m.vocoder(mel)  # noqa: E731
    res = {"fallback": [], "report": []}
    try:
        for _ in range(3):
            for pol in ("fallback", "report"):
                m.set_range_policy(pol)
                cx.settle(step, 20.0)
                elapsed, _ = cx.timed(step, args.steps, 3, hm if mask else None, kernel_mask=mask, stride=stride)
                res[pol].append(elapsed / args.steps * 1e3)
    finally:
        m.set_range_policy("fallback")
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    return {"value": round(samples_per(B, T) * cx.world / (med["report"] * 1e-3), 1),
            "ms_per_step": round(med["report"], 5), "steps": args.steps, "range_policy": "report",
            "default_policy_ms_per_step_same_runs": round(med["fallback"], 5),
            "default_policy_cost_ms_per_call": round(med["fallback"] - med["report"], 5),
            "runs_ms": {k: [round(x, 5) for x in v] for k, v in res.items()},
            "method": "fallback and report alternated 3x in one process, each timed like the headline "
                      "(same steps and event sampling); cost = difference of the medians"}


def pipeline_line(cx: Ctx, B: int, S: int, args, settle_ms: float):
    m = cx.model("s1")
    g = torch.Generator().manual_seed(1000 + cx.rank)
    ids = torch.randint(0, 42, (B, S), generator=g).to(cx.dev)
    lens = torch.full((B,), S, dtype=torch.long, device=cx.dev)
    step = lambda: m.inference(ids, lens)  # noqa: E731
    settled = cx.settle(step, settle_ms)
    steps = max(10, args.steps // 2)
    elapsed, _ = cx.timed(step, steps, max(3, args.warmup // 2))
    T = 5 * S
    # the frame counts and how far the durations sit from the
    # int() truncation points (a duration within ~1e-6 of an integer could
    # flip a frame count between the GPU and the CPU path)
    with torch.no_grad():
        mel, _ = m.inference(ids, lens)
        dur = m(ids, lens)["duration_pred"].double()
    tot = torch.trunc(dur).clamp(min=0).sum(1).to(torch.int64).cpu()
    frames = {"gpu_T_per_utt": tot.tolist(), "T": int(mel.shape[1]),
              "T_is_batch_max": int(mel.shape[1]) == max(1, int(tot.max())),
              "min_duration_dist_to_int": float((dur - dur.round()).abs().min()),
              "ids_seed": 1000 + cx.rank}
    return {"value": round(samples_per(B, T) * steps * cx.world / elapsed, 1),
            "ms_per_step": round(elapsed / steps * 1e3, 5), "steps": steps, "settle_ms": round(settled, 1),
            "scaling": "weak", "frames": frames,
            "config": {"workload": "stage1_poc M2TTSModel.inference (configs[2])",
                       "per_gpu_batch": B, "global_batch": B * cx.world, "phonemes": S, "mel_frames": T}}


def sharded_line(cx: Ctx, Bg: int, S: int, chunk: int, args, settle_ms: float, steps: int, share: bool = False,
                 depth: int = 1):
    """stage2 inference over a global batch of Bg utterances sharded across the
    ranks (configs[3] / [4]): per step the front half (T_max into a device
    word), RCCL all_reduce(MAX) of that word, the back half reading T from it
    and a gather of mel / audio to rank 0.  depth > 1: ShardedPipeline with
    that many global batches in flight per rank (one stream and model handle
    per lane; step i + 1's front half beside step i's back half and gather)."""
    from m2amd.parallel import ShardedPipeline, hip_stages, shard_bounds, sharded_inference
    import torch.distributed as td
    m = cx.model("s2")
    m.set_vocoder_chunking(chunk)
    try:
        g = torch.Generator().manual_seed(2024)  # every rank draws the same global batch
        ids = torch.randint(0, 42, (Bg, S), generator=g).to(cx.dev)
        lens = torch.full((Bg,), S, dtype=torch.long, device=cx.dev)
        st = hip_stages(m)
        # the global batch's mel / audio are gathered to rank 0 (RCCL gather over xGMI)
        # share: one rank's two-phase flow (front, T exchange, back) timed alone
        if depth > 1:
            pipe = ShardedPipeline(m, depth=depth, gather_to=0)
            prev = [None]

            def step():
                r = pipe.submit(ids, lens)
                if prev[0] is not None:
                    prev[0].wait()
                prev[0] = r
                return r

            mel, audio = pipe.submit(ids, lens).wait()
        else:
            step = lambda: sharded_inference(st, ids, lens, gather_to=0, one_call_world1=not share)  # noqa: E731
            mel, audio = step()
        T = 5 * S  # pinned durations: every utterance has 5 frames per phoneme
        if cx.rank == 0:
            assert mel.shape == (Bg, T, 80) and audio.shape == (Bg, 1, 64 * T)
        settled = cx.settle(step, settle_ms)
        elapsed, _ = cx.timed(step, steps, 2)
        # the outputs of one more step against a world-1 inference of the same
        # global batch on rank 0 (tts_model.py:402-438): the first multi-GPU
        # run checks its own gathered results
        if depth > 1:
            if prev[0] is not None:
                prev[0].wait()
                prev[0] = None
            mel, audio = pipe.submit(ids, lens).wait()
        else:
            mel, audio = step()
        parity = None
        if cx.rank == 0:
            with torch.no_grad():
                rmel, raudio = m.inference(ids, lens)
            T_eq = tuple(mel.shape) == tuple(rmel.shape) and tuple(audio.shape) == tuple(raudio.shape)
            parity = {"reference": "world-1 M2TTSModel.inference of the global batch on rank 0",
                      "T_equal": T_eq, "bitwise_equal": bool(T_eq and torch.equal(mel, rmel) and
                                                             torch.equal(audio, raudio))}
            if T_eq:
                parity["mel_maxabs"] = float((mel - rmel).abs().max())
                parity["audio_rms"] = float((audio.double() - raudio.double()).pow(2).mean().sqrt())
                parity["within_tolerance"] = parity["mel_maxabs"] <= 1e-3 and parity["audio_rms"] <= 1e-4
            # the same rows as world-1 inference() calls of each rank's shard:
            # a rank's kernels pick their tilings (e.g. the attention form) by
            # ITS batch size, so against the whole-batch call the bits may
            # differ at ~1e-6 when the shard size changes the tiling (world 4
            # and 8 of configs[3]); every utterance of this batch has T = 5 S,
            # so a shard's own T is the global T and this reference is exact
            with torch.no_grad():
                sh = [m.inference(ids[a:b], lens[a:b]) for a, b in
                      (shard_bounds(Bg, cx.world, r) for r in range(cx.world)) if b > a]
            smel, saudio = torch.cat([x[0] for x in sh]), torch.cat([x[1] for x in sh])
            parity["bitwise_equal_shardwise"] = bool(tuple(smel.shape) == tuple(mel.shape) and torch.equal(mel, smel)
                                                     and torch.equal(audio, saudio))
        # split of one step on the device-T flow the timed line uses (rank-local
        # wall times): front half writing T_max to a device word, all_reduce(MAX)
        # of that word, back half launched for the capacity reading T from it
        lo, hi = shard_bounds(Bg, cx.world, cx.rank)
        hm = m._hip(cx.dev)
        cap = st.tcap.get((Bg, S, 1.0), T)
        M = 80
        mel_o = torch.empty(max(1, hi - lo) * cap * M, dtype=torch.float32, device=cx.dev)
        aud_o = torch.empty(max(1, hi - lo) * 64 * cap, dtype=torch.float32, device=cx.dev)
        tw = torch.empty(1, dtype=torch.int32, device=cx.dev)
        # the timed flow: device-T when the handle supports the capacity (not
        # with the long-form's streamed vocoder), else the host-T two-phase flow
        dev_T = hm.dev_supported(cap)
        # host wall phases and GPU-elapsed (events on the launch stream) of the
        # two halves, median of 21 steps: host-bound iff wall >> GPU-elapsed
        ph = []
        for _ in range(21):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            torch.cuda.synchronize(cx.dev)
            t0 = time.perf_counter()
            ev[0].record()
            if dev_T:
                state = hm.inference_front_dev(ids[lo:hi], lens[lo:hi], 1.0, tw)
            else:
                state, tl = hm.inference_front(ids[lo:hi], lens[lo:hi], 1.0)
                tw.fill_(tl)
            ev[1].record()
            t1 = time.perf_counter()
            if cx.dist:
                if cx.backend == "RCCL":
                    td.all_reduce(tw, op=td.ReduceOp.MAX)
                else:
                    t = tw.cpu()
                    td.all_reduce(t, op=td.ReduceOp.MAX)
                    tw.copy_(t)
            t2 = time.perf_counter()
            ev[2].record()
            if dev_T:
                hm.inference_back_dev(state, cap, tw, mel_o, aud_o)
            else:
                hm.inference_back(state, max(1, int(tw.item())))
            ev[3].record()
            t3 = time.perf_counter()
            torch.cuda.synchronize(cx.dev)
            t4 = time.perf_counter()
            ph.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3,
                       ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])))
        med = [sorted(c)[len(c) // 2] for c in zip(*ph)]
    finally:
        m.set_vocoder_chunking(0)
    return {"value": round(samples_per(Bg, T) * steps / elapsed, 1), "ms_per_step": round(elapsed / steps * 1e3, 4),
            "steps": steps, "settle_ms": round(settled, 1), "scaling": "strong", "in_flight": depth,
            "rtf_x_realtime": round(samples_per(Bg, T) * steps / elapsed / SAMPLE_RATE, 1),
            "config": {"stage": "stage2_quality", "global_batch": Bg, "per_gpu_batch": hi - lo, "phonemes": S,
                       "mel_frames": T, "vocoder_chunk_frames": chunk, "n_ranks": cx.world,
                       "collectives": f"all_reduce(MAX) 1 x int32 + gather of mel/audio to rank 0 ({cx.backend})" if cx.dist
                       else "none (world 1)"},
            "parity": parity,
            "rank0_phase_ms": {"front_enqueue": round(med[0], 3), "all_reduce_enqueue": round(med[1], 3),
                               "back_enqueue": round(med[2], 3), "drain": round(med[3], 3),
                               "front_gpu_elapsed": round(med[4], 3), "back_gpu_elapsed": round(med[5], 3),
                               "flow": "device-T" if dev_T else "host-T (streamed vocoder)",
                               "def": "the timed line's flow - device-T: m2_inference_front_dev -> all_reduce(MAX) "
                                      "of the device word -> m2_inference_back_dev at the learnt capacity; host-T: "
                                      "m2_inference_front (T_max read) -> all_reduce -> m2_inference_back - median "
                                      "of 21 steps; "
                                      "*_gpu_elapsed = HIP events on the launch stream around each half (GPU "
                                      "time incl. any launch gaps); gloo stages the all_reduce through the host"}}


class _Progress(dict):
    """The extras dict; every line stored prints a progress note to stderr (a
    multi-line run is otherwise silent until its one JSON line)."""

    def __init__(self, rank: int):
        super().__init__()
        self.rank, self.t0 = rank, time.perf_counter()

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        ms = value.get("ms_per_step") if isinstance(value, dict) else None
        print(f"[bench rank {self.rank}] {key}: {ms} ms/step ({time.perf_counter() - self.t0:.1f} s)",
              file=sys.stderr, flush=True)


def run(args):
    if args.dry_run:
        return dry_run(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = local % max(1, torch.cuda.device_count())  # gloo rehearsal: ranks may share a GPU
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            td.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            td.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cx = Ctx(dev, world, rank, dist)
    cx.backend = "RCCL" if args.dist_backend == "nccl" else "gloo"
    B, S = args.batch, args.phonemes
    wl = args.workload
    extras = _Progress(rank)

    if wl == "vocoder":
        head = vocoder_line(cx, "s1", B, 5 * S, args, args.settle_ms, 1000)
        desc = "stage1_poc SimpleVocoder B=32 per GPU (configs[1])"
    elif wl == "s2_vocoder":
        b2, t2 = (int(v) for v in args.s2_shape.split("x"))
        head = vocoder_line(cx, "s2", b2, t2, args, args.settle_ms, 3000)
        desc = f"stage2_quality SimpleVocoder B={b2} T={t2} per GPU (configs[3] per-GPU shape: 8x500)"
    elif wl == "pipeline":
        head = pipeline_line(cx, B, S, args, args.settle_ms)
        desc = head["config"]["workload"]
    else:
        Bg, Sg, chunk = (64, 100, 0) if wl == "s2_b64" else (128, 520, 256)
        head = sharded_line(cx, Bg, Sg, chunk, args, args.settle_ms, args.steps if wl == "s2_b64" else
                            max(5, args.steps // 10))
        desc = f"stage2_quality M2TTSModel.inference global B={Bg} S={Sg} sharded x{world} ({wl}, configs[" \
               f"{3 if wl == 's2_b64' else 4}])"

    print(f"[bench rank {rank}] {wl}: {head['ms_per_step']} ms/step", file=sys.stderr, flush=True)
    if not args.no_extras:
        if wl != "pipeline":
            extras["pipeline"] = pipeline_line(cx, B, S, args, 100.0)
        if wl == "vocoder":
            extras["vocoder_report_policy"] = report_policy_line(cx, B, 5 * S, args, head)
            f32 = vocoder_line(cx, "s1", B, 5 * S, args, 100.0, 1000, f32=True)
            extras["vocoder_exact_f32"] = {k: f32[k] for k in ("value", "ms_per_step", "dtype", "roofline",
                                                              "vocoder_kernels", "vocoder_tflops")}
            # the strict-fp32 figure's own roofline at the top level (fp32 MFMA
            # peak 157.3 TF): the credited number for a reader who does not
            # accept the split-f16 arithmetic
            strict = f32.get("roofline")
            if strict:
                strict = {**strict, "value": f32["value"], "ms_per_step": f32["ms_per_step"], "dtype": f32["dtype"]}
            extras["roofline_exact_f32"] = strict
        if wl != "s2_vocoder":
            s2v = vocoder_line(cx, "s2", 8, 500, args, 100.0, 3000)
            extras["s2_vocoder_b8_t500"] = s2v
        s2l = vocoder_line(cx, "s2", 16, 2600, type(args)(**{**vars(args), "steps": max(5, args.steps // 10)}),
                           100.0, 4000)
        extras["s2_vocoder_b16_t2600"] = s2l
        if wl != "s2_b64":
            extras["s2_b64_sharded"] = sharded_line(cx, 64, 100, 0, args, 100.0, max(10, args.steps // 4))
        if world == 1:
            # the per-GPU share of configs[3] at N=8 (8 utterances), run alone:
            # what bounds a small per-GPU batch (host phases vs GPU-elapsed)
            extras["s2_b8_per_gpu_share"] = sharded_line(cx, 8, 100, 0, args, 100.0, max(20, args.steps // 2),
                                                         share=True)
            # the same share with two global batches in flight (ShardedPipeline)
            extras["s2_b8_per_gpu_share_2inflight"] = sharded_line(cx, 8, 100, 0, args, 100.0,
                                                                   max(20, args.steps // 2), share=True, depth=2)
        if wl != "s2_b64":
            extras["s2_b64_sharded_2inflight"] = sharded_line(cx, 64, 100, 0, args, 100.0, max(10, args.steps // 4),
                                                              depth=2)
        if wl != "s2_longform":
            extras["s2_longform_sharded"] = sharded_line(cx, 128, 520, 256, args, 100.0, max(3, args.steps // 40))

    out = {"metric": METRIC, "value": head["value"], "unit": "audio samples/s", "n_gpus": world,
           "steps": args.steps if wl != "pipeline" else head["steps"], "warmup": args.warmup,
           "ms_per_step": head["ms_per_step"], "higher_is_better": True,
           "scaling": head.get("scaling", "weak"), "vs_baseline": None,
           "dtype": head.get("dtype", VOC_PATHS[2][0]),
           "data": "synthetic (seeded N(0,1) mel / U{0..41} phoneme ids; random-init weights, seed 1234, "
                   "durations pinned to 5 frames/phoneme)",
           "config": {"workload": desc, **head["config"],
                      "parallelism": (f"weak-scaled replicas x{world} (dp{world}, no collective in the data path)"
                                      if head.get("scaling", "weak") == "weak" else
                                      f"utterance-sharded x{world} (RCCL all_reduce + all_gather)")},
           "settle_ms": head["settle_ms"],
           "range_policy": "fallback (the public default; the opt-in report policy: vocoder_report_policy)",
           "rtf_x_realtime": round(head["value"] / SAMPLE_RATE, 1),
           "rtf_x_realtime_per_gpu": round(head["value"] / SAMPLE_RATE / world, 1)}
    for k in ("roofline", "vocoder_kernels", "vocoder_hbm", "vocoder_flop_per_sample", "vocoder_tflops", "mrf_hbm_fraction",
              "mrf_hbm_fraction_def", "fp32_valu_fraction", "fp32_valu_fraction_def", "rank0_phase_ms"):
        if k in head:
            out[k] = head[k]
    out.update(extras)
    # the driver keeps only the contract keys of the line: the strict-fp32
    # roofline rides inside `roofline` so it reaches the record
    if isinstance(out.get("roofline"), dict) and extras.get("roofline_exact_f32"):
        out["roofline"]["exact_f32"] = extras["roofline_exact_f32"]

    if rank == 0 and world == 1 and not args.no_cpu_baseline and wl in ("vocoder", "pipeline"):
        pipe = out.get("pipeline") if wl == "vocoder" else head
        cb = cpu_baseline(B, S, 5 * S, runs=args.cpu_runs,
                          ids_seed=pipe["frames"]["ids_seed"] if isinstance(pipe, dict) and "frames" in pipe else None)
        if "value" in cb:
            cb["gpu_over_cpu"] = round(out["value"] / cb["value"], 1)
            # the ratio moves with the CPU figure: its range over the kept runs
            cb["gpu_over_cpu_range"] = [round(out["value"] / cb["max"], 1), round(out["value"] / cb["min"], 1)]
            if isinstance(pipe, dict):
                cb["inference_as_written"]["gpu_pipeline_over_cpu"] = round(
                    pipe["value"] / cb["inference_as_written"]["value"], 1)
                fr, cf = pipe.get("frames"), cb.pop("frames", None)
                if fr and cf:  # T equality GPU vs the reference's CPU op sequence
                    fr["cpu_T_per_utt_equal"] = fr["gpu_T_per_utt"] == cf["cpu_T_per_utt"]
                    fr["cpu_min_duration_dist_to_int"] = cf["min_duration_dist_to_int"]
                    fr.pop("gpu_T_per_utt")
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        import torch.distributed as td
        td.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if "--cpu-child" in argv:
        return cpu_child_main(json.loads(argv[argv.index("--cpu-child") + 1]))
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args, argv)
        return
    run(args)


if __name__ == "__main__":
    main()
