"""GPU: the device-side frame count (speculative back half).

m2_inference enqueues the expansion / decoder / vocoder right behind the count
kernel, before the host reads T_max, with grids sized for the frame capacity
of the caller's buffers; the kernels take T = max(1, T_max) from the device
(dev_frames) and do nothing when T outgrows the capacity.  The sharded path's
m2_inference_front_dev / m2_inference_back_dev keep T on the device across the
ranks' all-reduce.  Checked against the host-T path (M2_SPECULATIVE=0 /
m2_inference_back at the exact T) bit for bit, the fixtures and the oracle
(reference: tts_model.py:158-176 - T is the batch maximum, max(1, .))."""
import os
import socket

import numpy as np
import pytest
import torch

import m2tts_oracle as orc
from conftest import AUDIO_RMS_TOL, MEL_MAXABS_TOL, golden, golden_state, maxabs, rms, stage_config

pytestmark = pytest.mark.gpu


def build_model(stage, dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config(stage).as_dict())
    m.load_state_dict(golden_state(stage))
    return m.to(dev).eval()


def _host_path(m, ids, lens, scale, monkeypatch):
    monkeypatch.setenv("M2_SPECULATIVE", "0")
    try:
        return m.inference(ids, lens, duration_scale=scale)
    finally:
        monkeypatch.delenv("M2_SPECULATIVE")


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_speculative_inference_equals_host_path(gpu, stage, monkeypatch):
    """A sequence of calls whose T shrinks under the capacity, grows past it
    (the speculative launches do nothing; the call finishes at the exact T)
    and repeats: every result equals the host-T path bit for bit."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(5)
    B, S = 6, 40
    ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
    lens = torch.tensor([40, 13, 27, 40, 1, 33]).to(gpu)
    seen_spec = False
    for scale in (1.0, 1.0, 0.8, 0.6, 1.4, 1.4, 1.0):
        cap = hm._tcap.get((B, S), 0)
        mel, audio = m.inference(ids, lens, duration_scale=scale)
        hmel, haudio = _host_path(m, ids, lens, scale, monkeypatch)
        assert mel.shape == hmel.shape and audio.shape == haudio.shape
        assert torch.equal(mel, hmel) and torch.equal(audio, haudio), (scale, cap, mel.shape)
        seen_spec |= 0 < mel.shape[1] <= cap
    assert seen_spec


def test_speculative_inference_fixture_and_oracle(gpu):
    """configs[3]'s fixture batch (B=64, S=100) on the speculative path: the
    reference fingerprints and the oracle on three rows."""
    from test_gpu_parity import _check_fingerprint
    fp = golden("fp_s2_B64_S100")
    m = build_model("s2", gpu)
    ids, lens = torch.from_numpy(fp["ids"]).to(gpu), torch.from_numpy(fp["lengths"]).to(gpu)
    m.inference(ids, lens)  # learns the capacity
    assert m._hip(gpu)._tcap[tuple(ids.shape)] > 0
    mel, audio = m.inference(ids, lens)
    _check_fingerprint(fp, mel, audio)
    rows = [1, 40]
    ref_mel, ref_audio = orc.inference(golden_state("s2"), stage_config("s2"), ids[rows].cpu(), lens[rows].cpu(),
                                       as_written=False)
    assert maxabs(mel[rows], ref_mel) <= MEL_MAXABS_TOL
    assert rms(audio[rows], ref_audio) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_back_dev_direct(gpu, stage):
    """HipModel.inference_front_dev / inference_back_dev: T from the device
    word at capacities T, T + 5 and 2T equal inference_back at the exact T;
    a capacity under T leaves the outputs untouched."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    M = stage_config(stage).mel_channels
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(0, 42, (3, 24), generator=g).to(gpu)
    lens = torch.tensor([24, 9, 17]).to(gpu)
    st, T = hm.inference_front(ids, lens, 1.0)
    rmel, raudio = hm.inference_back(st, max(1, T))
    T = max(1, T)
    for cap in (T, T + 5, 2 * T, T - 1):
        if cap <= 0 or not hm.dev_supported(cap):
            continue
        tw = torch.empty(1, dtype=torch.int32, device=gpu)
        st = hm.inference_front_dev(ids, lens, 1.0, tw)
        mel_out = torch.full((3 * cap * M,), float("nan"), device=gpu)
        audio_out = torch.full((3 * 64 * cap,), float("nan"), device=gpu)
        hm.inference_back_dev(st, cap, tw, mel_out, audio_out)
        assert hm.frames_wait() == T  # posted by the first launch, also past the capacity
        torch.cuda.synchronize()
        assert int(tw.item()) == T
        if cap < T:
            assert torch.isnan(mel_out).all() and torch.isnan(audio_out).all()
            continue
        assert torch.equal(mel_out[: 3 * T * M].view(3, T, M), rmel)
        assert torch.equal(audio_out[: 3 * 64 * T].view(3, 1, 64 * T), raudio)


@pytest.mark.parametrize("B", [8, 64])
def test_sharded_device_T_world1(gpu, B):
    """sharded_inference(..., one_call_world1=False) - the flow of one rank of
    a multi-GPU job: the first step learns the capacity on the host path, the
    next ones keep T on the device; bit for bit equal to inference()."""
    from m2amd.parallel import hip_stages, sharded_inference
    m = build_model("s2", gpu)
    st = hip_stages(m)
    g = torch.Generator().manual_seed(B)
    ids = torch.randint(0, 42, (B, 100), generator=g).to(gpu)
    lens = torch.randint(20, 101, (B,), generator=g).to(gpu)
    ref_mel, ref_audio = m.inference(ids, lens)
    for _ in range(3):
        mel, audio = sharded_inference(st, ids, lens, gather_to=0, one_call_world1=False)
        assert torch.equal(mel, ref_mel) and torch.equal(audio, ref_audio)
    assert st.tcap[(B, 100, 1.0)] >= ref_mel.shape[1]
    pend = sharded_inference(st, ids, lens, one_call_world1=False, async_gather=True)
    mel, audio = pend.wait()
    assert torch.equal(mel, ref_mel) and torch.equal(audio, ref_audio)
    mel, audio, (lo, hi) = sharded_inference(st, ids, lens, gather=False, one_call_world1=False)
    assert (lo, hi) == (0, B) and torch.equal(mel, ref_mel)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dev_worker(rank, world, port, outfile):
    """Two gloo ranks sharing cuda:0 on the device-T path (gloo stages the
    one-word all-reduce through the host); a batch smaller than the world on
    the last step gives rank 1 an empty shard."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m2amd.parallel import hip_stages, sharded_inference
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        m = build_model("s1", dev)
        st = hip_stages(m)
        g = torch.Generator().manual_seed(21)
        ids = torch.randint(0, 42, (5, 30), generator=g)
        lens = torch.tensor([30, 12, 25, 7, 30])
        outs = {}
        for i, scale in enumerate((1.0, 1.0, 0.7, 1.6, 1.0)):
            mel, audio = sharded_inference(st, ids.to(dev), lens.to(dev), duration_scale=scale)
            outs[f"mel{i}"], outs[f"audio{i}"] = mel.cpu().numpy(), audio.cpu().numpy()
        for i in range(2):  # B = 1 < world: rank 1's shard is empty
            mel, audio = sharded_inference(st, ids[:1].to(dev), lens[:1].to(dev))
            outs[f"one{i}"] = mel.cpu().numpy()
        # only rank 0 holds the inputs, as host tensors: broadcast to the
        # model's device on every rank, so both ranks take the same (device-T
        # from the second step) path and issue the same collectives
        for i in range(3):
            mel, audio = sharded_inference(st, ids if rank == 0 else None, lens if rank == 0 else None, src=0)
            outs[f"src{i}"], outs[f"srca{i}"] = mel.cpu().numpy(), audio.cpu().numpy()
        if rank == 0:
            np.savez(outfile, ids=ids.numpy(), lens=lens.numpy(), **outs)
    finally:
        dist.destroy_process_group()


def test_sharded_device_T_two_ranks_gloo(gpu, tmp_path):
    import torch.multiprocessing as mp
    outfile = str(tmp_path / "dev.npz")
    mp.spawn(_dev_worker, args=(2, _free_port(), outfile), nprocs=2, join=True)
    z = np.load(outfile)
    m = build_model("s1", gpu)
    ids, lens = torch.from_numpy(z["ids"]).to(gpu), torch.from_numpy(z["lens"]).to(gpu)
    for i, scale in enumerate((1.0, 1.0, 0.7, 1.6, 1.0)):
        mel, audio = m.inference(ids, lens, duration_scale=scale)
        assert torch.equal(torch.from_numpy(z[f"mel{i}"]), mel.cpu()), i
        assert torch.equal(torch.from_numpy(z[f"audio{i}"]), audio.cpu()), i
    mel1, _ = m.inference(ids[:1], lens[:1])
    for i in range(2):
        assert torch.equal(torch.from_numpy(z[f"one{i}"]), mel1.cpu())
    for i in range(3):
        assert torch.equal(torch.from_numpy(z[f"src{i}"]), torch.from_numpy(z["mel0"])), i
        assert torch.equal(torch.from_numpy(z[f"srca{i}"]), torch.from_numpy(z["audio0"])), i


@pytest.mark.parametrize("depth", [2, 3])
def test_sharded_pipeline_world1(gpu, depth):
    """ShardedPipeline: several global batches in flight on their own streams
    and handles; each result equals inference() on its inputs bit for bit
    (batches alternate between two inputs of different T, so lanes also
    cross the capacity bookkeeping)."""
    from m2amd.parallel import ShardedPipeline
    m = build_model("s2", gpu)
    g = torch.Generator().manual_seed(depth)
    batches = []
    for k in range(2):
        ids = torch.randint(0, 42, (8, 100), generator=g).to(gpu)
        lens = torch.randint(30 + 40 * k, 101, (8,), generator=g).to(gpu)
        batches.append((ids, lens, m.inference(ids, lens)))
    pipe = ShardedPipeline(m, depth=depth)
    pend = []
    for i in range(7):
        ids, lens, _ = batches[i % 2]
        pend.append((pipe.submit(ids, lens), i % 2))
        if len(pend) > depth:
            r, k = pend.pop(0)
            mel, audio = r.wait()
            assert torch.equal(mel, batches[k][2][0]) and torch.equal(audio, batches[k][2][1])
    for r, k in pend:
        mel, audio = r.wait()
        assert torch.equal(mel, batches[k][2][0]) and torch.equal(audio, batches[k][2][1])


def test_sharded_pipeline_interleaved_with_inference(gpu):
    """Pipeline lanes use handles of their own: model.inference() on the
    caller's stream, between submits whose steps are still in flight, shares
    no device state (work-queue counters, frame mailbox) with them."""
    from m2amd.parallel import ShardedPipeline
    m = build_model("s2", gpu)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 42, (8, 100), generator=g).to(gpu)
    lens = torch.randint(30, 101, (8,), generator=g).to(gpu)
    ids2 = torch.randint(0, 42, (6, 64), generator=g).to(gpu)
    lens2 = torch.randint(10, 65, (6,), generator=g).to(gpu)
    ref = m.inference(ids, lens)
    ref2 = m.inference(ids2, lens2)
    pipe = ShardedPipeline(m, depth=2)
    pend = []
    for i in range(6):
        pend.append(pipe.submit(ids, lens))
        mel2, audio2 = m.inference(ids2, lens2)
        assert torch.equal(mel2, ref2[0]) and torch.equal(audio2, ref2[1]), i
        if len(pend) > 2:
            mel, audio = pend.pop(0).wait()
            assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1]), i
    for r in pend:
        mel, audio = r.wait()
        assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1])


@pytest.mark.parametrize("stage,B,S,scale", [("s2", 8, 100, 1.0), ("s1", 64, 128, 1.0), ("s1", 65, 128, 1.0),
                                             ("s2", 3, 700, 1.7), ("s1", 5, 40, 0.0), ("s1", 1, 1, 1.0),
                                             ("s2", 16, 100, 0.45)])
def test_fused_frame_count_equals_count_kernel(gpu, stage, B, S, scale, monkeypatch):
    """The frame count run by the duration kernel's last workgroup (durations
    handed over with write-through stores and a ticket; M2_DUR_COUNT=1 forces
    it up to B*S = 8192, the default fuses up to 2048) leaves the front buffer - durations, prefix sums,
    totals - and the T_max word bit for bit as the separate count kernel
    (M2_DUR_COUNT=0) does, over repeated calls (the ticket is reset by the
    last workgroup) and ragged lengths (tts_model.py:146-166)."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(B * 1000 + S)
    ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
    lens = torch.randint(1, S + 1, (B,), generator=g).to(gpu)
    res = {}
    for mode in ("0", "1", "1", "0", "1"):
        monkeypatch.setenv("M2_DUR_COUNT", mode)
        tword = torch.full((1,), -7, dtype=torch.int32, device=gpu)
        state = hm.inference_front_dev(ids, lens, scale, tword)
        torch.cuda.synchronize(gpu)
        got = (state[2].clone(), int(tword.item()))
        if mode in res:
            assert torch.equal(got[0], res[mode][0]) and got[1] == res[mode][1]
        res[mode] = got
    assert torch.equal(res["0"][0], res["1"][0])
    assert res["0"][1] == res["1"][1] >= 0
    # and through the whole one-call inference (mailbox post from the fused count)
    monkeypatch.setenv("M2_DUR_COUNT", "0")
    mel0, audio0 = m.inference(ids, lens, duration_scale=scale)
    monkeypatch.setenv("M2_DUR_COUNT", "1")
    for _ in range(2):
        mel1, audio1 = m.inference(ids, lens, duration_scale=scale)
        assert torch.equal(mel0, mel1) and torch.equal(audio0, audio1)


def test_fused_frame_count_stress(gpu, monkeypatch):
    """The fused count's hand-off (write-through duration stores, a relaxed
    ticket, sc1 loads by the last workgroup; duration.hip) at the kernel's
    limit B*S = 8192 (hundreds of workgroups over all eight XCDs), 60 calls
    back to back with new lengths every call, each equal to the separate
    count kernel's front buffer and T_max."""
    m = build_model("s1", gpu)
    hm = m._hip(gpu)
    B, S = 64, 128
    g = torch.Generator().manual_seed(77)
    ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
    lens_all = [torch.randint(1, S + 1, (B,), generator=g).to(gpu) for _ in range(6)]
    ref = []
    monkeypatch.setenv("M2_DUR_COUNT", "0")
    for lens in lens_all:
        tw = torch.full((1,), -7, dtype=torch.int32, device=gpu)
        st = hm.inference_front_dev(ids, lens, 1.0, tw)
        torch.cuda.synchronize(gpu)
        ref.append((st[2].clone(), int(tw.item())))
    monkeypatch.setenv("M2_DUR_COUNT", "1")
    words = [torch.full((1,), -7, dtype=torch.int32, device=gpu) for _ in range(60)]
    for i in range(60):
        st = hm.inference_front_dev(ids, lens_all[i % 6], 1.0, words[i])
        if i % 6 == 5 or i == 59:
            torch.cuda.synchronize(gpu)
            assert torch.equal(st[2], ref[i % 6][0]), i
    torch.cuda.synchronize(gpu)
    for i in range(60):
        assert int(words[i].item()) == ref[i % 6][1], i


@pytest.mark.parametrize("stage,B,S", [("s2", 64, 100), ("s1", 3, 1), ("s1", 9, 31), ("s2", 5, 61), ("s1", 40, 45)])
def test_duration_two_row_block_tiles_bit_identical(gpu, stage, B, S, monkeypatch):
    """30-phoneme duration tiles (two 16-position row blocks per wave sharing
    each weight fragment; the default once 14-phoneme tiles exceed 256
    workgroups) give the 14-phoneme tiles' durations, encoder output and
    inference results bit for bit (the same MFMA chain per output), and both
    match the oracle (tts_model.py:99-117)."""
    m = build_model(stage, gpu)
    g = torch.Generator().manual_seed(B * 100 + S)
    ids = torch.randint(0, 42, (B, S), generator=g)
    lens = torch.randint(1, S + 1, (B,), generator=g)
    out = {}
    for rb in ("1", "2"):
        monkeypatch.setenv("M2_DUR_RB", rb)
        with torch.no_grad():
            d = m(ids.to(gpu), lens.to(gpu))["duration_pred"]
        out[rb] = (d.clone(),) + tuple(t.clone() for t in m.inference(ids.to(gpu), lens.to(gpu)))
    for a, b in zip(out["1"], out["2"]):
        assert a.shape == b.shape and torch.equal(a, b)
    sd = golden_state(stage)
    enc, _ = orc.text_encoder(sd, stage_config(stage), ids, lens)
    ref = orc.duration_predictor(sd, enc)
    assert maxabs(out["2"][0], ref) <= 1e-4  # test_gpu_parity.py ENC_TOL


@pytest.mark.parametrize("stage,B,S", [("s2", 8, 100), ("s1", 32, 100), ("s2", 64, 100), ("s1", 3, 17), ("s2", 40, 61)])
def test_duration_split_convs(gpu, stage, B, S, monkeypatch):
    """The duration convs of the inference path on split-f16 MFMA
    (hi.hi + lo.hi + hi.lo, fp32 accumulate; the model's static bound allows
    it) against the exact-f32 MFMA convs (M2_DUR_SPLIT=0): durations within
    2e-6 relative, the frame counts, prefix sums and T_max identical, and the
    oracle's durations within the fixture tolerance (tts_model.py:99-117)."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(B * 7 + S)
    ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
    lens = torch.randint(1, S + 1, (B,), generator=g).to(gpu)
    H = stage_config(stage).hidden_dim
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("M2_DUR_SPLIT", v)
        tw = torch.full((1,), -7, dtype=torch.int32, device=gpu)
        st = hm.inference_front_dev(ids, lens, 1.0, tw)
        torch.cuda.synchronize(gpu)
        front = st[2]
        # front buffer: encoder output [B,S,H] f32 then durations [B,S] f32, then int32 counts
        out[v] = (front.clone(), int(tw.item()))
    f1, f0 = out["1"][0], out["0"][0]
    nb = B * S * H * 4
    do = (nb + 255) // 256 * 256  # carve_front: 256-B aligned pieces
    enc1, enc0 = f1[:nb].view(torch.float32), f0[:nb].view(torch.float32)
    assert torch.equal(enc1, enc0)  # the fused LayerNorm is the same code
    d1 = f1[do:do + B * S * 4].view(torch.float32).view(B, S)
    d0 = f0[do:do + B * S * 4].view(torch.float32).view(B, S)
    rel = float(((d1 - d0).abs() / d0.abs().clamp(min=1e-6)).max())
    assert rel <= 2e-6, rel
    assert out["1"][1] == out["0"][1]
    assert torch.equal(torch.trunc(d1), torch.trunc(d0))
    sd = golden_state(stage)
    cfg = stage_config(stage)
    with torch.no_grad():
        enc, _ = orc.text_encoder(sd, cfg, ids.cpu(), lens.cpu())
        dref = orc.duration_predictor(sd, enc)
    assert maxabs(d1, dref) <= 1e-4


@pytest.mark.parametrize("stage,B,S", [("s2", 64, 300), ("s1", 128, 130), ("s2", 37, 517)])
def test_duration_persistent_tiles(gpu, stage, B, S, monkeypatch):
    """Grids past two rounds of the CUs run the duration kernel persistent
    (one workgroup per CU walking the tiles, weights loaded once): the same
    per-tile arithmetic as one tile per workgroup (M2_DUR_PERS=0), so the
    front buffer (encoder output, durations, counts) and T_max are bit for bit
    equal, and the durations match the oracle (tts_model.py:99-117)."""
    m = build_model(stage, gpu)
    hm = m._hip(gpu)
    g = torch.Generator().manual_seed(B * 11 + S)
    ids = torch.randint(0, 42, (B, S), generator=g).to(gpu)
    lens = torch.randint(1, S + 1, (B,), generator=g).to(gpu)
    H = stage_config(stage).hidden_dim
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("M2_DUR_PERS", v)
        tw = torch.full((1,), -7, dtype=torch.int32, device=gpu)
        st = hm.inference_front_dev(ids, lens, 1.0, tw)
        torch.cuda.synchronize(gpu)
        out[v] = (st[2].clone(), int(tw.item()))
    assert torch.equal(out["1"][0], out["0"][0])
    assert out["1"][1] == out["0"][1]
    nb = B * S * H * 4
    do = (nb + 255) // 256 * 256
    d = out["1"][0][do:do + B * S * 4].view(torch.float32).view(B, S)
    sd = golden_state(stage)
    cfg = stage_config(stage)
    with torch.no_grad():
        enc, _ = orc.text_encoder(sd, cfg, ids.cpu(), lens.cpu())
        dref = orc.duration_predictor(sd, enc)
    assert maxabs(d, dref) <= 1e-4


_FIRST_CALL_SIDE_STREAM = r"""
import sys, torch
sys.path[:0] = [sys.argv[1] + "/m2-tts_amd/src", sys.argv[1] + "/tests", sys.argv[1] + "/oracle"]
from test_gpu_device_T import build_model
from m2amd.parallel import ShardedPipeline
dev = torch.device("cuda", 0)
m = build_model("s2", dev)
g = torch.Generator().manual_seed(9)
ids = torch.randint(0, 42, (8, 100), generator=g).to(dev)
lens = torch.randint(30, 101, (8,), generator=g).to(dev)
pipe = ShardedPipeline(m, depth=2)
outs = [pipe.submit(ids, lens) for _ in range(2)]   # the process's first library calls: side streams
outs = [o.wait() for o in outs]
ref = m.inference(ids, lens)
assert all(torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]) for o in outs)
side = torch.cuda.Stream()
with torch.cuda.stream(side):
    mel, audio = m.inference(ids, lens)
torch.cuda.current_stream().wait_stream(side)
assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1])
print("ok")
"""


def test_first_call_from_a_side_stream(gpu):
    """The process's first T_max read from a non-blocking stream
    (ShardedPipeline's first submit): the per-device mailbox ticket is zeroed
    on the caller's stream, not by a null-stream memset that stream does not
    wait for (which left the first count kernel without its post: "stream
    idle but T_max not posted").  A fresh process, so the mailbox is new."""
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    p = subprocess.run([sys.executable, "-c", _FIRST_CALL_SIDE_STREAM, root], capture_output=True, text=True,
                       timeout=180)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-2000:]
