"""GPU: utterance-sharded inference through the HIP phases (m2amd.parallel
HipStages = m2_inference_front / m2_inference_back), the streamed vocoder
(m2_vocoder_chunk / m2_vocoder_set_chunking) and run-time vocoder path
selection, against the reference fixtures, the oracle and the unsharded /
unchunked HIP path."""
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


def test_hip_stages_sharded_world1_matches_fixture(gpu):
    """sharded_inference(hip_stages(model)) at world = 1 (no process group):
    fp_s2_B64_S100 (configs[3]'s global batch) against the reference
    fingerprints, the oracle and M2TTSModel.inference bit for bit."""
    from m2amd.parallel import hip_stages, sharded_inference
    from test_gpu_parity import _check_fingerprint
    fp = golden("fp_s2_B64_S100")
    m = build_model("s2", gpu)
    ids, lens = torch.from_numpy(fp["ids"]), torch.from_numpy(fp["lengths"])
    mel, audio = sharded_inference(hip_stages(m), ids.to(gpu), lens.to(gpu))
    _check_fingerprint(fp, mel, audio)
    mel1, audio1 = m.inference(ids.to(gpu), lens.to(gpu))
    assert torch.equal(mel, mel1) and torch.equal(audio, audio1)
    rows = [0, 33, 63]
    ref_mel, ref_audio = orc.inference(golden_state("s2"), stage_config("s2"), ids[rows], lens[rows], as_written=False)
    assert maxabs(mel[rows], ref_mel) <= MEL_MAXABS_TOL
    assert rms(audio[rows], ref_audio) <= AUDIO_RMS_TOL


def test_sharded_pipeline_matches_fixture(gpu):
    """ShardedPipeline (front halves on one stream, back halves on another,
    two lanes) over configs[3]'s global batch fp_s2_B64_S100 and over its
    8-utterance slices (the per-GPU share's shape): the global batch against
    the reference fingerprints, every step bit-equal to M2TTSModel.inference
    of the same rows, with several steps in flight."""
    from m2amd.parallel import ShardedPipeline
    from test_gpu_parity import _check_fingerprint
    fp = golden("fp_s2_B64_S100")
    m = build_model("s2", gpu)
    ids, lens = torch.from_numpy(fp["ids"]).to(gpu), torch.from_numpy(fp["lengths"]).to(gpu)
    pipe = ShardedPipeline(m, depth=2)
    steps = [(slice(0, 64), pipe.submit(ids, lens))]
    for i in range(8):
        rows = slice(8 * i, 8 * i + 8)
        steps.append((rows, pipe.submit(ids[rows], lens[rows])))
    steps.append((slice(0, 64), pipe.submit(ids, lens)))
    for rows, r in steps:
        mel, audio = r.wait()
        ref = m.inference(ids[rows], lens[rows])
        assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1]), rows
        if rows == slice(0, 64):
            _check_fingerprint(fp, mel, audio)


def test_sharded_pipeline_no_lengths_scaled(gpu):
    """ShardedPipeline with phoneme_lengths=None (no padding mask), int32
    ids and a duration scale: each step bit-equal to M2TTSModel.inference
    with the same arguments (tts_model.py:402-438)."""
    from m2amd.parallel import ShardedPipeline
    m = build_model("s1", gpu)
    g = torch.Generator().manual_seed(13)
    ids = torch.randint(0, 42, (6, 40), generator=g).to(gpu)
    pipe = ShardedPipeline(m, depth=2)
    for scale in (1.0, 1.3, 1.3, 0.7):
        ref = m.inference(ids, None, duration_scale=scale)
        r1 = pipe.submit(ids.to(torch.int32), None, scale)
        r2 = pipe.submit(ids, None, scale)
        for r in (r1, r2):
            mel, audio = r.wait()
            assert torch.equal(mel, ref[0]) and torch.equal(audio, ref[1]), scale


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, outfile):
    """Two ranks sharing cuda:0 (gloo moves the tiny all-reduce through the host
    and all-gathers the device shards); each rank runs the HIP phases on its
    shard.  Ragged lengths make the shards' local frame counts differ, so the
    global-T coupling (tts_model.py:165-176 + the unmasked decoder) is live."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m2amd.parallel import hip_stages, sharded_inference
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        m = build_model("s1", dev)
        g = torch.Generator().manual_seed(11)
        ids = torch.randint(0, 42, (5, 30), generator=g)
        lens = torch.tensor([30, 12, 25, 7, 30])
        mel, audio = sharded_inference(hip_stages(m), ids.to(dev), lens.to(dev))
        mel_s, audio_s, (lo, hi) = sharded_inference(hip_stages(m), ids.to(dev), lens.to(dev), duration_scale=1.3,
                                                     gather=False)
        if rank == 0:
            np.savez(outfile, mel=mel.cpu().numpy(), audio=audio.cpu().numpy(), mel_s=mel_s.cpu().numpy(),
                     audio_s=audio_s.cpu().numpy(), lo=lo, hi=hi, ids=ids.numpy(), lens=lens.numpy())
    finally:
        dist.destroy_process_group()


def test_hip_stages_two_ranks_gloo_on_one_gpu(gpu, tmp_path):
    import torch.multiprocessing as mp
    outfile = str(tmp_path / "shard.npz")
    mp.spawn(_sharded_worker, args=(2, _free_port(), outfile), nprocs=2, join=True)
    z = np.load(outfile)
    m = build_model("s1", gpu)
    ids, lens = torch.from_numpy(z["ids"]).to(gpu), torch.from_numpy(z["lens"]).to(gpu)
    mel, audio = m.inference(ids, lens)
    assert z["mel"].shape == tuple(mel.shape)
    assert torch.equal(torch.from_numpy(z["mel"]), mel.cpu())
    assert torch.equal(torch.from_numpy(z["audio"]), audio.cpu())
    lo, hi = int(z["lo"]), int(z["hi"])
    mel_s, audio_s = m.inference(ids, lens, duration_scale=1.3)
    assert torch.equal(torch.from_numpy(z["mel_s"]), mel_s[lo:hi].cpu())
    assert torch.equal(torch.from_numpy(z["audio_s"]), audio_s[lo:hi].cpu())


@pytest.mark.parametrize("stage", ["s1", "s2"])
@pytest.mark.parametrize("T,chunk", [(1, 1), (7, 3), (100, 64), (257, 256), (300, 1), (1000, 256)])
def test_streamed_vocoder_bitwise(gpu, stage, T, chunk):
    """Chunked / streamed audio equals the whole-utterance vocoder bit for bit
    (the 3-frame halo covers the receptive field; every kernel computes a
    sample with the same operations wherever its tile falls)."""
    m = build_model(stage, gpu)
    M = stage_config(stage).mel_channels
    mel = torch.randn(2, M, T, generator=torch.Generator().manual_seed(T * 7 + chunk)).to(gpu)
    full = m.vocoder(mel)
    parts = list(m.vocoder.stream(mel, chunk))
    assert len(parts) == -(-T // chunk)
    assert torch.equal(torch.cat(parts, dim=2), full)
    m.set_vocoder_chunking(chunk)
    assert torch.equal(m.vocoder(mel), full)
    hm = m._hip(gpu)
    assert torch.equal(hm.vocoder(mel.transpose(1, 2).contiguous(), layout_btm=True), full)
    m.set_vocoder_chunking(0)
    assert torch.equal(m.vocoder(mel), full)


def test_streamed_vocoder_longform_stage2(gpu):
    """T = 2600 (configs[4]'s utterance length), 256-frame chunks: max-abs
    against the unchunked call <= 1e-6 (observed: 0), and against the oracle
    within the waveform bound."""
    m = build_model("s2", gpu)
    mel = torch.randn(2, 80, 2600, generator=torch.Generator().manual_seed(26))
    full = m.vocoder(mel.to(gpu))
    chunked = torch.cat(list(m.vocoder.stream(mel.to(gpu), 256)), dim=2)
    assert maxabs(chunked, full) <= 1e-6
    assert torch.equal(chunked, full)
    ref = orc.vocoder(golden_state("s2"), mel)
    assert rms(chunked, ref) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage,T", [("s1", 1_100_000), ("s2", 540_000)])
def test_vocoder_u2_past_2gb(gpu, stage, T):
    """One utterance whose U2 hand-off (16 T rows of 128 / 256 B) passes 2^31
    bytes: the pipelined tails' LDS-DMA loaders address U2 through 32-bit
    buffer offsets, so their descriptors start at each strip (not at the
    utterance).  The whole call equals the same vocoder chunked by 65,536
    frames (whose U2 is small) bit for bit."""
    m = build_model(stage, gpu)
    M = stage_config(stage).mel_channels
    assert 16 * T * (128 if stage == "s1" else 256) > 2**31
    mel = torch.randn(1, M, T, generator=torch.Generator().manual_seed(31)).to(gpu)
    full = m.vocoder(mel)
    m.set_vocoder_chunking(65536)
    try:
        chunked = m.vocoder(mel)
    finally:
        m.set_vocoder_chunking(0)
    assert torch.isfinite(full).all()
    assert torch.equal(chunked, full)


def test_streamed_vocoder_standalone_module(gpu):
    """A SimpleVocoder outside an M2TTSModel streams through the per-op kernels
    over the same widened windows: equal to its own forward up to the per-op
    kernels' tiling noise, and to the reference fixture."""
    from models.tts_model import SimpleVocoder
    sd = golden_state("s1")
    voc = SimpleVocoder(64, 128)
    voc.load_state_dict({k[len("vocoder."):]: v for k, v in sd.items() if k.startswith("vocoder.")})
    voc = voc.to(gpu).eval()
    mel = torch.randn(2, 64, 50, generator=torch.Generator().manual_seed(3)).to(gpu)
    full = voc(mel)
    chunked = torch.cat(list(voc.stream(mel, 16)), dim=2)
    assert maxabs(chunked, full) <= 1e-6


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_inference_with_chunking(gpu, stage):
    """inference() with the streamed vocoder: identical to the unchunked run."""
    g = golden(f"{stage}_small")
    m = build_model(stage, gpu)
    ids, lens = torch.from_numpy(g["ids"]).to(gpu), torch.from_numpy(g["lengths"]).to(gpu)
    mel0, audio0 = m.inference(ids, lens)
    m.set_vocoder_chunking(16)
    mel1, audio1 = m.inference(ids, lens)
    assert torch.equal(mel0, mel1) and torch.equal(audio0, audio1)
    assert rms(audio1, g["audio"]) <= AUDIO_RMS_TOL


@pytest.mark.parametrize("stage", ["s1", "s2"])
def test_vocoder_select_paths(gpu, stage):
    """m2_vocoder_select switches between exact-f32 and split-f16 at run time;
    both within the waveform bound of the oracle."""
    m = build_model(stage, gpu)
    mel = torch.randn(2, stage_config(stage).mel_channels, 61, generator=torch.Generator().manual_seed(9))
    ref = orc.vocoder(golden_state(stage), mel)
    hm = m._hip(gpu)
    assert hm.vocoder_path() == 2
    split = m.vocoder(mel.to(gpu))
    m.set_vocoder_precision("f32")
    assert hm.vocoder_path() == 1
    f32 = m.vocoder(mel.to(gpu))
    m.set_vocoder_precision("split")
    assert hm.vocoder_path() == 2
    assert torch.equal(m.vocoder(mel.to(gpu)), split)
    for a in (split, f32):
        assert rms(a, ref) <= AUDIO_RMS_TOL and maxabs(a, ref) <= 1e-4
