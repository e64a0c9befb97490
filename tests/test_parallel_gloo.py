"""Utterance sharding (m2amd.parallel) on 2 CPU ranks over gloo, with the CPU
oracle bound as the per-shard stages: the sharded result must equal the
unsharded reference forward, including the batch-global frame padding that
the unmasked decoder makes observable."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import m2tts_oracle as orc
from conftest import golden, golden_state


def oracle_stages(sd, cfg):
    from m2amd.parallel import Stages

    def frame_totals(dur, scale):
        d = (dur * scale).trunc()
        return torch.where(d > 0, d, torch.zeros_like(d)).sum(1).to(torch.int32)

    return Stages(encode=lambda ids, lens: orc.text_encoder(sd, cfg, ids, lens)[0],
                  durations=lambda enc: orc.duration_predictor(sd, enc),
                  frame_totals=frame_totals,
                  regulate=lambda enc, dur, T, scale: orc.length_regulator(enc, dur * scale if scale != 1.0 else dur, T),
                  decode=lambda x: orc.mel_decoder(sd, cfg, x),
                  vocode=lambda mel: orc.vocoder(sd, mel.transpose(1, 2)),
                  mel_width=cfg.mel_channels)


def _worker(rank, world, port, outfile):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m2amd.parallel import sharded_inference
        torch.set_num_threads(2)
        sd = golden_state("s1")
        st = oracle_stages(sd, orc.STAGE1)
        g = golden("s1_target_free")  # lengths [24, 17]
        ids, lens = torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"])
        # uneven global batch of 5 with different lengths -> different per-shard T
        ids5 = torch.cat([ids, ids[:1], ids.flip(1)[:2]])
        lens5 = torch.tensor([24, 17, 24, 9, 3])
        out = {}
        for tag, (i, l, scale) in {"b2": (ids, lens, 1.0), "b5": (ids5, lens5, 1.0), "b5s": (ids5, lens5, 1.3)}.items():
            mel, audio = sharded_inference(st, i, l, duration_scale=scale)
            out[tag] = (mel, audio)
        # gather to one rank only (the serving layout: rank 1 collects, rank 0 gets None)
        mel_r, audio_r = sharded_inference(st, ids5, lens5, gather_to=1)
        assert (mel_r is None) == (rank != 1) and (audio_r is None) == (rank != 1)
        # inputs on rank 0 only (broadcast), gather left in flight while another step runs
        pend = sharded_inference(st, ids5 if rank == 0 else None, lens5 if rank == 0 else None, src=0,
                                 gather_to=0, async_gather=True)
        mel_n, _ = sharded_inference(st, ids5 if rank == 0 else None, lens5 if rank == 0 else None, src=0)
        mel_b, audio_b = pend.wait()
        assert (mel_b is None) == (rank != 0)
        assert torch.equal(mel_n, out["b5"][0])
        # B = 1 < world: rank 1's shard is empty and it still joins every collective
        one = {}
        one["all"] = sharded_inference(st, ids[:1], lens[:1])
        one["to1"] = sharded_inference(st, ids[:1], lens[:1], gather_to=1)
        one["src"] = sharded_inference(st, ids[:1] if rank == 0 else None, lens[:1] if rank == 0 else None, src=0)
        assert (one["to1"][0] is None) == (rank != 1)
        import numpy as np
        if rank == 1:
            np.savez(outfile + ".root1.npz", mel=mel_r.numpy(), audio=audio_r.numpy(),
                     one_mel=one["to1"][0].numpy(), one_audio=one["to1"][1].numpy(),
                     src_mel=one["src"][0].numpy())
        if rank == 0:
            np.savez(outfile + ".bcast.npz", mel=mel_b.numpy(), audio=audio_b.numpy(),
                     one_mel=one["all"][0].numpy(), one_audio=one["all"][1].numpy())
        dist.barrier()
        if rank == 0:
            np.savez(outfile, **{f"{k}_{j}": v[j].numpy() for k, v in out.items() for j in range(2)})
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_inference_matches_unsharded_two_ranks(tmp_path):
    import numpy as np
    outfile = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(2, _free_port(), outfile), nprocs=2, join=True)
    z = np.load(outfile)
    res = {k: (z[f"{k}_0"], z[f"{k}_1"]) for k in ("b2", "b5", "b5s")}
    r1 = np.load(outfile + ".root1.npz")
    assert np.array_equal(r1["mel"], res["b5"][0]) and np.array_equal(r1["audio"], res["b5"][1])
    bc = np.load(outfile + ".bcast.npz")
    assert np.array_equal(bc["mel"], res["b5"][0]) and np.array_equal(bc["audio"], res["b5"][1])
    assert np.array_equal(bc["one_mel"], r1["one_mel"]) and np.array_equal(bc["one_audio"], r1["one_audio"])
    assert np.array_equal(bc["one_mel"], r1["src_mel"])
    sd = golden_state("s1")
    g = golden("s1_target_free")
    ids, lens = torch.from_numpy(g["ids"]), torch.from_numpy(g["lengths"])
    ids5 = torch.cat([ids, ids[:1], ids.flip(1)[:2]])
    lens5 = torch.tensor([24, 17, 24, 9, 3])
    for tag, (i, l, scale) in {"b2": (ids, lens, 1.0), "b5": (ids5, lens5, 1.0), "b5s": (ids5, lens5, 1.3)}.items():
        mel, audio = orc.inference(sd, orc.STAGE1, i, l, duration_scale=scale, as_written=False)
        assert res[tag][0].shape == tuple(mel.shape), tag
        assert float(abs(res[tag][0] - mel.numpy()).max()) <= 1e-5, tag
        assert float(abs(res[tag][1] - audio.numpy()).max()) <= 1e-5, tag
    mel1, audio1 = orc.inference(sd, orc.STAGE1, ids[:1], lens[:1], as_written=False)
    assert bc["one_mel"].shape == tuple(mel1.shape)
    assert float(abs(bc["one_mel"] - mel1.numpy()).max()) <= 1e-5
    assert float(abs(bc["one_audio"] - audio1.numpy()).max()) <= 1e-5


def test_shard_bounds_cover_batch():
    from m2amd.parallel import shard_bounds
    for B in range(0, 20):
        for N in range(1, 9):
            spans = [shard_bounds(B, N, r) for r in range(N)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
