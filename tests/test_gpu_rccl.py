"""GPU, >= 2 devices: the RCCL ("nccl" backend) branches of m2amd.parallel.

The other sharding tests run gloo (CPU ranks, or two ranks sharing one GPU).
Here each rank owns its own MI355X and the collectives run over RCCL: the
one-word device all_reduce(MAX) of the device-T flow, the host-T flow's
two-word all_reduce, the device-resident gather / all_gather, the input
broadcast from rank 0 and ShardedPipeline with two lanes.  Rank 0's gathered
mel / audio must equal a one-GPU inference() of the global batch bit for bit
(the reference's output for the global batch, tts_model.py:402-438: every
utterance's kernels see the same T and the same operation sequence).
Skipped when fewer than two GPUs are visible (the round-end 1-GPU box)."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import golden_state, stage_config

pytestmark = pytest.mark.gpu


def _two_gpus():
    return torch.cuda.device_count() >= 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build(stage, dev):
    from models.tts_model import M2TTSModel
    m = M2TTSModel(**stage_config(stage).as_dict())
    m.load_state_dict(golden_state(stage))
    return m.to(dev).eval()


def _worker(rank, world, port, outfile):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        from m2amd.parallel import ShardedPipeline, hip_stages, sharded_inference
        m = _build("s2", dev)
        st = hip_stages(m)
        g = torch.Generator().manual_seed(11)
        ids = torch.randint(0, 42, (9, 60), generator=g)
        lens = torch.randint(10, 61, (9,), generator=g)
        outs = {}
        # host-T first step, device-T from the second; all_gather on the last
        for i in range(3):
            mel, audio = sharded_inference(st, ids.to(dev), lens.to(dev), gather_to=0)
            if rank == 0:
                outs[f"mel{i}"], outs[f"audio{i}"] = mel.cpu().numpy(), audio.cpu().numpy()
        mel, audio = sharded_inference(st, ids.to(dev), lens.to(dev))
        outs[f"ag_mel_r{rank}"] = mel.cpu().numpy()
        # inputs on rank 0 only (host tensors), broadcast over RCCL
        for i in range(2):
            mel, audio = sharded_inference(st, ids if rank == 0 else None, lens if rank == 0 else None, src=0,
                                           gather_to=0)
            if rank == 0:
                outs[f"src_mel{i}"], outs[f"src_audio{i}"] = mel.cpu().numpy(), audio.cpu().numpy()
        # two global batches in flight per rank
        pipe = ShardedPipeline(m, depth=2, gather_to=0)
        rs = [pipe.submit(ids.to(dev), lens.to(dev)) for _ in range(3)]
        for i, r in enumerate(rs):
            mel, audio = r.wait()
            if rank == 0:
                outs[f"pipe_mel{i}"], outs[f"pipe_audio{i}"] = mel.cpu().numpy(), audio.cpu().numpy()
        torch.cuda.synchronize(dev)
        if rank == 0:
            np.savez(outfile, ids=ids.numpy(), lens=lens.numpy(), **outs)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not _two_gpus(), reason="needs >= 2 visible GPUs (RCCL between two devices)")
def test_sharded_inference_rccl_two_gpus(gpu, tmp_path):
    import torch.multiprocessing as mp
    outfile = str(tmp_path / "rccl.npz")
    mp.spawn(_worker, args=(2, _free_port(), outfile), nprocs=2, join=True)
    z = np.load(outfile)
    m = _build("s2", gpu)
    ids, lens = torch.from_numpy(z["ids"]).to(gpu), torch.from_numpy(z["lens"]).to(gpu)
    rmel, raudio = (t.cpu().numpy() for t in m.inference(ids, lens))
    keys = [f"mel{i}" for i in range(3)] + ["ag_mel_r0", "ag_mel_r1"] + [f"src_mel{i}" for i in range(2)] + \
        [f"pipe_mel{i}" for i in range(3)]
    for k in keys:
        assert np.array_equal(z[k], rmel), k
    for k in [f"audio{i}" for i in range(3)] + [f"src_audio{i}" for i in range(2)] + [f"pipe_audio{i}" for i in range(3)]:
        assert np.array_equal(z[k], raudio), k
