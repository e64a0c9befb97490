#!/usr/bin/env python3
"""Two gloo ranks sharing cuda:0 running sharded_inference(gather_to=0) on the
device-T path, with a stack dump of every thread if a step hangs (diagnosis
of the N=2 bench rehearsal)."""
import faulthandler
import os
import socket
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "m2-tts_amd" / "src"))
sys.path.insert(0, str(ROOT))


def worker(rank, world, port, B, S, gather_to, depth):
    import torch.distributed as dist
    faulthandler.dump_traceback_later(40, exit=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from m2amd.parallel import ShardedPipeline, hip_stages, sharded_inference
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = bench.fixture_model(bench.STAGE2, dev)
    g = torch.Generator().manual_seed(2024)
    ids = torch.randint(0, 42, (B, S), generator=g).to(dev)
    lens = torch.full((B,), S, dtype=torch.long, device=dev)
    st = hip_stages(m)
    pipe = ShardedPipeline(m, depth=depth, gather_to=gather_to) if depth > 1 else None
    for i in range(4):
        print(f"rank {rank} step {i} start", flush=True)
        if pipe is None:
            out = sharded_inference(st, ids, lens, gather_to=gather_to, one_call_world1=False)
        else:
            out = pipe.submit(ids, lens).wait()
        torch.cuda.synchronize()
        print(f"rank {rank} step {i} done {None if out[0] is None else tuple(out[0].shape)}", flush=True)
    faulthandler.cancel_dump_traceback_later()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    B, S, gt, depth = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    mp.spawn(worker, args=(2, port, B, S, None if gt == "all" else int(gt), depth), nprocs=2, join=True)
