"""Utterance-sharded inference across GPUs (one process per GPU, torch.distributed).

The reference has no distributed code.  Sharding a
global batch by utterance is exact with ONE coupling: the mel decoder is
unmasked over frames and the length regulator pads every utterance to the
batch maximum (tts_model.py:165-176, 211-228), so each utterance's mel depends
on the GLOBAL frame count T.  The ranks therefore agree on T with one
all-reduce(MAX) of a single int32 before the decoder; everything else is
independent.  Collectives (RCCL over xGMI with the "nccl" backend; gloo in the
CPU tests):
  all_reduce(MAX)  1 x int32                       after the duration predictor
  all_gather       mel [b, T, M] and audio [b, 1, 64T] shards (padded to ceil(B/N)),
                   one collective over rows [mel | audio] per utterance
Payloads are KB..MB, so the path is latency-bound; weights are replicated.

A step is two phases around the all-reduce: ``front`` (encoder, durations,
frame counts -> local T_max) and ``back`` (expansion to the global T, decoder,
vocoder).  On the GPU each phase is ONE library call (m2_inference_front /
m2_inference_back); the oracle-backed ``Stages`` used by the CPU tests compose
the same phases from per-stage functions.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Optional, Tuple

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def shard_bounds(batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split: rank r gets [lo, hi) (first B % N ranks get one more)."""
    base, rem = divmod(batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@dataclass
class Stages:
    """Per-shard stage functions composed into the two phases.  Tests bind the
    CPU oracle here to check the sharding logic on gloo."""
    encode: Callable[[Tensor, Optional[Tensor]], Tensor]          # ids, lengths -> enc [b,S,H]
    durations: Callable[[Tensor], Tensor]                         # enc -> dur [b,S]
    frame_totals: Callable[[Tensor, float], Tensor]               # dur, scale -> T_b [b] (int)
    regulate: Callable[[Tensor, Tensor, int, float], Tensor]      # enc, dur, T, scale -> [b,T,H]
    decode: Callable[[Tensor], Tensor]                            # [b,T,H] -> mel [b,T,M]
    vocode: Callable[[Tensor], Tensor]                            # mel [b,T,M] -> audio [b,1,64T]

    def front(self, ids: Tensor, lens: Optional[Tensor], scale: float) -> Tuple[Any, int]:
        enc = self.encode(ids, lens)
        dur = self.durations(enc)
        return (enc, dur, scale), int(self.frame_totals(dur, scale).max().item())

    def back(self, state: Any, T: int) -> Tuple[Tensor, Tensor]:
        enc, dur, scale = state
        mel = self.decode(self.regulate(enc, dur, T, scale))
        return mel, self.vocode(mel)


class HipStages:
    """The MI355X phases: one m2_inference_front and one m2_inference_back call
    per step on the model's packed handle (models/tts_model.py)."""

    def __init__(self, model):
        self.model = model

    def front(self, ids: Tensor, lens: Optional[Tensor], scale: float) -> Tuple[Any, int]:
        # one handle lookup per step (its weight-identity check walks every
        # parameter, ~25 us of host time): the back half reuses this handle
        hm = self.model._hip(ids.device)
        state, t = hm.inference_front(ids, lens, scale)
        return (hm, state), t

    def back(self, state: Any, T: int) -> Tuple[Tensor, Tensor]:
        hm, st = state
        return hm.inference_back(st, T)


def hip_stages(model) -> HipStages:
    return HipStages(model)


def _gather_shards(local: Tensor, batch: int, world: int, group, dst: Optional[int] = None) -> Optional[Tensor]:
    """Gather per-rank utterance shards of unequal sizes -> [batch, ...]:
    all_gather (every rank gets the batch) or, with ``dst``, gather to that
    rank only (the others return None)."""
    per = -(-batch // world)
    if local.shape[0] == per:
        pad = local.contiguous()
    else:
        pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    me = dist.get_rank(group)
    if dst is None:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
    else:
        parts = [torch.empty_like(pad) for _ in range(world)] if me == dst else None
        dist.gather(pad, parts, dst=dist.get_global_rank(group, dst) if group is not None else dst, group=group)
        if me != dst:
            return None
    n = [shard_bounds(batch, world, r)[1] - shard_bounds(batch, world, r)[0] for r in range(world)]
    if all(k == per for k in n):
        return torch.stack(parts).flatten(0, 1) if world > 1 else parts[0]
    return torch.cat([parts[r][: n[r]] for r in range(world)], dim=0)


def _collective_device(ids: Tensor, group) -> torch.device:
    """nccl (RCCL) reduces device tensors only; gloo host tensors."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device()) if not ids.is_cuda else ids.device
    return torch.device("cpu")


def sharded_inference(stages, phoneme_ids: Tensor, phoneme_lengths: Optional[Tensor],
                      duration_scale: float = 1.0, group=None, gather: bool = True,
                      gather_to: Optional[int] = None):
    """M2TTSModel.inference (tts_model.py:402-438) over a global batch sharded by
    utterance.  Every rank passes the same global ``phoneme_ids``/lengths
    (or the same seed-generated tensors); rank r computes utterances
    shard_bounds(B, N, r).  Returns (mel, audio) for the global batch when
    ``gather`` (on every rank; with ``gather_to=r`` on rank r only, None
    elsewhere), else this rank's shard and its bounds."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    B = phoneme_ids.shape[0]
    if gather and world > 1 and B < world:  # same decision on every rank, before any collective
        raise ValueError("sharded_inference with gather needs at least one utterance per rank (B >= world)")
    lo, hi = shard_bounds(B, world, rank)
    ids = phoneme_ids[lo:hi]
    lens = phoneme_lengths[lo:hi] if phoneme_lengths is not None else None
    with torch.no_grad():
        state, t_local = stages.front(ids, lens, duration_scale) if hi > lo else (None, 0)
        if world > 1:
            t = torch.tensor([t_local], dtype=torch.int32, device=_collective_device(phoneme_ids, group))
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            t_local = int(t.item())
        T = max(1, t_local)  # all-empty batch -> one zero frame (tts_model.py:158-160)
        mel, audio = stages.back(state, T) if hi > lo else (None, None)
    if not gather or world == 1:
        return (mel, audio) if gather else (mel, audio, (lo, hi))
    # one collective for both outputs: each utterance's mel and audio as one row
    b, Mw = mel.shape[0], mel[0].numel()
    both = torch.cat([mel.reshape(b, -1), audio.reshape(b, -1).to(mel.dtype)], dim=1)
    g = _gather_shards(both, B, world, group, gather_to)
    if g is None:
        return None, None
    return (g[:, :Mw].reshape((B,) + tuple(mel.shape[1:])).contiguous(),
            g[:, Mw:].reshape((B,) + tuple(audio.shape[1:])).to(audio.dtype).contiguous())
