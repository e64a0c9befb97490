"""Utterance-sharded inference across GPUs (one process per GPU, torch.distributed).

The reference has no distributed code.  Sharding a
global batch by utterance is exact with ONE coupling: the mel decoder is
unmasked over frames and the length regulator pads every utterance to the
batch maximum (tts_model.py:165-176, 211-228), so each utterance's mel depends
on the GLOBAL frame count T.  The ranks therefore agree on T with one
all-reduce(MAX) of one int32 pair before the decoder; everything else is
independent.  Collectives (RCCL over xGMI with the "nccl" backend; gloo in the
CPU tests):
  broadcast        (optional, src=r) the global phoneme ids / lengths from rank r
  all_reduce(MAX)  2 x int32 (T_local, M)          after the duration predictor
  gather / all_gather  mel [b, T, M] and audio [b, 1, 64T] shards (padded to
                   ceil(B/N)), one collective over rows [mel | audio] per
                   utterance; optionally left in flight (async_gather) so it
                   overlaps the next step
Payloads are KB..MB, so the path is latency-bound; weights are replicated.

A step is two phases around the all-reduce: ``front`` (encoder, durations,
frame counts -> local T_max) and ``back`` (expansion to the global T, decoder,
vocoder).  On the GPU each phase is ONE library call; the oracle-backed
``Stages`` used by the CPU tests compose the same phases from per-stage
functions.

On the GPU the frame count normally never visits the host between the phases
(device-T path): m2_inference_front_dev writes the shard's T_max into a device
word, the RCCL all-reduce(MAX) runs on that word in stream order, and
m2_inference_back_dev launches the back half with grids sized for a frame
capacity learnt from earlier steps (the last global T that exceeded it or fell
under half of it - the same on every rank), its kernels reading T from the word.  The gather is
enqueued right behind it on buffers laid out for that capacity; the host reads
T (posted to host-mapped memory by the back half's first launch) only to shape
the outputs.  A step whose T exceeds the capacity re-runs its back
half and gather for the exact T (every rank sees the same T and capacity).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Optional, Tuple

import ctypes

import torch
import torch.distributed as dist

from . import _lib

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
    mel_width: int = 0                                            # M (for ranks with an empty shard)

    def mel_channels(self) -> int:
        return self.mel_width

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
    per step on the model's packed handle (models/tts_model.py), or their
    device-T forms (m2_inference_front_dev / m2_inference_back_dev).  ``lane``
    picks a handle of its own (ShardedPipeline: one per stream)."""

    def __init__(self, model, lane: int = 0, tcap: Optional[dict] = None):
        self.model = model
        self.lane = lane
        # frame capacity of the device-T path per (global B, S, duration_scale):
        # the last global T that exceeded it or fell under half of it -
        # identical on every rank
        self.tcap = {} if tcap is None else tcap

    def mel_channels(self) -> int:
        return int(self.model._m2_cfg.mel_channels)

    def front(self, ids: Tensor, lens: Optional[Tensor], scale: float) -> Tuple[Any, int]:
        # one handle lookup per step (its weight-identity check walks every
        # parameter, ~25 us of host time): the back half reuses this handle
        hm = self.model._hip(ids.device, self.lane)
        state, t = hm.inference_front(ids, lens, scale)
        return (hm, state), t

    def back(self, state: Any, T: int) -> Tuple[Tensor, Tensor]:
        hm, st = state
        return hm.inference_back(st, T)

    def both(self, ids: Tensor, lens: Optional[Tensor], scale: float) -> Tuple[Tensor, Tensor]:
        """Both phases with no collective between them (world 1): the one-call
        m2_inference (the back half is launched from C right after the T_max
        read, no Python between the phases)."""
        return self.model._hip(ids.device, self.lane).inference(ids, lens, scale)

    def dev_handle(self, device: torch.device, T_cap: int):
        """The HipModel of the device-T path at capacity T_cap, or None."""
        hm = self.model._hip(device, self.lane)
        return hm if hm.dev_supported(T_cap) else None


def hip_stages(model) -> HipStages:
    return HipStages(model)


def _stages_device(stages) -> Optional[torch.device]:
    """The device the stages compute on (the model's parameters for
    HipStages; None for host stages such as the oracle-backed Stages).  It is
    the same on every rank, unlike the placement of a rank's input tensors."""
    model = getattr(stages, "model", None)
    if model is None:
        return None
    for p in model.parameters():
        return p.device
    return None


def _collective_device(ref: Optional[Tensor], group) -> torch.device:
    """nccl (RCCL) moves device tensors only; gloo host tensors."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return ref.device if (ref is not None and ref.is_cuda) else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_inputs(phoneme_ids: Optional[Tensor], phoneme_lengths: Optional[Tensor], src: int = 0,
                     group=None, device: Optional[torch.device] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """Rank ``src`` holds the global batch (e.g. the CLI's text); every rank
    returns it.  One broadcast of the header (B, S, lengths present) and one of
    the payload [B, S + 1] int64 (ids and lengths as one row per utterance;
    RCCL over xGMI with the "nccl" backend, 51 KB for configs[3])."""
    me = dist.get_rank(group)
    ref = phoneme_ids if me == src else None
    cdev = _collective_device(ref, group)
    g_src = dist.get_global_rank(group, src) if group is not None else src
    hdr = torch.zeros(3, dtype=torch.int64, device=cdev)
    if me == src:
        if phoneme_ids is None or phoneme_ids.dim() != 2:
            raise ValueError("broadcast_inputs: the source rank needs phoneme_ids [B, S]")
        hdr[0], hdr[1] = phoneme_ids.shape
        hdr[2] = int(phoneme_lengths is not None)
    dist.broadcast(hdr, src=g_src, group=group)
    B, S, has_len = (int(v) for v in hdr.tolist())
    if me == src:
        rows = torch.empty(B, S + 1, dtype=torch.int64, device=cdev)
        rows[:, :S] = phoneme_ids.to(cdev, torch.int64)
        rows[:, S] = phoneme_lengths.to(cdev, torch.int64) if has_len else 0
    else:
        rows = torch.empty(B, S + 1, dtype=torch.int64, device=cdev)
    if B * (S + 1):
        dist.broadcast(rows, src=g_src, group=group)
    out_dev = device if device is not None else (phoneme_ids.device if phoneme_ids is not None else cdev)
    rows = rows.to(out_dev)
    return rows[:, :S].contiguous(), (rows[:, S].contiguous() if has_len else None)


def _gather_shards(local: Tensor, batch: int, world: int, group, dst: Optional[int] = None,
                   async_op: bool = False):
    """Gather per-rank utterance shards of unequal sizes -> [batch, ...]:
    all_gather (every rank gets the batch) or, with ``dst``, gather to that
    rank only (the others get None).  A rank with an empty shard joins with
    padding rows.  With ``async_op`` the collective is left in flight (RCCL
    runs it on its own stream, after the work already queued on the current
    one) and a callable that waits and assembles the result is returned."""
    per = -(-batch // world)
    if local.shape[0] == per:
        pad = local.contiguous()
    else:
        pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    me = dist.get_rank(group)
    parts = None
    if dst is None:
        parts = [torch.empty_like(pad) for _ in range(world)]
        work = dist.all_gather(parts, pad, group=group, async_op=async_op)
    else:
        parts = [torch.empty_like(pad) for _ in range(world)] if me == dst else None
        work = dist.gather(pad, parts, dst=dist.get_global_rank(group, dst) if group is not None else dst,
                           group=group, async_op=async_op)
    n = [shard_bounds(batch, world, r)[1] - shard_bounds(batch, world, r)[0] for r in range(world)]

    def finish():
        if async_op and work is not None:
            work.wait()
        if parts is None:
            return None
        if all(k == per for k in n):
            return torch.stack(parts).flatten(0, 1) if world > 1 else parts[0]
        return torch.cat([parts[r][: n[r]] for r in range(world)], dim=0)

    return finish if async_op else finish()


class PendingGather:
    """The (mel, audio) of a sharded step whose gather is still in flight
    (``sharded_inference(..., async_gather=True)``): ``wait()`` returns them
    (None on ranks that are not the destination)."""

    def __init__(self, finish: Callable, mel_shape, audio_shape, audio_dtype):
        self._finish, self._ms, self._as, self._ad = finish, mel_shape, audio_shape, audio_dtype
        self._out = None
        self._assemble = None  # device-T path: waits and returns (mel, audio) itself

    def wait(self):
        if self._assemble is not None:
            self._out = self._assemble()
            self._assemble = None
        if self._finish is not None:
            g = self._finish()
            self._finish = None
            if g is None:
                self._out = (None, None)
            else:
                Mw = 1
                for v in self._ms[1:]:
                    Mw *= v
                self._out = (g[:, :Mw].reshape(self._ms).contiguous(),
                             g[:, Mw:].reshape(self._as).to(self._ad).contiguous())
        return self._out


def _learn_cap(caps: dict, key, T: int) -> None:
    cap = caps.get(key, 0)
    if T > cap or 2 * T < cap:
        caps[key] = T  # exact: launch configurations chosen from the capacity are T's own


def _sharded_dev(stages, hm, ids, lens, scale, B, lo, hi, world, group, cap, key, gather, gather_to, async_gather):
    """One step of the device-T path (module docstring) on HipModel hm; None
    when T outgrew the capacity (the caller re-runs the step on the host path)."""
    dev = ids.device
    M = stages.mel_channels()
    b = hi - lo
    nccl = world > 1 and dist.get_backend(group) == "nccl"
    tw = torch.empty(1, dtype=torch.int32, device=dev)
    state = hm.inference_front_dev(ids[lo:hi], lens[lo:hi] if lens is not None else None, scale, tw) if b else None
    if not b:
        tw.zero_()
    if world > 1:
        if nccl:  # RCCL on the device word, in stream order: no host read
            dist.all_reduce(tw, op=dist.ReduceOp.MAX, group=group)
        else:  # gloo (tests): staged through the host
            t = tw.cpu()
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            tw.copy_(t)
    rows = -(-B // world) if (gather and world > 1) else b
    moff = (rows * cap * M + 63) // 64 * 64
    buf = torch.empty(moff + rows * 64 * cap, dtype=torch.float32, device=dev)
    if b:
        hm.inference_back_dev(state, cap, tw, buf[: b * cap * M], buf[moff: moff + b * 64 * cap])
    parts, work = None, None
    if gather and world > 1:
        me = dist.get_rank(group)
        dst = None if gather_to is None else (dist.get_global_rank(group, gather_to) if group is not None
                                              else gather_to)
        if gather_to is None or me == gather_to:
            parts = [torch.empty_like(buf) for _ in range(world)]
        if gather_to is None:
            work = dist.all_gather(parts, buf, group=group, async_op=async_gather)
        else:
            work = dist.gather(buf, parts, dst=dst, group=group, async_op=async_gather)
    # T as the back half's first launch posted it (the back half keeps running);
    # a rank with an empty shard reads the word
    T = hm.frames_wait() if b else max(1, int(tw.item()))
    _learn_cap(stages.tcap, key, T)
    if T > cap:
        if async_gather and work is not None:
            work.wait()
        return None

    def view(flat, n):
        return flat[: n * T * M].view(n, T, M), flat[moff: moff + n * 64 * T].view(n, 1, 64 * T)

    if not gather or world == 1:
        mel, audio = view(buf, b)
        if not gather:
            return mel, audio, (lo, hi)
        if async_gather:
            out = PendingGather(None, None, None, None)
            out._out = (mel, audio)
            return out
        return mel, audio

    counts = [shard_bounds(B, world, r)[1] - shard_bounds(B, world, r)[0] for r in range(world)]

    def finish():
        if async_gather and work is not None:
            work.wait()
        if parts is None:
            return None, None
        vs = [view(parts[r], counts[r]) for r in range(world) if counts[r]]
        return torch.cat([v[0] for v in vs]), torch.cat([v[1] for v in vs])

    if async_gather:
        out = PendingGather(None, None, None, None)
        out._assemble = finish
        return out
    return finish()


def sharded_inference(stages, phoneme_ids: Optional[Tensor], phoneme_lengths: Optional[Tensor],
                      duration_scale: float = 1.0, group=None, gather: bool = True,
                      gather_to: Optional[int] = None, src: Optional[int] = None,
                      async_gather: bool = False, one_call_world1: bool = True, device_T: bool = True):
    """M2TTSModel.inference (tts_model.py:402-438) over a global batch sharded by
    utterance.

    Inputs: with ``src=r`` only rank r needs ``phoneme_ids`` / lengths (the
    others may pass None): it broadcasts them (``broadcast_inputs``).
    Without ``src`` every rank passes the same global tensors (e.g. generated
    from one seed).  Rank r computes utterances shard_bounds(B, N, r); a rank
    whose shard is empty (B < N) still joins every collective.

    Returns (mel, audio) for the global batch when ``gather`` (on every rank;
    with ``gather_to=r`` on rank r only, None elsewhere), else this rank's
    shard and its bounds.  ``async_gather`` (with ``gather``) leaves the
    gather in flight and returns a PendingGather, so the next step's work
    overlaps it; call ``.wait()`` for the tensors.  At world 1 the two phases
    run as one library call (``one_call_world1``; False keeps the two-phase
    form the ranks of a multi-GPU job run, e.g. to time one rank's share).
    ``device_T`` (stages with ``front_dev``, CUDA inputs): the frame count
    stays on the device between the phases once a capacity is known (module
    docstring); the first step of a (B, S) shape runs the host path."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    sdev = _stages_device(stages)
    if src is not None and world > 1:
        phoneme_ids, phoneme_lengths = broadcast_inputs(phoneme_ids, phoneme_lengths, src, group, device=sdev)
    elif sdev is not None and phoneme_ids.device != sdev:
        phoneme_ids = phoneme_ids.to(sdev)
        phoneme_lengths = phoneme_lengths.to(sdev) if phoneme_lengths is not None else None
    B = phoneme_ids.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    ids = phoneme_ids[lo:hi]
    lens = phoneme_lengths[lo:hi] if phoneme_lengths is not None else None
    key = (B, phoneme_ids.shape[1], float(duration_scale))
    # decided from values every rank shares (the stages' type and device, the
    # world size): the device-T and host paths issue different collectives
    use_dev = device_T and hasattr(stages, "dev_handle") and sdev is not None and sdev.type == "cuda" and \
        not (one_call_world1 and world == 1 and hasattr(stages, "both"))
    if use_dev:
        cap = stages.tcap.get(key, 0)
        hm = stages.dev_handle(phoneme_ids.device, cap) if cap > 0 else None
        if hm is not None:
            with torch.no_grad():
                out = _sharded_dev(stages, hm, phoneme_ids, phoneme_lengths, duration_scale, B, lo, hi, world,
                                   group, cap, key, gather, gather_to, async_gather)
            if out is not None:
                return out
    if one_call_world1 and world == 1 and hi > lo and hasattr(stages, "both"):
        with torch.no_grad():
            mel, audio = stages.both(ids, lens, duration_scale)
        if async_gather and gather:
            out = PendingGather(None, None, None, None)
            out._out = (mel, audio)
            return out
        return (mel, audio) if gather else (mel, audio, (lo, hi))
    with torch.no_grad():
        state, t_local = stages.front(ids, lens, duration_scale) if hi > lo else (None, 0)
        M = stages.mel_channels()
        if world > 1:
            # one all_reduce(MAX) of (T_local, M): the batch-global frame count,
            # and the mel width for ranks whose shard is empty
            t = torch.tensor([t_local, M], dtype=torch.int32, device=_collective_device(phoneme_ids, group))
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            t_local, M = (int(v) for v in t.tolist())
        T = max(1, t_local)  # all-empty batch -> one zero frame (tts_model.py:158-160)
        if hasattr(stages, "tcap"):
            _learn_cap(stages.tcap, key, T)
        if hi > lo:
            mel, audio = stages.back(state, T)
        else:
            dev = phoneme_ids.device
            mel = torch.zeros(0, T, M, dtype=torch.float32, device=dev)
            audio = torch.zeros(0, 1, 64 * T, dtype=torch.float32, device=dev)
    if not gather or world == 1:
        if async_gather and gather:
            out = PendingGather(None, None, None, None)
            out._out = (mel, audio)
            return out
        return (mel, audio) if gather else (mel, audio, (lo, hi))
    # one collective for both outputs: each utterance's mel and audio as one row
    b, Mw = mel.shape[0], T * M
    both = torch.cat([mel.reshape(b, Mw), audio.reshape(b, 64 * T).to(mel.dtype)], dim=1)
    fin = _gather_shards(both, B, world, group, gather_to, async_op=async_gather)
    pend = PendingGather(fin if async_gather else (lambda: fin), (B, T, M), (B, 1, 64 * T), audio.dtype)
    return pend if async_gather else pend.wait()


class _LaneResult:
    """A pipelined step's (mel, audio): ``wait()`` joins the lane's stream into
    the caller's and returns them (None on non-destination ranks)."""

    def __init__(self, out, stream, caller):
        self._out, self._stream, self._caller = out, stream, caller
        self._res = None

    def wait(self):
        if self._out is not None and self._stream is None:  # host stages: no stream to join
            self._res = self._out.wait() if isinstance(self._out, PendingGather) else self._out
            self._out = None
        if self._out is not None:
            # the gather's wait and the assembly of rank 0's outputs run on the
            # lane's stream, where the gathered buffers were allocated
            with torch.cuda.stream(self._stream):
                r = self._out.wait() if isinstance(self._out, PendingGather) else self._out
            self._caller.wait_stream(self._stream)
            for t in r:
                if t is not None:
                    t.record_stream(self._caller)
            self._res, self._out = r, None
        return self._res


class _SplitStep:
    """A step of ShardedPipeline's split-stream schedule: ``wait()`` waits
    for the step's back half (on the host with ``host_wait``, else by an
    event wait on the caller's stream), reads T (posted by the back half's
    first launch) and returns (mel, audio) (None on non-destination ranks).  A step whose T outgrew the capacity is re-run
    on the host-T path (every rank sees the same T and capacity)."""

    __slots__ = ("pipe", "lane", "caller", "bind", "b", "key", "cap", "work", "ids", "lens", "scale", "moff", "B",
                 "world", "buf", "parts", "_res")

    def __init__(self, pipe, lane, caller, bind, b, key, cap, work, ids, lens, scale, moff, B, world, buf, parts):
        self.pipe, self.lane, self.caller, self.bind, self.b, self.key, self.cap = pipe, lane, caller, bind, b, key, cap
        self.work, self.ids, self.lens, self.scale, self.moff, self.B = work, ids, lens, scale, moff, B
        self.world, self.buf, self.parts = world, buf, parts
        self._res = None

    def wait(self):
        if self._res is not None:
            return self._res
        p = self.pipe
        if p._pending[self.lane] is self:
            p._pending[self.lane] = None
        caller = self.caller
        if p.host_wait:  # the host waits; the caller's (possibly shared) hardware queue gets no barrier
            p._done[self.lane].synchronize()
        else:
            caller.wait_event(p._done[self.lane])
        st = p.lanes[self.lane]
        if self.b:
            T = ctypes.c_int32(0)
            _lib.check(p._wait_fn(self.bind.handle, p._bs_h, ctypes.byref(T)), "m2_frames_wait")
            T = int(T.value)
        else:
            T = max(1, int(self.bind.tw.item()))
        _learn_cap(st.tcap, self.key, T)
        if T > self.cap:  # rare: re-run the step for the exact T on the host-T path
            if self.work is not None:
                self.work.wait()
            with torch.no_grad():
                out = sharded_inference(st, self.ids, self.lens, self.scale, group=p.group,
                                        gather_to=p.gather_to, one_call_world1=False, device_T=False)
            self._res = out
            return out
        if self.work is not None:
            self.work.wait()  # the caller's stream waits for the gather
        M, moff, B, world = p._M, self.moff, self.B, self.world

        def view(flat, n):
            return flat[: n * T * M].view(n, T, M), flat[moff: moff + n * 64 * T].view(n, 1, 64 * T)

        if world == 1:
            self._res = view(self.buf, self.b)
        elif self.parts is None:
            self._res = (None, None)
        else:
            counts = [shard_bounds(B, world, r)[1] - shard_bounds(B, world, r)[0] for r in range(world)]
            for t in self.parts:
                t.record_stream(caller)
            vs = [view(self.parts[r], counts[r]) for r in range(world) if counts[r]]
            self._res = (torch.cat([v[0] for v in vs]), torch.cat([v[1] for v in vs]))
        return self._res


class _LaneBind:
    """A lane's handle and buffers for one (B, S, scale, capacity): the
    library is called with these raw pointers and the pipeline's raw stream
    handles (no per-step wrapper work)."""

    def __init__(self, hm, b, S, cap, dev):
        self.hm, self.handle = hm, hm.handle
        self.front = hm._scratch("_front", hm._size("m2_front_bytes", max(b, 1), S))
        self.ws = hm._scratch("_ws", hm._size("m2_inference_workspace_bytes", max(b, 1), S, cap))
        self.tw = torch.empty(1, dtype=torch.int32, device=dev)
        self.args = (self.front.data_ptr(), self.front.numel(), self.ws.data_ptr(), self.ws.numel(),
                     self.tw.data_ptr())


class ShardedPipeline:
    """Sharded inference with ``depth`` global batches in flight per rank.

    Two streams per pipeline, shared by all lanes: every step's front half
    (encoder, durations, the shard's T_max into a device word) and the ranks'
    all_reduce(MAX) of that word go on the FRONT stream, its back half
    (expansion, decoder, vocoder reading T from the word) and the gather of
    mel / audio on the BACK stream, behind an event of its front half.  So
    step i + 1's front half (a few small launches: 50 workgroups at configs[3]'s
    8-utterance share) runs beside step i's back half, and the back halves run
    back to back.  Each lane has its own model handle (a handle's front
    buffer, workspace and device words are reused by its next step, whose
    front half waits for this step's back-half event).  With several ranks
    the gathers use a communicator of their own, so step i + 1's T exchange
    is not queued behind step i's gather.  ``submit`` returns at once; the
    device-T path needs a capacity, so the first step of a (B, S) shape runs
    as one sharded_inference on the back stream.  Every rank submits the
    same sequence, so the collectives of each communicator are issued in the
    same order everywhere.  Results are identical to sharded_inference.
    A step calls the library with raw pointers on the two streams' raw
    handles (the host enqueue is ~0.1 ms per step at configs[3]'s share,
    under its GPU time); the weights are re-validated every step (the
    model's handle cache), as ``inference()`` does.

    ``host_wait`` (default): a step's ``wait()`` blocks the host until the
    step's back half is done instead of enqueueing a wait on the caller's
    stream.  HIP maps streams onto GPU_MAX_HW_QUEUES (4) in-order hardware
    queues; when the caller's stream shares one with a pipeline stream, a
    wait enqueued there holds the pipeline's next launches behind it (B=64:
    0.673 -> 0.641 ms per step in such a layout, profiles/r06/r06p_q4.txt).

    ``model`` may also be a host ``Stages`` (the oracle-backed stages of the
    CPU tests): the lanes then share it and have no stream; the lane
    rotation and the in-flight gathers are the same."""

    def __init__(self, model, depth: int = 2, group=None, gather_to: Optional[int] = 0, host_wait: bool = True):
        self.group, self.gather_to = group, gather_to
        self.host_wait = host_wait
        self._next = 0
        self.host = isinstance(model, Stages)
        if self.host:
            self.lanes = [model for _ in range(depth)]
            return
        tcap: dict = {}
        # lanes 1..depth: lane 0 is the model's default handle, which
        # model.inference() / forward() use on the caller's stream
        self.lanes = [HipStages(model, lane=i + 1, tcap=tcap) for i in range(depth)]
        # Two normal-priority streams (measured and dropped: the back stream at
        # high priority, -2 % at B=8 with raw calls but up to 3x slower in other
        # stream layouts and +35 % at B=64, profiles/r06/r06j_prio.txt,
        # r06l_prio_ab.txt).  HIP maps streams onto GPU_MAX_HW_QUEUES (4)
        # in-order hardware queues, so either stream can share a queue with
        # the caller's; in the layouts measured that cost up to 1.5x at B=8
        # (profiles/r06/r06n_q*.txt)
        self.front_stream, self.back_stream = torch.cuda.Stream(), torch.cuda.Stream()
        self._fs_h, self._bs_h = self.front_stream.cuda_stream, self.back_stream.cuda_stream
        self._pending = [None] * depth
        self._front_ev = [torch.cuda.Event() for _ in range(depth)]
        self._done = [torch.cuda.Event() for _ in range(depth)]
        self._used = [False] * depth  # a lane's done event has been recorded
        self._binds = [{} for _ in range(depth)]
        self._M = self.lanes[0].mel_channels()
        lib = _lib.load()
        self._front_fn, self._back_fn, self._wait_fn = (lib.m2_inference_front_dev, lib.m2_inference_back_dev,
                                                        lib.m2_frames_wait)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.ggroup = None
        self._nccl = False
        if self.world > 1:  # collective: every rank constructs the pipeline
            ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
            self.ggroup = dist.new_group(ranks=ranks)
            self._nccl = dist.get_backend(group) == "nccl"

    def submit(self, phoneme_ids: Optional[Tensor], phoneme_lengths: Optional[Tensor],
               duration_scale: float = 1.0):
        h = self._next % len(self.lanes)
        self._next += 1
        st = self.lanes[h]
        if self.host:
            out = sharded_inference(st, phoneme_ids, phoneme_lengths, duration_scale, group=self.group,
                                    gather_to=self.gather_to, async_gather=True, one_call_world1=False)
            return _LaneResult(out, None, None)
        if self._pending[h] is not None:  # the lane's buffers are reused below
            self._pending[h].wait()
        dev = phoneme_ids.device
        caller = torch.cuda.current_stream(dev)
        B, S = phoneme_ids.shape
        key = (B, S, float(duration_scale))
        cap = st.tcap.get(key, 0)
        # the lane's handle, re-validated against the model's weights every step
        hm = st.dev_handle(dev, cap) if cap > 0 else None
        fs, bs = self.front_stream, self.back_stream
        # int64 contiguous inputs, converted on the caller's stream before the
        # front stream waits for it
        ids = phoneme_ids if phoneme_ids.dtype == torch.int64 and phoneme_ids.is_contiguous() else \
            phoneme_ids.to(torch.int64).contiguous()
        lens = phoneme_lengths
        if lens is not None and (lens.dtype != torch.int64 or not lens.is_contiguous()):
            lens = lens.to(torch.int64).contiguous()
        fs.wait_stream(caller)  # the inputs were produced on the caller's stream
        if self._used[h]:
            fs.wait_event(self._done[h])
        if hm is None:  # no capacity yet: one whole step on the back stream
            for t in (ids, lens):
                if t is not None:
                    t.record_stream(bs)
            bs.wait_stream(fs)
            with torch.cuda.stream(bs):
                out = sharded_inference(st, ids, lens, duration_scale, group=self.group,
                                        gather_to=self.gather_to, async_gather=True, one_call_world1=False)
            self._done[h].record(bs)
            self._used[h] = True
            return _LaneResult(out, bs, caller)
        world, M = self.world, self._M
        lo, hi = shard_bounds(B, world, self.rank)
        b = hi - lo
        bind = self._binds[h].get((key, cap))
        if bind is None or bind.hm is not hm:
            if bind is not None:  # the weights changed: a new handle
                self._binds[h].clear()
            bind = self._binds[h][(key, cap)] = _LaneBind(hm, b, S, cap, dev)
        fr, fn, wsp, wsn, twp = bind.args
        for t in (ids, lens):
            if t is not None:
                t.record_stream(fs)
        with torch.no_grad():
            if b:
                _lib.check(self._front_fn(bind.handle, ids.data_ptr() + lo * S * 8,
                                          None if lens is None else lens.data_ptr() + lo * 8, b, S,
                                          float(duration_scale), fr, fn, wsp, wsn, twp, self._fs_h),
                           "m2_inference_front_dev")
            if world > 1 or not b:
                with torch.cuda.stream(fs):
                    if not b:
                        bind.tw.zero_()
                    if world > 1:
                        if self._nccl:
                            dist.all_reduce(bind.tw, op=dist.ReduceOp.MAX, group=self.group)
                        else:  # gloo: staged through the host
                            t = bind.tw.cpu()
                            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                            bind.tw.copy_(t)
            self._front_ev[h].record(fs)
            bs.wait_event(self._front_ev[h])
            rows = -(-B // world) if world > 1 else b
            moff = (rows * cap * M + 63) // 64 * 64
            buf = torch.empty(moff + rows * 64 * cap, dtype=torch.float32, device=dev)
            buf.record_stream(bs)
            if b:
                bp = buf.data_ptr()
                _lib.check(self._back_fn(bind.handle, b, S, cap, twp, fr, fn, bp, bp + moff * 4, wsp, wsn,
                                         self._bs_h), "m2_inference_back_dev")
            parts, work = None, None
            if world > 1:
                with torch.cuda.stream(bs):
                    me = dist.get_rank(self.ggroup)
                    if self.gather_to is None or me == self.gather_to:
                        parts = [torch.empty_like(buf) for _ in range(world)]
                    if self.gather_to is None:
                        work = dist.all_gather(parts, buf, group=self.ggroup, async_op=True)
                    else:
                        dst = dist.get_global_rank(self.ggroup, self.gather_to)
                        work = dist.gather(buf, parts, dst=dst, group=self.ggroup, async_op=True)
            self._done[h].record(bs)
            self._used[h] = True
        step = _SplitStep(self, h, caller, bind, b, key, cap, work, phoneme_ids, phoneme_lengths, duration_scale,
                          moff, B, world, buf, parts)
        self._pending[h] = step
        return step
