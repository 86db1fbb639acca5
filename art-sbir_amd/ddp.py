"""Data-parallel triplet training over RCCL (xGMI) — one process per GPU.

The reference trains on one GPU (sbatch_train.sh:4 "-G 1"); SURVEY §8(e) row 1:
each rank takes its own minibatch of triplets, runs the three local-BN branch
forwards/backwards (no SyncBN in the reference, so BN statistics stay
per-replica), then gradients are averaged with an all-reduce and every rank
applies the same Adam step.

Because libartsbir_hip accumulates every parameter gradient into ONE
contiguous f32 buffer (engine.GradBuffer), the exchange is a handful of large
all-reduces over that buffer (bucketed so RCCL can pipeline them over the 7
xGMI links) — no per-parameter flatten/unflatten copies.  BatchNorm running
statistics follow torch DDP's broadcast_buffers=True: rank 0's buffers are
broadcast to the other ranks.

OverlappedReducer starts those all-reduces DURING the backward (SURVEY §8e
"overlapped with backward", torch DDP's bucket hooks): the engine reports, block
by block in backward order, which ranges of the buffer hold final gradients
(the attention pool first, the stem last — the buffer is in parameter order, so
the ready part grows from the end); once bucket_bytes of them are pending they
are all-reduced on a communication stream that waits only for the main and
weight-gradient streams' work enqueued so far, so RCCL traffic over xGMI runs
under the remaining layers' backward instead of after it.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

import _hip
from _hip import call, ptr

BUCKET_BYTES = 64 << 20


def init_distributed() -> None:
    """one process per GPU (torch.distributed.run): RCCL ("nccl") on the GPU of
    LOCAL_RANK; ARTSBIR_DIST_BACKEND=gloo for several ranks sharing one device
    (tests) or CPU-only hosts"""
    if dist.is_initialized():
        return
    backend = os.environ.get("ARTSBIR_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local % torch.cuda.device_count() if torch.cuda.is_available() else 0  # one index for both uses
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    else:
        dist.init_process_group(backend)


def is_distributed() -> bool:
    """a process group of more than one rank (ARTSBIR_DDP_WORLD1=1: also a
    one-rank group, so that a one-GPU box runs every collective through RCCL —
    tests/test_ddp_gpu.py::test_rccl_world1_collectives)"""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or os.environ.get("ARTSBIR_DDP_WORLD1") == "1"


def _avg_op():
    return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM


def allreduce_gradients(model, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Average param.grad over all ranks (call after loss.backward())."""
    if not is_distributed():
        return
    gb = getattr(getattr(model, "_hip_engine", None), "_grads", None)
    if gb is None:
        # a model whose gradients autograd accumulates (vit.VisionTransformer):
        # plain param.grad tensors, all-reduced in coalesced buckets
        return allreduce_tensors([p.grad for p in model.parameters() if p.grad is not None], bucket_bytes)
    flat = gb.flat
    world = dist.get_world_size()
    op = _avg_op()
    per = max(1, bucket_bytes // flat.element_size())
    works = [dist.all_reduce(flat[i:i + per], op=op, async_op=True) for i in range(0, flat.numel(), per)]
    for w in works:
        w.wait()
    if op != dist.ReduceOp.AVG:
        # gloo (CPU tests): sum then scale in place; flat is f32
        flat.mul_(1.0 / world)


def allreduce_tensors(tensors, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Average a list of tensors over all ranks in place: consecutive tensors of
    one dtype / device are flattened into buckets of about bucket_bytes, each
    bucket is one all-reduce (torch DDP's coalesced buckets), then copied back."""
    if not is_distributed() or not tensors:
        return
    op = _avg_op()
    world = dist.get_world_size()
    buckets, cur, nbytes = [], [], 0
    for t in tensors:
        if cur and (t.dtype != cur[0].dtype or t.device != cur[0].device or nbytes >= bucket_bytes):
            buckets.append(cur)
            cur, nbytes = [], 0
        cur.append(t)
        nbytes += t.numel() * t.element_size()
    if cur:
        buckets.append(cur)
    pending = []
    for b in buckets:
        flat = torch.cat([t.reshape(-1) for t in b])
        pending.append((b, flat, dist.all_reduce(flat, op=op, async_op=True)))
    for b, flat, w in pending:
        w.wait()
        if op != dist.ReduceOp.AVG:
            flat.mul_(1.0 / world)
        o = 0
        for t in b:
            t.copy_(flat[o:o + t.numel()].view_as(t))
            o += t.numel()


class OverlappedReducer:
    """Bucketed gradient all-reduce launched while the backward still runs.

    Protocol (engine.HipEncoder.backward drives it through ``grad_hook``):
      begin(flat)            a backward over this flat gradient buffer starts
      ready(ranges, streams) elements [lo, hi) of each range are final once the
                             work enqueued so far on ``streams`` has run
      end()                  the backward has been fully enqueued: flush the rest
    ``finish()`` (called by the training loop after loss.backward()) waits for
    every all-reduce and, on backends without AVG, scales by 1/world.
    Ranges of one backward must not overlap; every element of the buffer must
    be reported exactly once before end() — what is not reported is all-reduced
    by end() all the same (so a caller that reports nothing gets the plain
    post-backward all-reduce)."""

    def __init__(self, bucket_bytes: int = BUCKET_BYTES, model=None):
        self.bucket_bytes = bucket_bytes
        self.model = model
        self.flat = None
        self.works = []
        self.pending = []
        self.done = []
        self._comm = None
        self.launches = []  # (lo, hi) per all-reduce, in launch order (tests)
        self.launched_before_end = 0

    def _stream(self, flat):
        if flat.is_cuda and self._comm is None:
            self._comm = torch.cuda.Stream(device=flat.device)
        return self._comm

    def begin(self, flat):
        if self.works:
            raise RuntimeError("OverlappedReducer.begin: previous step not finished")
        self.flat, self.pending, self.done, self.launches = flat, [], [], []

    def ready(self, ranges, streams=()):
        if self.flat is None or not is_distributed():
            return
        for lo, hi in ranges:
            if hi > lo:
                self.pending.append((int(lo), int(hi)))
        if sum(h - l for l, h in self.pending) * self.flat.element_size() >= self.bucket_bytes:
            self._launch(streams)

    def end(self, streams=()):
        if self.flat is None or not is_distributed():
            return
        self.launched_before_end = len(self.launches)
        covered = sorted(self.done + self.pending)
        lo = 0
        for a, b in covered:  # whatever was not reported goes now
            if a > lo:
                self.pending.append((lo, a))
            lo = max(lo, b)
        if lo < self.flat.numel():
            self.pending.append((lo, self.flat.numel()))
        self._launch(streams)

    def _launch(self, streams):
        if not self.pending:
            return
        op = _avg_op()
        per = max(1, self.bucket_bytes // self.flat.element_size())
        merged = []
        for lo, hi in sorted(self.pending):  # coalesce adjacent ranges (a module's parameters are adjacent)
            if merged and lo <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], hi))
            else:
                merged.append((lo, hi))
        comm = self._stream(self.flat)
        if comm is not None:
            for st in streams:
                comm.wait_event(st.record_event())
        ctx = torch.cuda.stream(comm) if comm is not None else _nullctx()
        with ctx:
            for lo, hi in reversed(merged):  # the buffer's end became ready first
                for a in range(lo, hi, per):
                    b = min(hi, a + per)
                    self.works.append(dist.all_reduce(self.flat[a:b], op=op, async_op=True))
                    self.launches.append((a, b))
        self.done += self.pending
        self.pending = []

    def finish(self):
        if not is_distributed():
            return
        if self.flat is None:  # no hooked backward ran (e.g. separate per-branch backwards): plain all-reduce
            if self.model is not None:
                allreduce_gradients(self.model, self.bucket_bytes)
            return
        if self.pending or not self.works:
            self.end()
        for w in self.works:
            w.wait()
        if _avg_op() != dist.ReduceOp.AVG:
            self.flat.mul_(1.0 / dist.get_world_size())
        self.works = []
        self.flat = None


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def attach_overlapped_reducer(model, bucket_bytes: int = BUCKET_BYTES):
    """Install an OverlappedReducer as the model engine's gradient hook (no-op
    when not distributed); the training loop calls its finish() after
    loss.backward() instead of allreduce_gradients()."""
    r = OverlappedReducer(bucket_bytes, model)
    eng = getattr(model, "_hip_engine", None)
    if is_distributed() and eng is not None:
        eng.grad_hook = r
    return r


def broadcast_buffers(model, src: int = 0) -> None:
    """torch DDP broadcast_buffers=True semantics for the BN running statistics."""
    if not is_distributed():
        return
    for b in model.buffers():
        dist.broadcast(b, src=src)
    eng = getattr(model, "_hip_engine", None)
    if eng is not None and hasattr(eng, "bn_stats_changed"):
        eng.bn_stats_changed()  # running statistics replaced: refold the eval weights


def broadcast_parameters(model, src: int = 0) -> None:
    """Start every rank from rank 0's weights (torch DDP constructor semantics)."""
    if not is_distributed():
        return
    for p in model.parameters():
        dist.broadcast(p.data, src=src)
