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
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import _hip
from _hip import call, ptr

BUCKET_BYTES = 64 << 20


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _avg_op():
    return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM


def allreduce_gradients(model, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Average param.grad over all ranks (call after loss.backward())."""
    if not is_distributed():
        return
    gb = model._hip_engine._grads
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


def broadcast_buffers(model, src: int = 0) -> None:
    """torch DDP broadcast_buffers=True semantics for the BN running statistics."""
    if not is_distributed():
        return
    for b in model.buffers():
        dist.broadcast(b, src=src)


def broadcast_parameters(model, src: int = 0) -> None:
    """Start every rank from rank 0's weights (torch DDP constructor semantics)."""
    if not is_distributed():
        return
    for p in model.parameters():
        dist.broadcast(p.data, src=src)
