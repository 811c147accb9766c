"""Data-parallel training over RCCL (xGMI) — one process per GPU.

The reference has no distributed code.  Every loss term is
per-sample (no BatchNorm, no cross-sample term in m_iwae / elbo,
losses.py:16-24,47-62), so the step shards by contiguous batch slices and the
only exchange is ONE all-reduce of the flat fp32 gradient per step
(SURVEY.md §8(e)):

  * m_iwae is a SUM over the batch  -> all-reduce SUM reproduces the
    single-process full-batch gradient exactly (up to summation order);
  * elbo is a MEAN over K*B         -> all-reduce SUM / world (equal shards).

Parameters are broadcast from rank 0 once at setup.  Backend "nccl" is RCCL on
ROCm; "gloo" is used by the CPU-side tests of the process-group logic.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard(batch, rank=None, world_size=None):
    """Contiguous slice [rank*b, (rank+1)*b) of every tensor of a (possibly
    multimodal) batch; b = B // world (the remainder goes to the last rank)."""
    if rank is None:
        rank, world_size = world()
    if world_size == 1:
        return batch

    def cut(t):
        B = t.shape[0]
        b = B // world_size
        lo = rank * b
        hi = B if rank == world_size - 1 else lo + b
        return t[lo:hi]

    if isinstance(batch, list):
        return [tuple(cut(t) for t in m) for m in batch]
    return tuple(cut(t) for t in batch)


def broadcast_parameters(module, src=0):
    """Make every rank start from rank `src`'s parameters (and buffers)."""
    if world()[1] == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


class GradAllReduce:
    """Hook for FusedAdamW(grad_hook=...): one all-reduce of the flat gradient."""

    def __init__(self, reduction="sum", group=None):
        if reduction not in ("sum", "mean"):
            raise ValueError(reduction)
        self.reduction = reduction
        self.group = group

    def __call__(self, flat_grad):
        ws = world()[1]
        if ws == 1:
            return
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)
        if self.reduction == "mean":
            flat_grad.div_(ws)


def allreduce_grads(params, reduction="sum"):
    """For optimizers other than FusedAdamW: flatten p.grad, all-reduce once,
    write back."""
    ws = world()[1]
    if ws == 1:
        return
    ps = [p for p in params if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if reduction == "mean":
        flat.div_(ws)
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n
