"""Data-parallel training over RCCL (xGMI) — one process per GPU.

The reference has no distributed code.  Every loss term is
per-sample (no BatchNorm, no cross-sample term in m_iwae / elbo,
losses.py:16-24,47-62), so the step shards by contiguous batch slices and the
only exchange is ONE all-reduce of the flat fp32 gradient per step
(SURVEY.md §8(e)):

  * m_iwae is a SUM over the batch  -> all-reduce SUM reproduces the
    single-process full-batch gradient exactly (up to summation order);
  * elbo is a MEAN over K*B         -> each rank scales its gradient by its
    shard's share of the batch (b_r / B; 1/world for equal shards), then SUM.

The one exception is the contrastive objective (losses.negInfoNCE over
ContraPhotSpec projections): its B x B logits couple every pair of samples, so
it has a real exchange step.  Each rank all-gathers the [b_r, proj_dim]
projections (a few KB), evaluates the full-batch loss scaled by 1/world, and
the gather's backward all-reduces the projection gradient and keeps its own
rows; the SUM gradient all-reduce then reproduces the full-batch gradient.

Parameters are broadcast from rank 0 once at setup.  Backend "nccl" is RCCL on
ROCm; "gloo" is used by the CPU-side tests of the process-group logic.
"""
from __future__ import annotations

import ctypes as C
import os

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def env_world():
    """(rank, world) from a launcher's environment (torchrun: RANK / WORLD_SIZE),
    whether or not the process group exists yet."""
    if dist.is_available() and dist.is_initialized():
        return world()
    ws = int(os.environ.get("WORLD_SIZE", "1") or 1)
    return (int(os.environ.get("RANK", "0") or 0), ws) if ws > 1 else (0, 1)


def init_from_env():
    """Bring up the process group the launcher describes, if it is not up yet:
    the cannon scripts never call init_process_group (training_util.py:17-53 has
    no distributed code), so `torchrun --nproc-per-node N script.py` with the
    script unchanged reaches here from training_step.  Backend "nccl" (RCCL over
    xGMI) when the ranks drive GPUs, "gloo" otherwise; VAESNE_DP_BACKEND overrides
    it (gloo lets several ranks share one GPU, which RCCL refuses).  Rank r drives
    GPU LOCAL_RANK mod the visible device count.  Returns (rank, world)."""
    if not dist.is_available() or dist.is_initialized():
        return world()
    rank, ws = env_world()
    if ws <= 1:
        return 0, 1
    backend = dp_backend()
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device_index())
    dist.init_process_group(backend)
    return world()


def local_device_index():
    """The GPU this rank drives: LOCAL_RANK mod the visible device count."""
    n = max(1, torch.cuda.device_count())
    return int(os.environ.get("LOCAL_RANK", "0") or 0) % n


def dp_backend():
    """VAESNE_DP_BACKEND if set, else "nccl" (RCCL) with GPUs and "gloo" without."""
    b = os.environ.get("VAESNE_DP_BACKEND", "").strip().lower()
    if b:
        if b not in ("nccl", "gloo"):
            raise ValueError(f"VAESNE_DP_BACKEND={b!r}: expected nccl or gloo")
        return b
    return "nccl" if torch.cuda.is_available() else "gloo"


def split_bounds(B, rank=None, world_size=None):
    """[lo, hi) of rank's contiguous batch slice: sizes differ by at most one
    (torch.tensor_split's rule: the first B % world ranks take one extra row)."""
    if rank is None:
        rank, world_size = world()
    b, r = divmod(int(B), int(world_size))
    lo = rank * b + min(rank, r)
    return lo, lo + b + (1 if rank < r else 0)


def shard(batch, rank=None, world_size=None):
    """This rank's contiguous slice (split_bounds) of every tensor of a (possibly
    multimodal) batch.  A rank can get an empty slice when B < world."""
    if rank is None:
        rank, world_size = world()
    if world_size == 1:
        return batch

    def cut(t):
        lo, hi = split_bounds(t.shape[0], rank, world_size)
        return t[lo:hi]

    if isinstance(batch, list):
        return [tuple(cut(t) for t in m) for m in batch]
    return tuple(cut(t) for t in batch)


def shard_fraction(B, rank=None, world_size=None):
    """b_r / B for the split `shard` makes (the weight of this rank's
    mean-objective gradient in the global mean)."""
    lo, hi = split_bounds(B, rank, world_size)
    return (hi - lo) / B


def sync_parameters_once(module, src=0):
    """broadcast_parameters the first time a module is trained data-parallel
    (ranks seeded alike already agree; this makes it a guarantee)."""
    if world()[1] > 1 and not getattr(module, "_vaesne_dp_synced", False):
        broadcast_parameters(module, src)
        module._vaesne_dp_synced = True


def broadcast_parameters(module, src=0):
    """Make every rank start from rank `src`'s parameters (and buffers)."""
    if world()[1] == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


class GradAllReduce:
    """Hook for FusedAdamW(grad_hook=...): one all-reduce of the flat gradient.
    For reduction="mean", `weight` is this rank's shard fraction b_r / B
    (None = 1/world, equal shards); training_step sets it per batch."""

    def __init__(self, reduction="sum", group=None, weight=None):
        if reduction not in ("sum", "mean"):
            raise ValueError(reduction)
        self.reduction = reduction
        self.group = group
        self.weight = weight

    def __call__(self, flat_grad):
        ws = world()[1]
        if ws == 1:
            return
        if self.reduction == "mean":
            flat_grad.mul_(self.weight if self.weight is not None else 1.0 / ws)
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)


def agree_grad_pattern(params):
    """Make every rank hold a gradient for the same parameters before the gradient
    all-reduce: one MAX all-reduce of a has-gradient mask; a parameter some rank has
    a gradient for and this rank does not (an empty batch slice, or a branch the
    loss does not reach here) gets a zero gradient.  Keeps the all-reduce sizes and
    FusedAdamW's per-parameter step counts identical on every rank."""
    ws = world()[1]
    params = list(params)
    if ws == 1 or not params:
        return
    dev = params[0].device
    mask = torch.tensor([p.grad is not None for p in params], dtype=torch.int32, device=dev)
    dist.all_reduce(mask, op=dist.ReduceOp.MAX)
    for p, m in zip(params, mask.tolist()):
        if m and p.grad is None:
            p.grad = torch.zeros_like(p)


def allreduce_grads(params, reduction="sum", weight=None):
    """For optimizers other than FusedAdamW: flatten p.grad, all-reduce once,
    write back.  `weight` as in GradAllReduce."""
    ws = world()[1]
    if ws == 1:
        return
    ps = [p for p in params if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    if reduction == "mean":
        flat.mul_(weight if weight is not None else 1.0 / ws)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n


class FlatExchange:
    """training_step's data-parallel exchange: ONE all-reduce (SUM) per batch of a
    persistent buffer [every gradient, in `params` order | loss | 2 guard words].

    * The gradients are gathered into the buffer by one pack launch (zeros for a
      parameter this rank has no gradient for), weighted by the rank's batch share for
      a mean objective, and after the all-reduce every `.grad` that should exist IS a
      view of the buffer: no per-parameter copies back.
    * The loss (times the same weight) and the guard words ride in the same
      collective: the reduced words are every rank's verdict, and the update kernels
      read them as their skip flag (a float word is non-zero iff its bits are), so all
      ranks skip or apply together without a host round trip.
    * Which parameters get a gradient (the MAX over ranks of "has a gradient", so an
      empty shard or an unreached branch still updates like the full batch) is agreed
      once per key (the step's loss function and batch size: identical on every rank,
      so every rank decides alike whether to agree again) and cached."""

    def __init__(self, params, device, buf=None):
        self.params = list(params)
        self.device = torch.device(device)
        self.ns = [p.numel() for p in self.params]
        self.n = sum(self.ns)
        # buf: storage to exchange in (FusedAdamW's own gradient buffer, so its flat
        # gradient IS the reduced one); at least n + 3 floats
        if buf is not None and (buf.numel() < self.n + 3 or buf.dtype != torch.float32
                                or buf.device != self.device):
            raise ValueError("FlatExchange: buffer too small or of the wrong dtype / device")
        self.buf = buf[:self.n + 3] if buf is not None else \
            torch.zeros(self.n + 3, dtype=torch.float32, device=self.device)
        self.views, o = [], 0
        self.offs = []
        for p, k in zip(self.params, self.ns):
            self.views.append(self.buf[o:o + k].view_as(p))
            self.offs.append(o)
            o += k
        self.patterns = {}

    def grads_flat(self):
        return self.buf[:self.n]

    def skip_ptr(self):
        return self.buf[self.n + 1:].data_ptr()

    # added to the loss-flag word by a rank whose gradients go beyond the agreed pattern:
    # the word rides in the batch's one collective, so every rank skips the update and
    # raises together (a rank raising alone would leave the others in the next collective)
    MISMATCH = 1 << 20

    def agree(self, key):
        local = tuple(p.grad is not None for p in self.params)
        mask = self.patterns.get(key)
        self.mismatch = False
        if mask is None:
            t = torch.tensor(local, dtype=torch.int32, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            mask = self.patterns[key] = tuple(bool(v) for v in t.tolist())
        elif any(a and not b for a, b in zip(local, mask)):
            self.mismatch = True
        return mask

    def run(self, val, scale, mean, flag, mask):
        """Gather, all-reduce, re-bind the gradients; returns the reduced
        [val * scale, post_flag, loss_flag] (a device view, no sync).  The gradient is
        multiplied by |scale| (the rank's batch share) for a mean objective."""
        n = self.n
        _lib = None
        if self.buf.is_cuda:
            from . import _lib      # the HIP library (the host path runs without it)
            srcs = [p.grad if p.grad is not None and p.grad.is_contiguous() else None
                    for p in self.params]
            _lib.lib.pack(_lib.ptr_array(srcs), (C.c_int64 * len(srcs))(*self.offs),
                          (C.c_int64 * len(srcs))(*self.ns), len(srcs), self.buf.data_ptr(), 0,
                          _lib.stream())
            for p, v, s in zip(self.params, self.views, srcs):
                if s is None and p.grad is not None:
                    v.copy_(p.grad)
        else:
            for p, v in zip(self.params, self.views):
                if p.grad is None:
                    v.zero_()
                elif p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
        weight = abs(scale)
        if mean and weight != 1.0:
            self.buf[:n].mul_(weight)
        if getattr(self, "mismatch", False) and flag is not None:
            flag[1:].add_(self.MISMATCH)     # sticky: every later update is skipped too
        if _lib is not None:
            v = val.detach()
            if v.dtype != torch.float32 or not v.is_contiguous():
                v = v.float().contiguous()
            _lib.lib.loss_stat(v.data_ptr(), float(scale), None if flag is None else flag.data_ptr(),
                               self.buf.data_ptr() + 4 * n, _lib.stream())
        else:
            torch.mul(val.detach().reshape(1).float(), scale, out=self.buf[n:n + 1])
            if flag is None:
                self.buf[n + 1:].zero_()
            else:
                self.buf[n + 1:].copy_(flag)
            if getattr(self, "mismatch", False) and flag is None:
                self.buf[n + 2] += self.MISMATCH
        dist.all_reduce(self.buf, op=dist.ReduceOp.SUM)
        for p, v, m in zip(self.params, self.views, mask):
            p.grad = v if m else None
        return self.buf[n:]


class _GatherRows(torch.autograd.Function):
    """all_gather along dim 0 in rank order (ragged shards allowed).  Backward:
    every rank holds the gradient of its own copy of the full-batch loss, so the
    full [B, ...] gradient is all-reduced (SUM) and this rank keeps its rows."""

    @staticmethod
    def forward(ctx, z, group):
        ws = dist.get_world_size(group)
        rank = dist.get_rank(group)
        n = torch.tensor([z.shape[0]], dtype=torch.int64, device=z.device)
        sizes = [torch.zeros_like(n) for _ in range(ws)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(t.item()) for t in sizes]
        zp = z.new_zeros((max(sizes),) + tuple(z.shape[1:]))
        zp[:z.shape[0]] = z
        outs = [torch.empty_like(zp) for _ in range(ws)]
        dist.all_gather(outs, zp, group=group)
        ctx.lo, ctx.n, ctx.group = sum(sizes[:rank]), z.shape[0], group
        return torch.cat([o[:k] for o, k in zip(outs, sizes)])

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
        return g[ctx.lo:ctx.lo + ctx.n], None


def global_rows(*zs, group=None):
    """For a batch-coupled objective: the full-batch rows of every per-sample
    tensor in `zs` (this rank's shard gathered with the others'), plus the
    factor 1/world the full-batch loss is scaled by on each rank, so that the
    SUM gradient all-reduce reproduces the single-process gradient.  Identity
    (factor 1) without a process group."""
    ws = world()[1]
    if ws == 1:
        return zs + (1.0,)
    return tuple(_GatherRows.apply(z, group) for z in zs) + (1.0 / ws,)
