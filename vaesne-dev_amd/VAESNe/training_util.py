"""One training epoch — reference training_util.py:17-53, unchanged in
behaviour for a single process.

Data parallel.  Under a launcher that describes a world
(`torchrun --nproc-per-node N script.py`: WORLD_SIZE / RANK / LOCAL_RANK), the
first call brings the process group up itself (distributed.init_from_env; the
scripts never do) and broadcasts the parameters from rank 0 once.  Each rank
trains on its contiguous slice of every batch (sizes differ by at most one) and
gradients are all-reduced once per step (VAESNe.distributed): SUM for
sum-over-batch objectives (m_iwae, the multimodal default) and, for mean
objectives (elbo, the single-modality default), each rank's gradient weighted by
its share of the batch before the SUM.  A rank whose slice is empty (B < world)
joins the all-reduce with zero gradients, and every rank holds a gradient for the
same parameters (distributed.agree_grad_pattern), so all ranks apply the same update.  Each rank draws its own noise / dropout streams
(rng.rank_seed).  The returned value is the mean full-batch loss on every rank.

Captured steps (VAESNe._stepgraph): after two eager batches of one signature
(input shapes, loss function, parameters), the forward + backward is captured
once as a hipGraph and replayed for every later batch of that signature; the
optimizer steps eagerly on the gradients as before.  Each batch draws its noise
and dropout masks under the same call ids and a per-batch device counter, so a
replayed batch computes exactly what the eager batch would (VAESNE_STEP_GRAPH=0:
always eager).

Non-finite values (VAESNe.guard): the HIP kernels flag a NaN posterior or a
NaN / Inf loss on the device.  The flag is cleared before each batch's forward
and read, with the loss, at ONE sync placed before `optimizer.step()` (the
reference's `.item()`, training_util.py:46, moves ahead of the update): under data
parallelism the loss and both flag words travel in one all-reduce, so every rank
sees the same verdict and all raise RuntimeError together (a rank-local raise
would leave the others blocked in the next all-reduce).  The update is never
applied for a flagged batch, as the reference stops before its update
(PhotometricVAE.py:160-161).  A non-finite loss also raises (stricter than the
reference, which would train on it)."""
import math

import torch

from . import _defer, _stepgraph, guard, rng
from . import distributed as D
from .losses import elbo
from .optim import FusedAdamW


_SEEDS = {}


def backward_negated(value):
    """`loss = -value; loss.backward()` (training_util.py:42-44) with the gradient seed
    -1 handed to `value` directly: the same gradients bit for bit (NegBackward
    multiplies the seed 1 by -1 exactly), without the fill and negation launches that
    sit between the forward and the backward of every step.  Returns -value
    (detached), negated after the backward was issued."""
    key = (value.device, value.dtype, tuple(value.shape))
    seed = _SEEDS.get(key)
    if seed is None:
        if value.is_cuda and torch.cuda.is_current_stream_capturing():
            loss = -value          # no persistent seed yet: never allocate one in a capture
            loss.backward()
            return loss.detach()
        seed = _SEEDS[key] = torch.full(key[2], -1.0, dtype=value.dtype, device=value.device)
    value.backward(seed)
    return -value.detach()


def safelog10(x):
    tmp = max(1e-10, x)
    return math.log10(tmp)


def training_step(network, optimizer, data_loader, loss_fn=elbo, multimodal=False,
                  release_memory=False, grad_reduction=None):
    network.train()
    total_loss = 0.
    num_batches = 0.
    device = next(network.parameters()).device
    rank, ws = D.init_from_env()
    reduction = grad_reduction or ("sum" if multimodal else "mean")
    fused = isinstance(optimizer, FusedAdamW)
    if ws > 1:
        D.sync_parameters_once(network)
        if fused and optimizer.grad_hook is None:
            optimizer.grad_hook = D.GradAllReduce(reduction)
    params = [p for p in network.parameters() if p.requires_grad]
    # the next batch is collated and copied to the device while this one runs (its copy
    # queued behind this batch's work, from pinned memory): the host's DataLoader work
    # leaves the per-batch idle window.  Not in the host-generator parity mode, where
    # the model's draws and a dataset's share torch's CPU generator in the reference's
    # order.
    ahead = device.type == "cuda" and rng.capturable()
    batches = iter(data_loader)
    nxt = _fetch(batches, device, multimodal, ahead)
    while nxt is not None:
        x = nxt
        nxt = None
        optimizer.zero_grad()
        w = 1.0
        empty = False
        if ws > 1:
            B = (x[0][0] if multimodal else x[0]).shape[0]
            lo, hi = D.split_bounds(B, rank, ws)
            empty = hi == lo
            w = (hi - lo) / B if reduction == "mean" else 1.0
            if fused and isinstance(optimizer.grad_hook, D.GradAllReduce):
                optimizer.grad_hook.weight = w if reduction == "mean" else None
            x = D.shard(x, rank, ws)
        guard.reset(device)       # a flag left by an unchecked eval call is not this batch's
        rng.reset_call_ids()      # every batch draws under call ids 1.. (eager or replayed)
        loss = None
        if empty:
            loss = torch.zeros((), dtype=torch.float32, device=device)
        elif _stepgraph.eligible(device):
            # replay of the captured forward + backward of this batch signature
            loss = _stepgraph.step(network, loss_fn, x, multimodal)
        if loss is None:
            # parameter-gradient sums batched into one launch at the end of backward
            with _defer.deferred():
                loss = backward_negated(loss_fn(network, x))
        if ahead:
            nxt = _fetch(batches, device, multimodal, True)
        if ws > 1:
            # every rank all-reduces the same set of gradients (an empty slice, or a
            # parameter the loss does not reach on some rank, gets zeros)
            D.agree_grad_pattern(params)
            if fused:
                optimizer.pack_grads()
                optimizer.reduce_grads()
            else:
                D.allreduce_grads(params, reduction, weight=w)
        # the one sync per batch, before the update: loss and the guard words
        stat = torch.cat([(loss.detach().float() * w).reshape(1), guard.words(device)])
        if ws > 1:
            torch.distributed.all_reduce(stat)
        loss_v, post_bad, loss_bad = stat.tolist()
        if post_bad or loss_bad or not math.isfinite(loss_v):
            if ws > 1:
                # every rank reached the same verdict: leave together, so no rank tears the
                # group down while another still completes the all-reduce above
                torch.distributed.barrier()
            guard.raise_for(device, (post_bad > 0, loss_bad > 0 or not math.isfinite(loss_v)),
                            "training_step")
        if fused and ws > 1:
            optimizer.apply_update()       # gradients already packed and all-reduced
        else:
            optimizer.step()
        if device.type == "cuda":
            rng.advance(device)            # the next batch draws fresh noise / dropout
        total_loss += loss_v
        num_batches += 1.
        if release_memory:
            del x
            torch.cuda.empty_cache()
        if not ahead:
            nxt = _fetch(batches, device, multimodal, False)
    return total_loss / num_batches


def _fetch(batches, device, multimodal, pinned):
    """The loader's next batch on `device` (training_util.py:38-41), or None at the end.
    pinned: staged through page-locked memory and copied without blocking the host."""
    x = next(batches, None)
    if x is None:
        return None

    def move(t):
        if pinned and t.device.type == "cpu":
            return t.pin_memory().to(device, non_blocking=True)
        return t.to(device)
    if multimodal:
        return [tuple(move(_x) for _x in modality) for modality in x]
    return tuple(move(_x) for _x in x)
