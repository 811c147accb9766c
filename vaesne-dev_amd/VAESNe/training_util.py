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
joins the all-reduce with a zero gradient for every trainable parameter, so all
ranks apply the same update.  Each rank draws its own noise / dropout streams
(rng.rank_seed).  The returned value is the mean full-batch loss on every rank.

Non-finite values: the HIP kernels flag a NaN / Inf posterior or loss on the
device (VAESNe.guard); it is read after the `.item()` the loop already does
(training_util.py:46) and raises RuntimeError where the reference would stop in
pdb (PhotometricVAE.py:160-161)."""
import math

import torch

from . import _defer, guard
from . import distributed as D
from .losses import elbo
from .optim import FusedAdamW


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
    if ws > 1:
        D.sync_parameters_once(network)
        if isinstance(optimizer, FusedAdamW) and optimizer.grad_hook is None:
            optimizer.grad_hook = D.GradAllReduce(reduction)
    for x in data_loader:
        optimizer.zero_grad()
        if multimodal:
            x = [tuple(_x.to(device) for _x in modality) for modality in x]
        else:
            x = tuple(_x.to(device) for _x in x)
        w = 1.0
        empty = False
        if ws > 1:
            B = (x[0][0] if multimodal else x[0]).shape[0]
            lo, hi = D.split_bounds(B, rank, ws)
            empty = hi == lo
            w = (hi - lo) / B if reduction == "mean" else 1.0
            if isinstance(optimizer, FusedAdamW) and isinstance(optimizer.grad_hook, D.GradAllReduce):
                optimizer.grad_hook.weight = w if reduction == "mean" else None
            x = D.shard(x, rank, ws)
        if empty:
            loss = torch.zeros((), dtype=torch.float32, device=device)
            for p in network.parameters():
                if p.requires_grad:
                    p.grad = torch.zeros_like(p)
        else:
            # parameter-gradient sums batched into one launch at the end of backward
            with _defer.deferred():
                loss = -loss_fn(network, x)
                loss.backward()
        if ws > 1 and not isinstance(optimizer, FusedAdamW):
            D.allreduce_grads(network.parameters(), reduction, weight=w)
        optimizer.step()
        if ws > 1:
            loss = loss.detach().clone() * w
            torch.distributed.all_reduce(loss)
        total_loss += loss.detach().cpu().item()
        guard.check(device, "training_step")
        num_batches += 1.
        if release_memory:
            del x
            torch.cuda.empty_cache()
    return total_loss / num_batches
