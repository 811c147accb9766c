"""One training epoch — reference training_util.py:17-53, unchanged in
behaviour for a single process.  Under torch.distributed (world > 1) each
rank trains on its contiguous slice of every batch and gradients are
all-reduced once per step (VAESNe.distributed): SUM for sum-over-batch
objectives (m_iwae, the multimodal default) and MEAN for mean objectives
(elbo, the single-modality default).  The returned value is the mean
full-batch loss on every rank."""
import math

import torch

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
    rank, ws = D.world()
    reduction = grad_reduction or ("sum" if multimodal else "mean")
    if ws > 1 and isinstance(optimizer, FusedAdamW) and optimizer.grad_hook is None:
        optimizer.grad_hook = D.GradAllReduce(reduction)
    for x in data_loader:
        optimizer.zero_grad()
        if multimodal:
            x = [tuple(_x.to(device) for _x in modality) for modality in x]
        else:
            x = tuple(_x.to(device) for _x in x)
        w = 1.0
        if ws > 1:
            B = (x[0][0] if multimodal else x[0]).shape[0]
            w = D.shard_fraction(B, rank, ws) if reduction == "mean" else 1.0
            if isinstance(optimizer, FusedAdamW) and isinstance(optimizer.grad_hook, D.GradAllReduce):
                optimizer.grad_hook.weight = w if reduction == "mean" else None
            x = D.shard(x, rank, ws)
        loss = -loss_fn(network, x)
        loss.backward()
        if ws > 1 and not isinstance(optimizer, FusedAdamW):
            D.allreduce_grads(network.parameters(), reduction, weight=w)
        optimizer.step()
        if ws > 1:
            loss = loss.detach().clone() * w
            torch.distributed.all_reduce(loss)
        total_loss += loss.detach().cpu().item()
        num_batches += 1.
        if release_memory:
            del x
            torch.cuda.empty_cache()
    return total_loss / num_batches
