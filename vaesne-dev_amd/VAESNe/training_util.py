"""One training epoch — reference training_util.py:17-53, unchanged in
behaviour for a single process.

Data parallel.  Under a launcher that describes a world
(`torchrun --nproc-per-node N script.py`: WORLD_SIZE / RANK / LOCAL_RANK), the
first call brings the process group up itself (distributed.init_from_env; the
scripts never do) and broadcasts the parameters from rank 0 once.  Each rank
trains on its contiguous slice of every batch (sizes differ by at most one) and
gradients are all-reduced once per step (distributed.FlatExchange): SUM for
sum-over-batch objectives (m_iwae, the multimodal default) and, for mean
objectives (elbo, the single-modality default), each rank's gradient weighted by
its share of the batch before the SUM.  A rank whose slice is empty (B < world)
joins the all-reduce with zero gradients, and every rank holds a gradient for the
same parameters (agreed once per loss function and batch size), so all ranks apply
the same update.  Each rank draws its own noise / dropout streams (rng.rank_seed).
The returned value is the mean full-batch loss on every rank.

Captured steps (VAESNe._stepgraph): after two eager batches of one signature
(input shapes, loss function, parameters), the forward + backward is captured
once as a hipGraph and replayed for every later batch of that signature; the
optimizer steps eagerly on the gradients as before.  Each batch draws its noise
and dropout masks under the same call ids and a per-batch device counter, so a
replayed batch computes exactly what the eager batch would (VAESNE_STEP_GRAPH=0:
always eager).

Non-finite values (VAESNe.guard): the HIP kernels flag a NaN posterior or a
NaN / Inf loss on the device.  The flag is cleared once when training_step starts
and stays set from the first flagged batch on; the update is enqueued at once
behind that device-side skip (VAESNe._update: FusedAdamW, and the scripts' own
torch.optim.AdamW applied op for op by a HIP kernel on its own state), and the
host reads each batch's (loss, flags) two batches late, while the next two run
(the reference's `.item()`, training_util.py:46).  A flagged batch raises
RuntimeError there, its update and any later one never applied (the reference
stops before its update, PhotometricVAE.py:160-161) and the optimizer's host-side
step counts rolled back.  Other optimizers step after their batch's verdict.  Under
data parallelism the gradients, the loss and both flag words travel in ONE
all-reduce (distributed.FlatExchange), so every rank skips, and raises, together.
A non-finite loss also raises (stricter than the reference, which would train on
it)."""
import collections
import math

import torch

from . import _defer, _lib, _stepgraph, _update, guard, rng
from . import distributed as D
from .losses import elbo


_SEEDS = {}


def backward_negated(value, out=None, negate=True):
    """`loss = -value; loss.backward()` (training_util.py:42-44) with the gradient seed
    -1 handed to `value` directly: the same gradients bit for bit (NegBackward
    multiplies the seed 1 by -1 exactly), without the fill and negation launches that
    sit between the forward and the backward of every step.  Returns -value
    (detached), negated after the backward was issued -- into `out` when given (one
    launch for the negation and the copy) -- or, with negate=False, `value` itself
    (detached: training_step folds the sign into its verdict words, no launch)."""
    key = (value.device, value.dtype, tuple(value.shape))
    seed = _SEEDS.get(key)
    if seed is None:
        if value.is_cuda and torch.cuda.is_current_stream_capturing():
            loss = -value          # no persistent seed yet: never allocate one in a capture
            loss.backward()
            if not negate:
                return value.detach()
            return loss.detach() if out is None else out.copy_(loss.detach())
        seed = _SEEDS[key] = torch.full(key[2], -1.0, dtype=value.dtype, device=value.device)
    value.backward(seed)
    if not negate:
        return value.detach()
    return -value.detach() if out is None else torch.neg(value.detach(), out=out)


def safelog10(x):
    tmp = max(1e-10, x)
    return math.log10(tmp)


class _Verdicts:
    """Each batch's [loss, posterior flag, loss flag], copied to pinned host memory
    behind the batch's work and read later: the host reads batch i's verdict while
    batch i+2 runs (one wait per batch, the GPU never idles for it)."""

    def __init__(self, device, slots=4):
        self.cuda = device.type == "cuda"
        self.q = collections.deque()
        self.i = 0
        if self.cuda:
            self.host = [torch.empty(3, dtype=torch.float32, pin_memory=True)
                         for _ in range(slots)]
            self.dev = torch.empty(slots, 3, dtype=torch.float32, device=device)
            self.ev = [torch.cuda.Event() for _ in range(slots)]

    def words(self, val, scale, flag):
        """[val * scale, flag words] for the next push: on the device in one launch
        (vaesne_loss_stat, into the slot's own buffer), or on the host."""
        if not self.cuda:
            return torch.cat([(val.detach().float() * scale).reshape(1), torch.zeros(2)])
        out = self.dev[self.i % len(self.host)]
        v = val.detach()
        if v.dtype != torch.float32 or not v.is_contiguous():
            v = v.float().contiguous()
        _lib.lib.loss_stat(v.data_ptr(), float(scale), flag.data_ptr(), out.data_ptr(),
                           _lib.stream())
        return out

    def push(self, stat, batch):
        if not self.cuda:
            self.q.append((batch, stat.tolist()))
            return
        k = self.i % len(self.host)
        self.i += 1
        self.host[k].copy_(stat, non_blocking=True)
        self.ev[k].record()
        self.q.append((batch, k))

    def __len__(self):
        return len(self.q)

    def pop(self):
        batch, k = self.q.popleft()
        if not self.cuda:
            return batch, k
        self.ev[k].synchronize()
        return batch, self.host[k].tolist()


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
    upd = _update.for_optimizer(optimizer)
    xchg = _exchange(upd, network, device) if ws > 1 else None
    cuda = device.type == "cuda"
    if cuda:
        guard.reset(device)      # a flag left by an unchecked eval call is not this call's
        rng.begin_training(device)
    verdicts = _Verdicts(device)
    last_update = [-1]           # index of the last batch whose update was enqueued

    def settle(keep):
        """Read verdicts until `keep` remain pending; raise on a flagged batch."""
        nonlocal total_loss, num_batches
        while len(verdicts) > keep:
            batch, (loss_v, post_bad, loss_bad) = verdicts.pop()
            if post_bad or loss_bad or not math.isfinite(loss_v):
                # the sticky flag made the device skip this batch's update and every later
                # one: undo their host bookkeeping, so the optimizer is as before the batch
                upd.rollback(max(0, last_update[0] - batch + 1))
                if cuda:
                    torch.cuda.synchronize(device)
                if ws > 1:
                    # every rank read the same reduced verdict: leave together, so no rank
                    # tears the group down while another is still in a collective
                    torch.distributed.barrier()
                    if loss_bad >= D.FlatExchange.MISMATCH:
                        guard.reset(device)
                        raise RuntimeError(
                            "VAESNe data parallel: a parameter got a gradient that the agreed "
                            "pattern of this step signature does not have (on some rank); the "
                            "update was not applied")
                guard.raise_for(device, (post_bad > 0, loss_bad > 0 or not math.isfinite(loss_v)),
                                "training_step")
            total_loss += loss_v
            num_batches += 1.

    # the next batch is collated and copied to the device while this one runs (its copy
    # queued behind this batch's work, from pinned memory): the host's DataLoader work
    # leaves the per-batch idle window.  Not in the host-generator parity mode, where
    # the model's draws and a dataset's share torch's CPU generator in the reference's
    # order.
    ahead = cuda and rng.capturable()
    batches = iter(data_loader)
    nxt = _fetch(batches, device, multimodal, ahead)
    index = 0
    while nxt is not None:
        x = nxt
        nxt = None
        optimizer.zero_grad()
        w = 1.0
        empty = False
        B = None
        if ws > 1:
            B = (x[0][0] if multimodal else x[0]).shape[0]
            lo, hi = D.split_bounds(B, rank, ws)
            empty = hi == lo
            w = (hi - lo) / B if reduction == "mean" else 1.0
            x = D.shard(x, rank, ws)
        rng.reset_call_ids()      # every batch draws under call ids 1.. (eager or replayed)
        # `val`: the objective (the loss is -val; the sign goes into the verdict words)
        val = None
        if empty:
            val = torch.zeros((), dtype=torch.float32, device=device)
        elif _stepgraph.eligible(device):
            # replay of the captured forward + backward of this batch signature
            val = _stepgraph.step(network, loss_fn, x, multimodal)
        if val is None:
            # parameter-gradient sums batched into one launch at the end of backward
            with _defer.deferred():
                val = backward_negated(loss_fn(network, x), negate=False)
        if ahead:
            nxt = _fetch(batches, device, multimodal, True)
        flag = guard.flag(device) if cuda else None
        if ws > 1:
            # ONE collective: gradients, loss and guard words (distributed.FlatExchange)
            key = (_stepgraph._fn_key(loss_fn), multimodal, B, reduction)
            stat = xchg.run(val, -w, reduction == "mean", flag, xchg.agree(key))
            skip, flat = xchg.skip_ptr(), xchg.grads_flat()
        else:
            stat = verdicts.words(val, -w, flag)     # [loss * w, flags]: one launch
            skip, flat = (flag.data_ptr() if cuda else None), None
        if cuda and upd.ready():
            upd.update(skip, flat)        # applied on the device unless a batch was flagged
            last_update[0] = index
            verdicts.push(stat, index)
            # the verdict of the batch before the previous one: two batches stay queued
            # on the device while the host prepares the next, so host jitter (a slow
            # collate, a page-in) does not drain the queue at small batches
            settle(2)
        else:
            verdicts.push(stat, index)
            settle(0)                     # the verdict first, then the optimizer's own step
            optimizer.step()
            last_update[0] = index
        if cuda:
            rng.advance(device)            # the next batch draws fresh noise / dropout
        index += 1
        if release_memory:
            del x
            torch.cuda.empty_cache()
        if not ahead:
            nxt = _fetch(batches, device, multimodal, False)
    settle(0)
    return total_loss / num_batches


def _exchange(upd, network, device):
    """The data-parallel buffer of (updater, network): the updater's parameters in its
    order (FusedAdamW: its flat layout) then any other trainable parameter."""
    order = upd.layout()
    seen = {id(p) for p in order}
    order += [p for p in network.parameters() if p.requires_grad and id(p) not in seen]
    key = tuple(id(p) for p in order)
    x = getattr(upd, "_exchange", None)
    if x is None or x[0] != key:
        buf = None
        if isinstance(upd, _update.FusedUpdater) and len(order) == len(upd.layout()):
            buf = upd.opt.exchange_buffer()       # FusedAdamW's flat gradient, reduced in place
        x = upd._exchange = (key, D.FlatExchange(order, device, buf))
    return x[1]


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
