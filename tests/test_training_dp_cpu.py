"""training_step under data parallelism, on CPU over gloo:

* the launcher's environment alone (RANK / WORLD_SIZE / MASTER_*, as torchrun sets
  them) is enough: training_step brings the process group up itself, as the
  unchanged cannon scripts need;
* sharding splits B as evenly as possible (sizes differ by <= 1), including B <
  world (a rank with an empty slice joins the all-reduce with zero gradients);
* mean objectives (elbo) weight each rank's gradient by its batch share, sum
  objectives (m_iwae-style) SUM: after two epochs the parameters equal a single
  process training on the full batches;
* every rank draws its own device noise / dropout streams (rng.rank_seed);
* a non-finite loss on ONE rank makes every rank raise RuntimeError before the
  update (the verdict rides the loss all-reduce), parameters unchanged.

The model is a small deterministic host-side VAE (no sampling), so a full batch
and its shards compose exactly; elbo runs through losses.elbo's host branch.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _ToyVAE(nn.Module):
    """Deterministic stand-in with the VAE attribute contract elbo reads
    (pz, pz_params, llik_scaling) and Laplace outputs: q(z|x) from a linear encoder,
    zs = its location repeated K times, p(x|z) from a linear decoder."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Linear(6, 4)
        self.dec = nn.Linear(2, 6)
        self.pz = torch.distributions.Laplace
        self._pz_params = nn.ParameterList([nn.Parameter(torch.zeros(1, 2), requires_grad=False),
                                            nn.Parameter(torch.ones(1, 2), requires_grad=False)])
        self.llik_scaling = 2.0
        # a trainable parameter the loss never reaches: every rank must leave its .grad
        # None (distributed.agree_grad_pattern), also the rank with an empty slice
        self.unused = nn.Parameter(torch.ones(3))

    @property
    def pz_params(self):
        return self._pz_params

    def forward(self, x, K=1):
        h = self.enc(x[0])
        mu, sc = h[:, None, :2], nn.functional.softplus(h[:, None, 2:])
        zs = mu.unsqueeze(0).expand(K, -1, -1, -1)
        loc = self.dec(zs[:, :, 0, :])
        L = torch.distributions.Laplace
        return L(mu, sc), L(loc, torch.ones_like(loc)), zs


def _data(B, nb=2):
    g = torch.Generator().manual_seed(5)
    return [(torch.randn(B, 6, generator=g), torch.zeros(B)) for _ in range(nb)]


def _train(model, batches, reduction, epochs=2):
    from VAESNe.losses import elbo
    from VAESNe.training_util import training_step
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    fn = elbo if reduction == "mean" else (lambda m, x: elbo(m, x) * x[0].shape[0])
    return [training_step(model, opt, batches, loss_fn=fn, grad_reduction=reduction)
            for _ in range(epochs)]


def _worker(rank, ws, port, B, reduction, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    try:
        torch.set_num_threads(1)
        torch.manual_seed(0)
        model = _ToyVAE()
        batches = _data(B)
        assert not dist.is_initialized()
        losses = _train(model, batches, reduction)        # brings the group up itself
        assert dist.is_initialized() and dist.get_world_size() == ws
        from VAESNe import distributed as D
        from VAESNe import rng
        seeds = [None] * ws
        dist.all_gather_object(seeds, rng.effective_seed())
        sizes = [D.split_bounds(B, r, ws) for r in range(ws)]
        q.put((rank, [p.detach().tolist() for p in model.parameters()], losses, seeds, sizes))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _single(B, reduction):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    torch.manual_seed(0)
    model = _ToyVAE()
    losses = _train(model, _data(B), reduction)
    return [p.detach() for p in model.parameters()], losses


@pytest.mark.parametrize("ws,B,reduction", [(2, 5, "mean"), (2, 5, "sum"), (3, 2, "mean"),
                                            (3, 2, "sum")])
def test_training_step_dp_equals_single_process(ws, B, reduction):
    ref_params, ref_losses = _single(B, reduction)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, B, reduction, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode}"
    res = sorted((q.get() for _ in range(ws)), key=lambda r: r[0])
    for rank, params, losses, seeds, sizes in res:
        for p, r in zip(params, ref_params):
            p = torch.tensor(p)
            assert torch.allclose(p, r, rtol=1e-5, atol=1e-6), (rank, (p - r).abs().max())
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (rank, losses, ref_losses)
        from VAESNe.rng import rank_seed   # every rank ran torch.manual_seed(0)
        assert seeds == [rank_seed(0, r) for r in range(ws)] and len(set(seeds)) == ws
        his = [hi - lo for lo, hi in sizes]
        assert sum(his) == B and max(his) - min(his) <= 1
        assert [lo for lo, _ in sizes] == sorted(lo for lo, _ in sizes)


def test_rank_seed_rule():
    from VAESNe.rng import rank_seed
    assert rank_seed(12345, 0) == 12345
    s = {rank_seed(0, r) for r in range(8)}
    assert len(s) == 8 and all(0 <= v < (1 << 63) for v in s)


def test_split_bounds_even():
    from VAESNe.distributed import shard, split_bounds
    assert [split_bounds(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert [split_bounds(2, r, 3) for r in range(3)] == [(0, 1), (1, 2), (2, 2)]
    x = [(torch.arange(10),), (torch.arange(10) * 2,)]
    parts = [shard(x, r, 3) for r in range(3)]
    assert torch.equal(torch.cat([p[1][0] for p in parts]), x[1][0])


def _fail_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    try:
        from VAESNe.losses import elbo
        from VAESNe.training_util import training_step
        torch.set_num_threads(1)
        torch.distributions.Distribution.set_default_validate_args(False)   # NaN gets to the loss
        torch.manual_seed(0)
        model = _ToyVAE()
        x, y = _data(4, nb=1)[0]
        x = x.clone()
        x[2:] = float("nan")          # rows 2..3: the slice of rank 1 only
        before = [p.detach().clone() for p in model.parameters()]
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        try:
            training_step(model, opt, [(x, y)], loss_fn=elbo)
            q.put((rank, False, "", True))
        except RuntimeError as e:
            same = all(torch.equal(a, p.detach()) for a, p in zip(before, model.parameters()))
            q.put((rank, True, str(e), same))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_nonfinite_loss_on_one_rank_raises_on_every_rank():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, ws, port, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode} (a hang ends in -15 / None)"
    res = sorted(q.get() for _ in range(ws))
    for rank, raised, msg, unchanged in res:
        assert raised, f"rank {rank} did not raise"
        assert "non-finite" in msg, msg
        assert unchanged, f"rank {rank}: parameters changed by a rejected step"


def _count_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    try:
        from VAESNe.losses import elbo
        from VAESNe.training_util import training_step
        torch.set_num_threads(1)
        torch.manual_seed(0)
        model = _ToyVAE()
        batches = [_data(4)[0] for _ in range(3)]
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        training_step(model, opt, batches, loss_fn=elbo)        # first epoch: agrees the pattern
        counts = {"all_reduce": 0, "tolist": 0, "item": 0}
        real_ar, real_tl, real_it = dist.all_reduce, torch.Tensor.tolist, torch.Tensor.item

        def ar(*a, **k):
            counts["all_reduce"] += 1
            return real_ar(*a, **k)

        def tl(self):
            counts["tolist"] += 1
            return real_tl(self)

        steps = {id(st["step"]) for st in opt.state.values()}   # torch's host step counts

        def it(self):
            if id(self) not in steps:
                counts["item"] += 1
            return real_it(self)
        dist.all_reduce, torch.Tensor.tolist, torch.Tensor.item = ar, tl, it
        try:
            training_step(model, opt, batches, loss_fn=elbo)    # steady state
        finally:
            dist.all_reduce, torch.Tensor.tolist, torch.Tensor.item = real_ar, real_tl, real_it
        q.put((rank, counts, len(batches)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_step_has_one_collective_and_one_host_read_per_batch():
    """in steady state a data-parallel training_step batch runs
    exactly ONE all-reduce (gradients, loss and guard words in one buffer: the
    gradient pattern is agreed once per loss function and batch size) and ONE host
    read (the batch's verdict), no per-parameter copies and no pattern all-reduce."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_count_worker, args=(r, ws, port, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode}"
    for rank, counts, nb in sorted(q.get() for _ in range(ws)):
        assert counts == {"all_reduce": nb, "tolist": nb, "item": 0}, (rank, counts)


def _mismatch_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    try:
        from VAESNe.losses import elbo
        from VAESNe.training_util import training_step
        torch.set_num_threads(1)
        torch.manual_seed(0)
        model = _ToyVAE()
        batches = [_data(4)[0] for _ in range(3)]
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        calls = type("Calls", (), {"n": 0})()    # an object: the step signature keys it by id

        def fn(m, x):
            calls.n += 1
            loss = elbo(m, x)
            if calls.n == 2 and dist.get_rank() == 1:   # beyond the pattern batch 0 agreed
                loss = loss + 0.0 * m.unused.sum()
            return loss
        try:
            training_step(model, opt, batches, loss_fn=fn)
            q.put((rank, ""))
        except RuntimeError as e:
            q.put((rank, str(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gradient_pattern_mismatch_raises_on_every_rank():
    """a rank whose gradients go beyond the cached agreed pattern does not raise
    alone (the others would wait in the next collective): the mismatch rides the batch's
    one all-reduce, every rank skips the update and raises the same error."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, ws, port, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode} (a hang ends in -15 / None)"
    for rank, msg in sorted(q.get() for _ in range(ws)):
        assert "agreed pattern" in msg, (rank, msg)
