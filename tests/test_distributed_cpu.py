"""Data-parallel logic (VAESNe.distributed) on CPU: world_size 2
over gloo.  Each rank runs the oracle's m_iwae / elbo on its contiguous batch
shard (VAESNe.distributed.shard), the gradients are all-reduced once
(allreduce_grads / GradAllReduce) and must equal the single-process
full-batch gradient:
  * m_iwae (sum over B)  -> SUM;
  * elbo   (mean over K*B) -> each rank weighted by b_r / B, then SUM
    (the B=3 case shards raggedly, 1 + 2).
The oracle is the checker here; the reduction code under test is the
product's (the same calls bench.py / training_step make over RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import fill_rule, golden_us, golden_x, load_golden, oracle_cfg


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grads(p):
    return {k: v.grad.detach().clone() for k, v in p.items() if v.requires_grad and v.grad is not None}


def _worker(rank, ws, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from oracle import vaesne_oracle as O
        from VAESNe import distributed as D
        torch.set_num_threads(2)
        g = load_golden(name)
        c = g["config"]
        cfg = oracle_cfg(c)
        x, us = golden_x(g), golden_us(g)
        B = (x[0][0] if c["kind"] == "mmvae" else x[0]).shape[0]

        def loss_of(p, xb, ub):
            if c["kind"] == "mmvae":
                return -O.m_iwae(p, cfg, xb, c["K"], ub)[0]
            return -O.elbo(p, cfg, xb, c["K"], ub[0])[0]

        # full batch, single process
        p_full = O.make_params(cfg, fill_rule.fill, requires_grad=True)
        loss_of(p_full, x, us).backward()
        ref = _grads(p_full)
        # this rank's shard; u is sliced on its batch axis (dim 1) the same way
        p = O.make_params(cfg, fill_rule.fill, requires_grad=True)
        xs = D.shard(x, rank, ws)
        lo, hi = D.split_bounds(B, rank, ws)
        us_r = [u[:, lo:hi] for u in us]
        loss_of(p, xs, us_r).backward()
        reduction = "sum" if c["kind"] == "mmvae" else "mean"
        keys = sorted(k for k in p if p[k].requires_grad and p[k].grad is not None)
        params = [p[k] for k in keys]
        w = D.shard_fraction(B, rank, ws) if reduction == "mean" else None
        D.allreduce_grads(params, reduction, weight=w)
        err = max(float((p[k].grad - ref[k]).abs().max() / ref[k].abs().max().clamp_min(1e-30))
                  for k in keys)
        # the FusedAdamW hook path: one flat buffer through GradAllReduce
        p2 = O.make_params(cfg, fill_rule.fill, requires_grad=True)
        loss_of(p2, xs, us_r).backward()
        flat = torch.cat([p2[k].grad.reshape(-1) for k in keys])
        D.GradAllReduce(reduction, weight=w)(flat)
        flat_ref = torch.cat([ref[k].reshape(-1) for k in keys])
        err_flat = float((flat - flat_ref).abs().max() / flat_ref.abs().max())
        # broadcast_parameters: rank 1 starts from different values
        m = torch.nn.Linear(4, 3)
        with torch.no_grad():
            m.weight.fill_(float(rank + 1))
            m.bias.fill_(float(10 * rank))
        D.broadcast_parameters(m)
        bcast_ok = bool((m.weight == 1.0).all() and (m.bias == 0.0).all())
        q.put((rank, err, err_flat, bcast_ok, D.world()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["mmvae_tiny", "elbo_spec_tiny_K3"])
def test_dp_gradient_equals_full_batch(name):
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, name, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode}"
    res = sorted(q.get() for _ in range(ws))
    for rank, err, err_flat, bcast_ok, wr in res:
        assert wr == (rank, ws)
        assert err < 1e-5, (rank, err)
        assert err_flat < 1e-5, (rank, err_flat)
        assert bcast_ok


def test_shard_slices():
    from VAESNe.distributed import shard
    x = [(torch.arange(10), torch.arange(10) * 2), (torch.arange(10)[:, None].repeat(1, 3),)]
    parts = [shard(x, r, 3) for r in range(3)]
    assert [len(p[0][0]) for p in parts] == [4, 3, 3]
    assert torch.equal(torch.cat([p[0][0] for p in parts]), x[0][0])
    assert torch.equal(torch.cat([p[1][0] for p in parts]), x[1][0])
    single = (torch.arange(5),)
    assert shard(single, 0, 1) is single


def _contrast_worker(rank, ws, port, name, q):
    """negInfoNCE couples the batch: shard -> forward -> distributed.global_rows
    (all-gather of the projections) -> full-batch loss / world -> backward ->
    SUM all-reduce must give the single-process full-batch gradient."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from conftest import contrast_oracle_cfg
        from oracle import vaesne_oracle as O
        from VAESNe import distributed as D
        torch.set_num_threads(2)
        g = load_golden(name)
        c = g["config"]
        cfg = contrast_oracle_cfg(c)
        # fp64: the CE gradient cancels heavily, so fp32 summation-order noise would
        # hide a wrong exchange; in fp64 the check is sharp
        x = golden_x(g, dtype=torch.float64)
        p_full = O.make_params(cfg, fill_rule.fill, dtype=torch.float64, requires_grad=True)
        full = -O.neg_info_nce(*O.contrast_forward(p_full, cfg, x), c["T"])
        full.backward()
        ref = _grads(p_full)
        p = O.make_params(cfg, fill_rule.fill, dtype=torch.float64, requires_grad=True)
        z1, z2 = O.contrast_forward(p, cfg, D.shard(x, rank, ws))
        z1a, z2a, scale = D.global_rows(z1, z2)
        loss = -O.neg_info_nce(z1a, z2a, c["T"]) * scale
        loss.backward()
        keys = sorted(ref)
        D.allreduce_grads([p[k] for k in keys], "sum")
        err = max(float((p[k].grad - ref[k]).abs().max() / ref[k].abs().max().clamp_min(1e-30))
                  for k in keys)
        tot = loss.detach().clone()
        dist.all_reduce(tot)              # training_step's logged value
        q.put((rank, err, abs(tot.item() - full.item()) / abs(full.item()), z1a.shape[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["contrast_tiny", "contrast_selfattn"])   # B = 6 (3+3), 5 (2+3)
def test_dp_contrastive_gradient_equals_full_batch(name):
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_contrast_worker, args=(r, ws, port, name, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode}"
    B = load_golden(name)["config"]["B"]
    for rank, err, lerr, nrows in sorted(q.get() for _ in range(ws)):
        assert nrows == B
        assert err < 1e-10, (rank, err)
        assert lerr < 1e-12, (rank, lerr)
