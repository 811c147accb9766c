"""Data parallelism on the HIP path, rehearsed on ONE GPU (two ranks on cuda:0 over
gloo, VAESNE_DP_BACKEND=gloo; RCCL refuses two ranks on one device):

* bench.py's own DP step (hipGraph 1: forward + backward + pack; the eager flat-gradient
  all-reduce; hipGraph 2: FusedAdamW + RNG advance), each rank on its half of the
  benchmarked B=16 golden batch and its half of the golden noise, gives the flat
  gradient of the single-process full-batch step;
* the device RNG folds the rank in (rng.rank_seed): without injected noise the two
  ranks draw different Laplace noise;
* a NaN on ONE rank (its half of the noise) makes BOTH ranks raise RuntimeError from
  training_step within the timeout, and neither rank's parameters change (the
  reference stops before its update, PhotometricVAE.py:160-161).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, build_model, golden_us, golden_x, load_golden

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, ws, *args, timeout=300):
    """Run target(rank, ws, port, q, *args) in ws fresh processes; the results are read
    BEFORE joining (a rank blocks in put() until its result leaves the pipe)."""
    import queue
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, ws, port, q) + args) for r in range(ws)]
    for pr in procs:
        pr.start()
    res = []
    try:
        for _ in range(ws):
            res.append(q.get(timeout=timeout))
    except queue.Empty:
        pass
    for pr in procs:
        pr.join(60)
        if pr.exitcode is None:
            pr.kill()
            pr.join(10)
    codes = [pr.exitcode for pr in procs]
    assert codes == [0] * ws and len(res) == ws, f"rank exit codes {codes}, {len(res)} results"
    return sorted(res, key=lambda r: r[0])


def _bench_steps(case, world, rank, us_list, graph, n_eager=3):
    """bench.Step on this rank's slice: 3 eager steps (capture warm-up) + the captured
    (or a 4th eager) step; every step consumes its own injected noise.  lr = 0, so
    every step sees the same parameters and the last step's all-reduced flat gradient
    can be compared to the single-process one at summation-order precision (AdamW
    would turn rounding-level differences of near-zero gradient elements into
    +-lr steps)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from VAESNe import distributed as D
    from VAESNe import rng
    g = load_golden(case)
    c = g["config"]
    model = build_model(c)
    x = golden_x(g, "cuda")
    B = x[0][0].shape[0]
    lo, hi = D.split_bounds(B, rank, world)
    x = [tuple(t[lo:hi] for t in m) for m in x]
    us = [[u[:, lo:hi].contiguous().cuda() for u in step_us] for step_us in us_list]
    step = bench.Step(model, x, torch.device("cuda", 0), world, use_graph=graph, lr=0.0)
    flat = [u for step_us in us for u in step_us]
    with rng.inject_uniform(flat):
        if graph:
            step.capture()          # 3 eager steps + capture (the capture draws the 4th noise)
        else:
            for _ in range(n_eager):
                step()
        step()
    torch.cuda.synchronize()
    return step.opt.flat_grad().clone().cpu(), step.loss.item()


def _us4(case):
    g = load_golden(case)
    base = golden_us(g)
    # four steps, each with its own (shifted) noise, so a step replaying another's
    # draws would show
    return [[torch.roll(u, s, dims=0) for u in base] for s in range(4)]


def _dp_bench_worker(rank, ws, port, q, case):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        grad, loss = _bench_steps(case, ws, rank, _us4(case), graph=True)
        # rank-folded device RNG: without injection the ranks draw different noise
        from VAESNe import rng
        rng.manual_seed(1234)
        u = rng.draw_uniform((64,), "cuda").cpu()
        us = [torch.empty_like(u) for _ in range(ws)]
        dist.all_gather(us, u)
        # plain arrays through the queue (a tensor would be shared by fd, dead with the rank)
        q.put((rank, grad.numpy(), loss, [t.numpy() for t in us]))
    finally:
        dist.destroy_process_group()


def test_bench_dp_step_world2_matches_single_process():
    case = "mmvae_cfg5_b16"
    ref, ref_loss = _bench_steps(case, 1, 0, _us4(case), graph=True)
    res = _spawn(_dp_bench_worker, 2, case)
    ref = ref.numpy()
    for rank, grad, loss, us in res:
        # the all-reduced flat gradient of the replayed DP step = the full batch's
        err = float(np.abs(grad - ref).max() / np.abs(ref).max())
        assert err < 1e-5, (rank, err)
        assert not np.array_equal(us[0], us[1])       # ranks draw their own noise
        assert np.array_equal(us[0], res[0][3][0]) and np.array_equal(us[1], res[1][3][1])
    # each rank's logged loss is its own shard's; together they make the full batch's
    total = sum(r[2] for r in res)
    assert abs(total - ref_loss) <= 1e-5 * abs(ref_loss), (total, ref_loss)


def _nan_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK="0", VAESNE_DP_BACKEND="gloo")
    try:
        from VAESNe import distributed as D
        from VAESNe import guard, rng
        from VAESNe.losses import m_iwae
        from VAESNe.optim import FusedAdamW
        from VAESNe.training_util import training_step
        g = load_golden("mmvae_tiny")
        c = g["config"]
        model = build_model(c)
        opt = FusedAdamW(model.parameters(), lr=1e-3)
        x = golden_x(g, "cuda")
        B = x[0][0].shape[0]
        D.init_from_env()
        lo, hi = D.split_bounds(B, rank, ws)
        us = [u[:, lo:hi].clone() for u in golden_us(g)]
        if rank == 1:
            us[1].fill_(float("nan"))       # rank 1's spectra noise only
        before = opt.flat_params().clone()
        try:
            with rng.inject_uniform(us):
                training_step(model, opt, [x], loss_fn=lambda m, xx: m_iwae(m, xx, K=c["K"]),
                              multimodal=True)
            q.put((rank, False, "", True, None))
        except RuntimeError as e:
            torch.cuda.synchronize()
            same = torch.equal(before, opt.flat_params())
            steps = opt._flat[0]["steps"].clone().cpu()
            q.put((rank, True, str(e), same, (guard.status("cuda"), float(steps.abs().max()))))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_nan_on_one_rank_raises_on_both_and_keeps_parameters():
    res = _spawn(_nan_worker, 2, timeout=240)
    for rank, raised, msg, same, extra in res:
        assert raised, f"rank {rank} did not raise"
        assert "non-finite" in msg, msg
        assert same, f"rank {rank}: a rejected step changed the parameters"
        flags, steps = extra
        assert flags == (False, False)      # cleared by the raise
        assert steps == 0.0                 # no AdamW step count advanced
