"""GPU checks of the drop-in boundary beyond the golden forward / gradient cases:

* checkpoints the reference wrote (its seeded default init, tests/golden/ckpt_*.pt,
  loaded with weights_only=True) reproduce the reference's loss on the HIP path;
* non-finite values raise RuntimeError from training_step (device flag read at the
  loop's existing sync; the reference stops in pdb, PhotometricVAE.py:160-161);
* training_step data parallel on the HIP path: two ranks (gloo, both on cuda:0)
  each take half of the batch with their half of the golden noise; the all-reduced
  flat gradient equals the single-process full-batch gradient and the updated
  parameters match.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, build_model, construct_model, golden_us, golden_x, load_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["mmvae_cfg5", "mmvae_bright"])
def test_reference_checkpoint_reproduces_loss(name):
    from VAESNe import rng
    from VAESNe.losses import m_iwae
    g = load_golden("ckpt_" + name)
    c = g["config"]
    model = construct_model(c)
    model.load_state_dict(torch.load(os.path.join(GOLDEN, f"ckpt_{name}.pt"), weights_only=True))
    model = model.cuda().train()
    x = golden_x(load_golden(name), "cuda")
    with torch.no_grad(), rng.inject_uniform(golden_us(g)):
        loss = -m_iwae(model, x, K=c["K"])
    ref = float(g["loss"])
    assert abs(loss.item() - ref) <= 1e-5 * abs(ref), (loss.item(), ref)


def _tiny():
    from VAESNe.optim import FusedAdamW
    g = load_golden("mmvae_tiny")
    model = build_model(g["config"])
    return g, model, FusedAdamW(model.parameters(), lr=1e-3)


def test_nonfinite_loss_raises_from_training_step():
    from VAESNe import guard, rng
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    g, model, opt = _tiny()
    K = g["config"]["K"]
    x = golden_x(g, "cuda")
    fn = lambda m, xx: m_iwae(m, xx, K=K)
    bad = [torch.full_like(u, float("nan")) for u in golden_us(g)]
    before = opt.flat_params().clone()
    with rng.inject_uniform(bad), pytest.raises(RuntimeError, match="non-finite loss"):
        training_step(model, opt, [x], loss_fn=fn, multimodal=True)
    assert guard.status("cuda") == (False, False)       # cleared by the raise
    # raised BEFORE the update (the reference stops before optimizer.step)
    assert torch.equal(opt.flat_params(), before)
    # a flag left by an unchecked eval call does not fail the next training batch
    guard.flag("cuda")[0] = 1
    g2, model2, opt2 = _tiny()
    with rng.inject_uniform(golden_us(g)):
        assert np.isfinite(training_step(model2, opt2, [x], loss_fn=fn, multimodal=True))


def test_nonfinite_posterior_is_flagged():
    from VAESNe import guard, rng
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    g, model, opt = _tiny()
    K = g["config"]["K"]
    x = golden_x(g, "cuda")
    with torch.no_grad():     # a diverged encoder head: NaN posterior location
        model.vaes[1].enc.inference_transformer.bottleneckfc.fc2.bias[0] = float("nan")
    with rng.inject_uniform(golden_us(g)), pytest.raises(RuntimeError, match="posterior"):
        training_step(model, opt, [x], loss_fn=lambda m, xx: m_iwae(m, xx, K=K), multimodal=True)
    assert guard.status("cuda") == (False, False)
    # non-finite data: caught at the latest by the loss flag
    g, model, opt = _tiny()
    x[1] = (x[1][0].clone().fill_(float("inf")),) + tuple(x[1][1:])
    with rng.inject_uniform(golden_us(g)), pytest.raises(RuntimeError, match="non-finite"):
        training_step(model, opt, [x], loss_fn=lambda m, xx: m_iwae(m, xx, K=K), multimodal=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, ws, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from VAESNe import distributed as D
    from VAESNe import rng
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    g, model, opt = _tiny()
    K = g["config"]["K"]
    x = golden_x(g, "cuda")
    us = golden_us(g)
    fn = lambda m, xx: m_iwae(m, xx, K=K)
    # single process, full batch
    with rng.inject_uniform(us):
        full_loss = training_step(model, opt, [x], loss_fn=fn, multimodal=True)
    ref_grad = opt.flat_grad().clone()
    ref_sd = {k: v.norm().item() for k, v in model.state_dict().items()}
    # data parallel: this rank's half of the batch and of the noise
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        g, model, opt = _tiny()
        B = x[0][0].shape[0]
        lo, hi = D.split_bounds(B, rank, ws)
        with rng.inject_uniform([u[:, lo:hi] for u in us]):
            dp_loss = training_step(model, opt, [x], loss_fn=fn, multimodal=True)
        gerr = float((opt.flat_grad() - ref_grad).abs().max() / ref_grad.abs().max())
        sd = {k: v.norm().item() for k, v in model.state_dict().items()}
        perr = max(abs(sd[k] - n) / max(n, 1.0) for k, n in ref_sd.items()
                   if not k.endswith("in_proj_bias"))
        q.put((rank, gerr, perr, abs(dp_loss - full_loss) / abs(full_loss)))
    finally:
        dist.destroy_process_group()


def test_training_step_data_parallel_matches_full_batch():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, ws, port, q)) for r in range(ws)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(240)
        assert pr.exitcode == 0, f"rank exit code {pr.exitcode}"
    for rank, gerr, perr, lerr in sorted(q.get() for _ in range(ws)):
        assert gerr < 1e-5, (rank, gerr)
        assert perr < 1e-5, (rank, perr)
        assert lerr < 1e-5, (rank, lerr)


def _b16_grads(streams):
    from VAESNe import _config, rng
    from VAESNe.losses import m_iwae
    saved = _config.streams
    _config.streams = streams == "1"
    try:
        g = load_golden("mmvae_cfg5_b16")
        c = g["config"]
        model = build_model(c)
        model.train()
        with rng.inject_uniform(golden_us(g)):
            loss = -m_iwae(model, golden_x(g, "cuda"), K=c["K"])
        loss.backward()
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    finally:
        _config.streams = saved


def test_side_streams_bitwise_equal_single_stream_at_bench_config():
    """The photometry branch and the encoder's context self-attention paths run on
    side streams; at the benchmarked B=16 their gradients must equal the one-stream
    run bit for bit (a cross-stream allocator reuse once corrupted two k|v weight
    gradients here while every B <= 4 case passed)."""
    one = _b16_grads("0")
    many = _b16_grads("1")
    assert set(one) == set(many)
    for k in one:
        assert torch.equal(one[k], many[k]), k


def test_captured_step_equals_eager_at_bench_config():
    """bench.py's hipGraph-captured step (forward, backward, pack, FusedAdamW) gives
    bit-identical parameters to the same steps run eagerly, at B=16."""
    import bench
    from VAESNe import rng
    g = load_golden("mmvae_cfg5_b16")
    c = g["config"]
    us = [u.cuda() for u in golden_us(g)]    # device tensors: no H2D copy inside the capture
    out = []
    for graph in (False, True):
        model = build_model(c)
        x = golden_x(g, "cuda")
        step = bench.Step(model, x, torch.device("cuda", 0), 1, use_graph=graph)
        with rng.inject_uniform(us * 4):      # 3 warm-up steps + the captured / 4th step
            if graph:
                step.capture()
            else:
                for _ in range(3):
                    step()
            step()
        torch.cuda.synchronize()
        out.append((step.opt.flat_params().clone(), step.loss.item()))
    assert out[0][1] == out[1][1]
    assert torch.equal(out[0][0], out[1][0])
