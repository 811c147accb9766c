"""Deferred parameter-gradient sums (VAESNe._defer, vaesne_colsum_flush): the
backward's ~90 per-op column sums batched into one or two launches at the end
of the backward pass.  The batched kernel adds in the same order as the per-op
one, so every gradient must be bit-identical to the immediate path; parameters
that cannot be deferred safely (accumulating into an existing .grad, used twice)
must fall back, and a parameter that also feeds a plain torch op must raise."""
import ctypes as C

import pytest
import torch

from conftest import build_model, golden_us, golden_x, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grads(case, defer, streams="1"):
    from VAESNe import _config, _defer, rng
    from VAESNe.losses import m_iwae
    saved = _config.streams
    _config.streams = streams == "1"
    try:
        g = load_golden(case)
        c = g["config"]
        model = build_model(c)
        model.train()
        with _defer.deferred(defer):
            with rng.inject_uniform(golden_us(g)):
                loss = -m_iwae(model, golden_x(g, "cuda"), K=c["K"])
            loss.backward()
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    finally:
        _config.streams = saved


@pytest.mark.parametrize("case,streams", [("mmvae_cfg5_b16", "1"), ("mmvae_cfg5_b16", "0"),
                                          ("mmvae_tiny", "1"), ("mmvae_bright", "1")])
def test_deferred_sums_bitwise_equal_immediate(case, streams):
    now = _grads(case, False, streams)
    later = _grads(case, True, streams)
    assert set(now) == set(later) and len(now) > 20
    for k in now:
        assert torch.equal(now[k], later[k]), k


def test_flush_batches_and_orders_overlapping_outputs():
    """One flush = few launches; two sums into one output (accumulate) stay ordered."""
    from VAESNe import _defer, _lib
    from VAESNe._ops import _ws
    lib = _lib.lib
    g = torch.Generator().manual_seed(0)
    M, O, I = 40000, 32, 32
    dys = [torch.randn(M, O, generator=g).to(DEV) for _ in range(3)]
    x = torch.randn(M, I, generator=g).to(DEV)
    store = (_defer.Entry * 16)()
    lst = _defer.List(C.cast(store, C.POINTER(_defer.Entry)), 0, 16)
    dW = torch.empty(O, I, device=DEV)
    db = torch.empty(O, device=DEV)
    wss = []
    for i, dy in enumerate(dys):   # dW = dys[0]^T x + dys[1]^T x + dys[2]^T x
        ws = _ws(lib.linear_bwd_weight_workspace(M, O, I), DEV)
        wss.append(ws)
        lib.linear_bwd_weight(dy.data_ptr(), O, None, 0, 0, x.data_ptr(), I, None, 0, M, O, I,
                              dW.data_ptr(), db.data_ptr(), int(i > 0), ws.data_ptr(),
                              C.byref(lst), _lib.stream())
    assert lst.count == 6
    lib.colsum_flush(C.byref(lst), _lib.stream())
    assert lst.count == 0
    ref = sum(dy.double().T @ x.double() for dy in dys)
    assert float((dW.double() - ref).abs().max() / ref.abs().max()) < 1e-5
    refb = sum(dy.double().sum(0) for dy in dys)
    assert float((db.double() - refb).abs().max() / refb.abs().max()) < 1e-5


def test_full_list_fails_loudly():
    from VAESNe import _defer, _lib
    from VAESNe._ops import _ws
    lib = _lib.lib
    store = (_defer.Entry * 1)()
    lst = _defer.List(C.cast(store, C.POINTER(_defer.Entry)), 0, 1)
    M = 40000
    dy, x = torch.randn(M, 32, device=DEV), torch.randn(M, 32, device=DEV)
    dW, db = torch.empty(32, 32, device=DEV), torch.empty(32, device=DEV)
    ws = _ws(lib.linear_bwd_weight_workspace(M, 32, 32), DEV)
    with pytest.raises(RuntimeError, match="hipError"):
        lib.linear_bwd_weight(dy.data_ptr(), 32, None, 0, 0, x.data_ptr(), 32, None, 0, M, 32, 32,
                              dW.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), C.byref(lst),
                              _lib.stream())


def test_accumulating_and_shared_parameters_fall_back():
    """.grad already set (two backward passes) and a weight used twice: correct sums."""
    from VAESNe import _defer
    from VAESNe.util_layers import Linear
    torch.manual_seed(0)
    lin = Linear(32, 32).to(DEV)
    x = torch.randn(5000, 32, device=DEV)
    with _defer.deferred():
        lin(x).square().sum().backward()
        first = lin.weight.grad.clone()
        lin(x).square().sum().backward()           # accumulates into .grad
    assert torch.allclose(lin.weight.grad, 2 * first, rtol=1e-6, atol=1e-6)
    lin.weight.grad = None
    lin.bias.grad = None
    with _defer.deferred():
        (lin(x).square().sum() + lin(2 * x).sum()).backward()   # the weight used twice
    xd = x.double().cpu()
    ref_y = torch.nn.functional.linear(xd, lin.weight.detach().double().cpu(),
                                       lin.bias.detach().double().cpu())
    gw = 2 * ref_y.T @ xd + torch.ones(5000, 32, dtype=torch.float64).T @ (2 * xd)
    assert float((lin.weight.grad.detach().double().cpu() - gw).abs().max() / gw.abs().max()) < 1e-5


def test_parameter_also_used_by_a_torch_op_raises():
    from VAESNe import _defer
    from VAESNe.util_layers import Linear
    lin = Linear(32, 32).to(DEV)
    x = torch.randn(5000, 32, device=DEV)
    with pytest.raises(RuntimeError, match="deferred gradient sums"):
        with _defer.deferred():
            (lin(x).square().sum() + lin.weight.square().sum()).backward()
    # outside deferred() the same model trains normally
    lin.weight.grad = None
    lin.bias.grad = None
    (lin(x).square().sum() + lin.weight.square().sum()).backward()
    assert torch.isfinite(lin.weight.grad).all()


def test_backward_that_raises_leaves_no_stale_deferred_state():
    """A backward that raises after some ops deferred their sums (before the flush
    callback ran) must not leave the deferral armed: the next backward queues its own
    flush and its gradients equal the immediate path bit for bit."""
    from VAESNe import _defer, rng
    from VAESNe.losses import m_iwae
    g = load_golden("mmvae_tiny")
    c = g["config"]
    model = build_model(c)
    model.train()
    # the photometry encoder's bottleneck queries are read first in the forward, so
    # their gradient arrives late in the backward, after the decoders deferred theirs
    p0 = model.vaes[0].enc.inference_transformer.initbottleneck

    def boom(_):
        raise RuntimeError("boom in backward")
    h = p0.register_hook(boom)
    with pytest.raises(RuntimeError, match="boom in backward"):
        with _defer.deferred(True):
            with rng.inject_uniform(golden_us(g)):
                loss = -m_iwae(model, golden_x(g, "cuda"), K=c["K"])
            loss.backward()
    h.remove()
    torch.cuda.synchronize()
    assert _defer._S.clist.count == 0 and not _defer._S.armed and not _defer._S.pending
    now = _grads("mmvae_tiny", False)
    later = _grads("mmvae_tiny", True)
    assert set(now) == set(later)
    for k in now:
        assert torch.equal(now[k], later[k]), k
