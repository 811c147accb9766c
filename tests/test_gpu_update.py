"""training_step's update behind the device-side skip (VAESNe._update).

* `vaesne_adamw_list` applies torch.optim.AdamW's foreach update (the scripts'
  `AdamW(params, lr)`, cannon/ZTF_photospect.py:119) BITWISE as torch does: two
  parameter groups, a parameter that gets its first gradient late and one that skips
  a step, the optimizer's own state tensors and state_dict;
* the script loop (training_step with torch.optim.AdamW, captured steps) gives the
  same parameters, losses and optimizer state bit for bit whether the update is
  torch's own step() after each batch's verdict or the kernel enqueued behind the
  device skip with the verdict read one batch late;
* a non-finite batch in the middle of an epoch raises, and the model and the
  optimizer (moments AND torch's host-side step counts) are exactly as after the
  batches before it -- for torch.optim.AdamW and FusedAdamW.
"""
import sys

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _tensors(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(33, 7, generator=g), torch.randn(5, generator=g),
            torch.randn(4, 4, 4, generator=g), torch.randn(3000, generator=g) * 1e-3]


def _grad(step, i, shape):
    if (step == 0 and i == 1) or (step == 2 and i == 2):
        return None           # 1 starts late, 2 skips a step
    g = torch.Generator().manual_seed(1000 + 10 * step + i)
    return torch.randn(shape, generator=g) * (10.0 ** (i - 2))


def _adamw_run(steps, device_update, fma=None, monkeypatch=None):
    from VAESNe import _update
    ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in _tensors(0)]
    opt = torch.optim.AdamW([{"params": ps[:2]}, {"params": ps[2:], "lr": 3e-3,
                                                  "weight_decay": 0.1, "betas": (0.8, 0.95)}],
                            lr=1e-2)
    upd = _update.TorchAdamWUpdater(opt)
    if fma is not None:
        monkeypatch.setattr(_update, "TORCH_FMA", fma)
    for s in range(steps):
        for i, p in enumerate(ps):
            g = _grad(s, i, p.shape)
            p.grad = None if g is None else g.to(DEV)
        if device_update:
            assert upd.ready()
            upd.update(None)
        else:
            opt.step()
    torch.cuda.synchronize()
    return [p.detach().clone() for p in ps], opt


def test_adamw_list_against_torch_adamw(monkeypatch):
    """Both contraction variants of vaesne_adamw_list against torch.optim.AdamW: each
    within fp32 rounding, and the shipped one (_update.TORCH_FMA) bitwise -- moments and
    state_dict included."""
    from VAESNe import _update
    shipped = _update.TORCH_FMA
    ref, ropt = _adamw_run(6, False)
    res = {}
    for fma in (1, 0):
        got, gopt = _adamw_run(6, True, fma=fma, monkeypatch=monkeypatch)
        for a, b in zip(got, ref):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (fma, (a - b).abs().max())
        rs, gs = ropt.state_dict(), gopt.state_dict()
        assert rs["param_groups"] == gs["param_groups"]
        assert set(rs["state"]) == set(gs["state"])
        same = all(torch.equal(a, b) for a, b in zip(got, ref))
        for k in rs["state"]:
            assert float(rs["state"][k]["step"]) == float(gs["state"][k]["step"]), k
            assert not gs["state"][k]["step"].is_cuda
            for name in ("exp_avg", "exp_avg_sq"):
                a, b = rs["state"][k][name], gs["state"][k][name]
                assert torch.allclose(a, b, rtol=1e-6, atol=1e-12), (fma, k, name)
                same = same and torch.equal(a, b)
        res[fma] = same
    monkeypatch.setattr(_update, "TORCH_FMA", shipped)
    assert res[shipped], f"bitwise equal to torch.optim.AdamW by variant (fma: bitwise): {res}"


def _script_run(device_update, monkeypatch, epochs=2, n=12, B=4, opt_kind="torch",
                batches=None, loss=None):
    sys.path.insert(0, ROOT)
    import bench
    from VAESNe import _update, rng
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.optim import FusedAdamW
    from VAESNe.training_util import training_step
    if not device_update:
        monkeypatch.setattr(_update, "for_optimizer", lambda opt: _update.Updater(opt))
    torch.manual_seed(0)
    model = bench.make_model(DEV, 0.1)
    rng.manual_seed(99)
    opt = (torch.optim.AdamW if opt_kind == "torch" else FusedAdamW)(model.parameters(), lr=1e-3)
    if batches is None:
        x = bench.synthetic_batch(n, 7, "cpu")
        batches = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                             batch_size=B, shuffle=False)
    fn = loss or (lambda m, xx: m_iwae(m, xx, K=3))
    losses, err = [], None
    try:
        for _ in range(epochs):
            losses.append(training_step(model, opt, batches, loss_fn=fn, multimodal=True))
    except RuntimeError as e:
        err = str(e)
    torch.cuda.synchronize()
    monkeypatch.undo()
    return [p.detach().clone() for p in model.parameters()], losses, opt, err


def _state_equal(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert set(sa["state"]) == set(sb["state"])
    for k in sa["state"]:
        for name, v in sa["state"][k].items():
            assert torch.equal(v.cpu(), sb["state"][k][name].cpu()), (k, name)


def test_script_loop_device_update_bitwise(monkeypatch):
    from VAESNe import _stepgraph
    ref = _script_run(False, monkeypatch)
    _stepgraph.clear()
    got = _script_run(True, monkeypatch)
    _stepgraph.clear()
    assert ref[3] is None and got[3] is None
    assert got[1] == ref[1], (got[1], ref[1])
    for a, b in zip(got[0], ref[0]):
        assert torch.equal(a, b)
    _state_equal(got[2], ref[2])


def _batches(nan_at=None, n=4, B=4):
    sys.path.insert(0, ROOT)
    import bench
    out = []
    for i in range(n):
        x = bench.synthetic_batch(B, 100 + i, "cpu")
        if i == nan_at:
            x[1] = (x[1][0].clone().fill_(float("inf")),) + tuple(x[1][1:])
        out.append(x)
    return out


@pytest.mark.parametrize("opt_kind", ["torch", "fused"])
def test_nonfinite_batch_mid_epoch_rolls_back(opt_kind, monkeypatch):
    """Batch 2 of 4 is non-finite: training_step raises (read one batch late), and the
    model and the optimizer are bit for bit those of a run over batches 0 and 1 only."""
    from VAESNe import _stepgraph, guard
    good = _batches()[:2]
    ref = _script_run(True, monkeypatch, epochs=1, opt_kind=opt_kind, batches=good)
    _stepgraph.clear()
    got = _script_run(True, monkeypatch, epochs=1, opt_kind=opt_kind, batches=_batches(nan_at=2))
    _stepgraph.clear()
    assert ref[3] is None
    assert got[3] is not None and "non-finite" in got[3], got[3]
    assert guard.status("cuda") == (False, False)
    for a, b in zip(got[0], ref[0]):
        assert torch.equal(a, b)
    if opt_kind == "torch":
        _state_equal(got[2], ref[2])
        steps = {float(s["step"]) for s in got[2].state_dict()["state"].values()}
        assert steps == {2.0}, steps
    else:
        fa, fb = got[2]._flat[0], ref[2]._flat[0]
        for k in ("flat", "m", "v", "steps"):
            assert torch.equal(fa[k], fb[k]), k
    assert np.isfinite(ref[1][0])


def test_loss_stat_words():
    """vaesne_loss_stat: a batch's verdict words [value * scale, flag0, flag1] in one launch
    (training_step's stat, the data-parallel exchange's tail words)."""
    from VAESNe import _lib
    v = torch.tensor([3.5], device=DEV)
    flag = torch.tensor([0, 7], dtype=torch.int32, device=DEV)
    out = torch.full((3,), 9.0, device=DEV)
    assert _lib.lib.loss_stat(v.data_ptr(), -0.25, flag.data_ptr(), out.data_ptr(), _lib.stream()) == 0
    torch.cuda.synchronize()
    assert out.tolist() == [-0.875, 0.0, 7.0]
    out.fill_(9.0)
    assert _lib.lib.loss_stat(v.data_ptr(), 1.0, None, out.data_ptr(), _lib.stream()) == 0
    torch.cuda.synchronize()
    assert out.tolist() == [3.5, 0.0, 0.0]
    # a non-finite value raises the loss flag word on the device (and in out[2])
    for bad in (float("nan"), float("inf")):
        v.fill_(bad)
        flag.zero_()
        assert _lib.lib.loss_stat(v.data_ptr(), 2.0, flag.data_ptr(), out.data_ptr(),
                                  _lib.stream()) == 0
        torch.cuda.synchronize()
        assert flag.tolist() == [0, 1] and out[1:].tolist() == [0.0, 1.0]
        assert not np.isfinite(out[0].item())
    assert _lib.lib.loss_stat(v.data_ptr(), 1.0, None, out.data_ptr(), _lib.stream()) == 0
    torch.cuda.synchronize()
    assert out[1:].tolist() == [0.0, 1.0]


def test_nonfinite_custom_torch_loss_rolls_back(monkeypatch):
    """A loss_fn composed of torch ops (no HIP loss kernel flags it) turns non-finite on
    batch 2 of 4: the verdict words flag it on the device, so the update queued behind them
    is skipped; training_step raises, and the model and torch.optim.AdamW (moments and host
    step counts) are bit for bit those of a run over batches 0 and 1."""
    from VAESNe import _stepgraph, guard

    def with_scale(batches, bad_at=None):
        # a third batch entry the model never sees: the loss's multiplier (NaN at bad_at)
        out = []
        for i, x in enumerate(batches):
            w = torch.full((x[0][0].shape[0], 1), float("nan") if i == bad_at else 1.0)
            out.append([x[0], x[1], (w,)])
        return out

    from VAESNe.losses import m_iwae
    fn = lambda m, xx: m_iwae(m, [xx[0], xx[1]], K=3) * xx[2][0].mean()
    ref = _script_run(True, monkeypatch, epochs=1, batches=with_scale(_batches()[:2]), loss=fn)
    _stepgraph.clear()
    got = _script_run(True, monkeypatch, epochs=1, batches=with_scale(_batches(), bad_at=2),
                      loss=fn)
    _stepgraph.clear()
    assert ref[3] is None
    assert got[3] is not None and "non-finite" in got[3], got[3]
    assert guard.status("cuda") == (False, False)
    for a, b in zip(got[0], ref[0]):
        assert torch.equal(a, b)
    _state_equal(got[2], ref[2])
    steps = {float(s["step"]) for s in got[2].state_dict()["state"].values()}
    assert steps == {2.0}, steps
