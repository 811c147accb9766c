"""Contrastive pretraining (ContraPhotSpec + negInfoNCE) and the regression heads
(§8(f) row 4).  Golden vectors: tests/golden/gen_golden_contrast.py ran the
reference package (contrastiveNets.py, losses.py:98-110, regression.py).

CPU: the oracle restatement and the module key layout against the fixtures.
GPU: the HIP build (encoders, projection MLPs, the fused InfoNCE kernels, AdamW)
against the fixtures, and the InfoNCE kernels against an fp64 restatement on
random and edge shapes (B = 1, zero-norm rows, D wider than a workgroup).
"""
import json

import numpy as np
import pytest
import torch

from conftest import (CONTRAST_CASES, END2END_CASES, build_contrast_model, contrast_oracle_cfg,
                      fill_rule, golden_x, load_golden)
from oracle import vaesne_oracle as O


def _rel(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _grad_names(g):
    return json.loads(str(g["grad_names"]))


def _end2end_shapes(c, cfg):
    s = O.encoder_param_shapes(cfg, "enc.")
    dims = [c["Lz"] * c["Dz"]] + list(c["hidden"]) + [c["out"]]
    for i in range(len(dims) - 1):
        s[f"outfc.mlp.{2 * i}.weight"] = (dims[i + 1], dims[i])
        s[f"outfc.mlp.{2 * i}.bias"] = (dims[i + 1],)
    return s


def _head_mlp(g, nm):
    return {"outfc." + k.split(":", 1)[1]: torch.from_numpy(g[k]) for k in g
            if k.startswith(nm + ":")}


# ----------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("name", CONTRAST_CASES)
def test_oracle_contrast_matches_reference(name):
    g = load_golden(name)
    c = g["config"]
    cfg = contrast_oracle_cfg(c)
    p = O.make_params(cfg, fill_rule.fill, requires_grad=True)
    x = golden_x(g)
    z1, z2 = O.contrast_forward(p, cfg, x)
    assert _rel(z1, g["z1"]) < 1e-5 and _rel(z2, g["z2"]) < 1e-5
    loss = -O.neg_info_nce(z1, z2, c["T"])
    assert abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])) < 1e-6
    loss.backward()
    names = _grad_names(g)
    assert set(names) == set(p)          # every parameter receives a gradient
    for k in names:
        assert _rel(p[k].grad, g["grad:" + k]) < 1e-3, k   # CE-gradient cancellation
    # frozen-encoder regression heads (regression.py:28-65)
    with torch.no_grad():
        pf = O.photo_encoder(p, "photometry_encoder", cfg.photo(), *x[0], 0.0, False)
        sf = O.spec_encoder(p, "spectra_encoder", cfg.spec(), *x[1], 0.0, False)
        for nm, h in (("photohead", pf), ("spechead", sf)):
            y = O.mlp(_head_mlp(g, nm), "outfc", h.reshape(h.shape[0], -1), 2)
            assert _rel(y, g[nm + "_y"]) < 1e-5, nm


@pytest.mark.parametrize("name", END2END_CASES)
def test_oracle_end2end_matches_reference(name):
    g = load_golden(name)
    c = g["config"]
    cfg = contrast_oracle_cfg(c)
    p = O.make_params(_end2end_shapes(c, cfg), fill_rule.fill, requires_grad=True)
    kind = "photo" if c["kind"] == "end2end_photo" else "spec"
    y = O.end2end_regression(p, kind, cfg, golden_x(g), len(c["hidden"]))
    assert _rel(y, g["y"]) < 1e-5
    loss = ((y - torch.from_numpy(g["target"])) ** 2).mean()
    assert abs(loss.item() - float(g["loss"])) / float(g["loss"]) < 1e-6
    loss.backward()
    for k in _grad_names(g):
        assert _rel(p[k].grad, g["grad:" + k]) < 1e-4, k


@pytest.mark.parametrize("name", CONTRAST_CASES + END2END_CASES)
def test_module_keys_match_reference(name):
    """state_dict keys / shapes of the build's modules = the reference's (the
    fixtures list every parameter the reference trained)."""
    g = load_golden(name)
    m = build_contrast_model(g["config"], device="cpu")
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ref = {k: tuple(g["grad:" + k].shape) for k in _grad_names(g)}
    assert sd == ref


def test_infonce_oracle_matches_torch_cross_entropy():
    """The restatement's explicit CE equals F.cross_entropy / F.normalize."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(5)
    z1, z2 = torch.randn(9, 4, generator=gen), torch.randn(9, 4, generator=gen)
    n1, n2 = F.normalize(z1, dim=-1), F.normalize(z2, dim=-1)
    lg = n1 @ n2.T / 0.07
    lab = torch.arange(9)
    ref = -(F.cross_entropy(lg, lab) + F.cross_entropy(lg.T, lab)) / 2
    assert abs(O.neg_info_nce(z1, z2, 0.07).item() - ref.item()) < 1e-5


# ----------------------------------------------------------------- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("name", CONTRAST_CASES)
def test_gpu_contrast_matches_reference(name):
    from VAESNe.losses import negInfoNCE
    from VAESNe.optim import FusedAdamW
    from VAESNe.regression import contrasphotoregressionHead, contrasspecregressionHead
    from VAESNe.training_util import training_step
    g = load_golden(name)
    c = g["config"]
    model = build_contrast_model(c)
    model.train()
    x = golden_x(g, "cuda")
    z1, z2 = model(x)
    assert _rel(z1, g["z1"]) < 1e-5 and _rel(z2, g["z2"]) < 1e-5
    loss = -negInfoNCE(model, x, temperature=c["T"])
    assert abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])) < 1e-5
    loss.backward()
    prm = dict(model.named_parameters())
    for k in _grad_names(g):
        assert _rel(prm[k].grad, g["grad:" + k]) < 1e-3, k
    # regression heads on the frozen encoders, the fixtures' MLP weights
    for nm, cls, xx in (("photohead", contrasphotoregressionHead, x[0]),
                        ("spechead", contrasspecregressionHead, x[1])):
        net = build_contrast_model(c)
        head = cls(net, outdim=3, MLPlatent=[16, 16]).cuda()
        assert not any(q.requires_grad for q in net.parameters())
        head.outfc.load_state_dict({k[len("outfc."):]: v for k, v in _head_mlp(g, nm).items()})
        y = head(xx)
        assert _rel(y, g[nm + "_y"]) < 1e-5, nm
    # AdamW trajectory through training_step (cannon/test_photospectra_contrast.py:124-127)
    model = build_contrast_model(c)
    opt = FusedAdamW(model.parameters(), lr=2.5e-4)
    losses = [training_step(model, opt, [x], multimodal=True,
                            loss_fn=lambda m, xx: negInfoNCE(m, xx, temperature=c["T"]))
              for _ in range(c["steps"])]
    np.testing.assert_allclose(losses, g["traj_losses"], rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", END2END_CASES)
def test_gpu_end2end_matches_reference(name):
    g = load_golden(name)
    c = g["config"]
    model = build_contrast_model(c)
    model.train()
    y = model(golden_x(g, "cuda"))
    assert _rel(y, g["y"]) < 1e-5
    loss = torch.nn.MSELoss()(y, torch.from_numpy(g["target"]).cuda())
    assert abs(loss.item() - float(g["loss"])) / float(g["loss"]) < 1e-5
    loss.backward()
    prm = dict(model.named_parameters())
    for k in _grad_names(g):
        assert _rel(prm[k].grad, g["grad:" + k]) < 1e-3, k


@pytest.mark.gpu
@pytest.mark.parametrize("B,D,T,zero_row", [(1, 8, 0.1, False), (6, 8, 0.07, False),
                                            (37, 8, 0.07, True), (256, 8, 0.1, False),
                                            (1000, 24, 0.07, False), (300, 300, 0.5, True),
                                            (64, 1, 0.2, False)])
def test_gpu_infonce_kernels_vs_fp64(B, D, T, zero_row):
    from VAESNe import _ops
    gen = torch.Generator().manual_seed(B * 1000 + D)
    z1 = torch.randn(B, D, generator=gen)
    z2 = torch.randn(B, D, generator=gen) + 0.5 * z1      # correlated pairs
    if zero_row:
        z1[B // 2] = 0.0
    a, b = z1.cuda().requires_grad_(True), z2.cuda().requires_grad_(True)
    out = _ops.InfoNCEFn.apply(a, b, T)
    gout = 1.7
    (out * gout).backward()
    r1, r2 = z1.double().requires_grad_(True), z2.double().requires_grad_(True)
    ref = O.neg_info_nce(r1, r2, T)
    (ref * gout).backward()
    assert abs(out.item() - ref.item()) <= 1e-5 * max(abs(ref.item()), 1.0)
    assert torch.isfinite(a.grad).all() and torch.isfinite(b.grad).all()
    if D == 1:   # n = sign(z): the normalisation's Jacobian is exactly 0
        assert a.grad.abs().max() < 1e-6 and b.grad.abs().max() < 1e-6
    else:
        assert _rel(a.grad, r1.grad) < 1e-4 and _rel(b.grad, r2.grad) < 1e-4
    # bitwise reproducible (fixed-order reductions)
    a2, b2 = z1.cuda().requires_grad_(True), z2.cuda().requires_grad_(True)
    out2 = _ops.InfoNCEFn.apply(a2, b2, T)
    (out2 * gout).backward()
    assert out2.item() == out.item() and torch.equal(a2.grad, a.grad)


@pytest.mark.gpu
def test_gpu_infonce_rejects_bad_shapes():
    from VAESNe import _ops
    with pytest.raises(RuntimeError):
        _ops.InfoNCEFn.apply(torch.randn(4, 8, device="cuda"), torch.randn(5, 8, device="cuda"),
                             0.1)
    with pytest.raises(RuntimeError):        # LDS limit: B too large for one row per workgroup
        _ops.InfoNCEFn.apply(torch.randn(20000, 2, device="cuda"),
                             torch.randn(20000, 2, device="cuda"), 0.1)
    with pytest.raises(RuntimeError):        # no CPU path
        _ops.InfoNCEFn.apply(torch.randn(4, 8), torch.randn(4, 8), 0.1)


@pytest.mark.gpu
def test_gpu_contrastive_step_graph_capturable():
    """The contrastive forward + backward has no host synchronisation: captured as a
    hipGraph (as bench.py's extras step) it replays to the eager loss and gradients
    bit for bit (dropout 0, fixed-order reductions)."""
    from VAESNe.losses import negInfoNCE
    g = load_golden("contrast_tiny")
    c = g["config"]
    model = build_contrast_model(c)
    model.train()
    x = golden_x(g, "cuda")
    params = [p for p in model.parameters()]

    def fwd_bwd():
        for p in params:
            p.grad = None
        loss = -negInfoNCE(model, x, temperature=c["T"])
        loss.backward()
        return loss

    ref = fwd_bwd().detach().clone()
    ref_g = [p.grad.clone() for p in params]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fwd_bwd()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    for p in params:
        p.grad = None
    with torch.cuda.graph(graph):
        loss = -negInfoNCE(model, x, temperature=c["T"])
        loss.backward()
    graph.replay()
    torch.cuda.synchronize()
    assert loss.item() == ref.item()
    for p, r in zip(params, ref_g):
        assert torch.equal(p.grad, r)
