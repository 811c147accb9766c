"""the inference paths around the training step, on the GPU.

* photospecMMVAE.reconstruct(data, K) (mmVAE.py:120-126; cannon/try_ZTF_photospect.py:74)
  and VAE.encode(x, mean) (PhotometricVAE.py:179-186, SpectraVAE.py:167-176) against the
  reference's golden vectors (same parameters / inputs / injected noise, dropout off);
* reconstruct at the scripts' K = 100 (batched, eval mode) against the oracle;
* generate (mmVAE.py:108-118, SpectraVAE.py:198-206) against the reference's outputs
  for its recorded prior draws, and shapes / finiteness at other sizes;
* VAEregressionHead (regression.py:9-26) forward/backward against an fp64 restatement
  on the oracle's encoder, with the VAE frozen;
* whole-module torch.save / torch.load round trip of the build's own model
  (the scripts pickle whole modules, cannon/test_photospectra.py:153).
"""
import io
import math

import numpy as np
import pytest
import torch

from conftest import build_model, fill_rule, golden_us, golden_x, load_golden, oracle_cfg
from oracle import vaesne_oracle as O

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a.detach().double().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().double().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("name", ["mmvae_tiny", "mmvae_cfg5"])
def test_reconstruct_and_encode_match_reference(name):
    from VAESNe import rng
    g = load_golden(name)
    c = g["config"]
    model = build_model(c)
    x = golden_x(g, "cuda")
    with rng.inject_uniform(golden_us(g)):
        rec = model.reconstruct(x, K=c["K"])
    for e in range(2):
        for d in range(2):
            assert _rel(rec[e][d], g[f"loc{e}{d}"]) < 1e-4, (e, d)
    for m in range(2):
        mu = model.vaes[m].encode(x[m], True)
        assert _rel(mu, g[f"mu{m}"]) < 1e-5
        q = model.vaes[m].encode(x[m], False)
        assert isinstance(q, torch.distributions.Laplace)
        assert _rel(q.scale, g[f"scale{m}"]) < 1e-5


def test_reconstruct_K100_matches_oracle():
    """The eval scripts' reconstruct(data, K=100) (spect_cond_LC.py:103)."""
    from VAESNe import rng
    g = load_golden("mmvae_tiny")
    c = g["config"]
    model = build_model(c)
    x = golden_x(g, "cuda")
    K = 100
    gen = torch.Generator().manual_seed(3)
    us = [O.draw_u((K, x[0][0].shape[0], c["Lz"], c["Dz"]), generator=gen) for _ in range(2)]
    with rng.inject_uniform(us):
        rec = model.reconstruct(x, K=K)
    p = O.make_params(oracle_cfg(c), fill_rule.fill)
    with torch.no_grad():
        _, px, _ = O.mmvae_forward(p, oracle_cfg(c), golden_x(g, "cpu"), K, us)
    for e in range(2):
        for d in range(2):
            assert rec[e][d].shape == px[e][d].loc.shape
            assert _rel(rec[e][d], px[e][d].loc) < 1e-4, (e, d)


@pytest.mark.parametrize("name", ["mmvae_tiny", "mmvae_cfg5"])
def test_generate_matches_reference(name):
    """photospecMMVAE.generate(N, x) (mmVAE.py:108-118: ONE prior draw [N, B, Lz, Dz]
    decoded by both modalities) and SpectraVAE.generate(N, x1) (SpectraVAE.py:198-206:
    draws [N, 1, Lz, Dz], one conditioning spectrum) against the reference's outputs for
    its recorded uniform draws (tests/golden/gen_*.npz)."""
    from VAESNe import rng
    g = load_golden("gen_" + name)
    c = g["config"]
    model = build_model(c)
    model.train()                         # generate() switches to eval itself
    x = golden_x(load_golden(name), "cuda")
    N = int(g["N"])
    with rng.inject_uniform([torch.from_numpy(g["u_gen"])]):
        gen = model.generate(N, x)
    assert not model.training
    for d in range(2):
        assert tuple(gen[d].shape) == g[f"gen{d}"].shape
        assert _rel(gen[d], g[f"gen{d}"]) < 1e-4, d
    with rng.inject_uniform([torch.from_numpy(g["u_sgen"])]):
        s = model.vaes[1].generate(N, tuple(t[:1] for t in x[1]))
    assert tuple(s.shape) == g["sgen"].shape and _rel(s, g["sgen"]) < 1e-4


def test_generate_shapes_and_scales():
    g = load_golden("mmvae_tiny")
    c = g["config"]
    model = build_model(c)
    x = golden_x(g, "cuda")
    out = model.generate(5, x)
    B = x[0][0].shape[0]
    assert out[0].shape == (5, B, x[0][0].shape[1]) and out[1].shape == (5, B, x[1][0].shape[1])
    assert all(torch.isfinite(o).all() for o in out)
    spec = model.vaes[1]     # SpectraVAE.generate (SpectraVAE.py:198-206): one grid, N prior draws
    x1 = tuple(t[:1] for t in x[1])
    s = spec.generate(3, x1)
    assert s.shape == (1, 3, 1, x[1][0].shape[1]) and torch.isfinite(s).all()


def test_regression_head_matches_fp64_restatement():
    from VAESNe.regression import VAEregressionHead
    from VAESNe.util_layers import MLP
    g = load_golden("mmvae_tiny")
    c = g["config"]
    model = build_model(c)
    x = golden_x(g, "cuda")
    torch.manual_seed(0)
    head = VAEregressionHead(model.vaes[0], outdim=3, MLPlatent=[16, 16]).cuda()
    assert not any(p.requires_grad for p in model.vaes[0].parameters())
    y = head(x[0])
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    # fp64 restatement: oracle encoder mean -> MLP (Linear-ReLU-Linear-ReLU-Linear)
    p = O.make_params(oracle_cfg(c), fill_rule.fill, dtype=torch.float64)
    xc = [tuple(t.double() if t.is_floating_point() else t for t in m) for m in golden_x(g, "cpu")]
    mu, _ = O.encode(p, "vaes.0.", oracle_cfg(c).photo, xc[0])
    h = mu.reshape(mu.shape[0], -1)
    ws = {k: v.detach().double().cpu().requires_grad_(True) for k, v in head.outfc.state_dict().items()}
    r = torch.relu(h @ ws["mlp.0.weight"].T + ws["mlp.0.bias"])
    r = torch.relu(r @ ws["mlp.2.weight"].T + ws["mlp.2.bias"])
    r = r @ ws["mlp.4.weight"].T + ws["mlp.4.bias"]
    (r * gy.double().cpu()).sum().backward()
    assert _rel(y, r) < 1e-4
    for k, prm in head.outfc.named_parameters():
        assert _rel(prm.grad, ws[k].grad) < 1e-4, k


def test_whole_module_save_load_roundtrip():
    from VAESNe import rng
    g = load_golden("mmvae_tiny")
    c = g["config"]
    model = build_model(c)
    buf = io.BytesIO()
    torch.save(model, buf)               # whole-module pickle, as the scripts do
    buf.seek(0)
    m2 = torch.load(buf, weights_only=False)   # our own file
    assert type(m2).__module__ == "VAESNe.mmVAE" and type(m2).__name__ == "photospecMMVAE"
    x = golden_x(g, "cuda")
    us = golden_us(g)
    with torch.no_grad(), rng.inject_uniform(us):
        a = model.reconstruct(x, K=c["K"])
    with torch.no_grad(), rng.inject_uniform(us):
        b = m2.reconstruct(x, K=c["K"])
    for e in range(2):
        for d in range(2):
            assert torch.equal(a[e][d], b[e][d])
