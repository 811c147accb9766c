"""Pin the CPU oracle (oracle/vaesne_oracle.py) to the golden fixtures that
tests/golden/gen_golden.py produced by running the reference package."""
import json

import numpy as np
import pytest
import torch

from conftest import ORACLE_CASES, fill_rule, golden_x, load_golden, oracle_cfg
from oracle import vaesne_oracle as O


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _loss(g, cfg, p, x, us):
    c = g["config"]
    if c["kind"] == "mmvae":
        val, lw, aux = O.m_iwae(p, cfg, x, c["K"], us)
        return -val, lw, aux
    val, aux = O.elbo(p, cfg, x, c["K"], us[0])
    return -val, None, aux


@pytest.mark.parametrize("name", ORACLE_CASES)
def test_oracle_forward_and_grads(name):
    g = load_golden(name)
    c = g["config"]
    cfg = oracle_cfg(c)
    p = O.make_params(cfg, fill_rule.fill, requires_grad=True)
    x = golden_x(g)
    us = [torch.from_numpy(g[k]) for k in sorted(k for k in g if k.startswith("u") and k[1:].isdigit())]
    loss, lw, aux = _loss(g, cfg, p, x, us)
    assert abs(loss.item() - float(g["loss"])) / abs(float(g["loss"])) < 1e-6
    if c["kind"] == "mmvae":
        assert _rel(lw.detach(), g["lw"]) < 1e-5
        qz, px, zss = aux
        for m in range(2):
            assert _rel(qz[m].loc.detach(), g[f"mu{m}"]) < 1e-5
            assert _rel(qz[m].scale.detach(), g[f"scale{m}"]) < 1e-5
            assert _rel(zss[m].detach(), g[f"zs{m}"]) < 1e-5
            for d in range(2):
                assert _rel(px[m][d].loc.detach(), g[f"loc{m}{d}"]) < 1e-5
                np.testing.assert_array_equal(px[m][d].scale.detach().numpy(), g[f"pxscale{m}{d}"])
    else:
        q, pxz, zs = aux
        assert _rel(q.loc.detach(), g["mu0"]) < 1e-5
        assert _rel(q.scale.detach(), g["scale0"]) < 1e-5
        assert _rel(pxz.loc.detach(), g["loc00"]) < 1e-5
    loss.backward()
    names = json.loads(str(g["grad_names"]))
    norms = g["grad_norms"]
    for k, n in zip(names, norms):
        gk = p[k].grad
        assert gk is not None, k
        assert abs(gk.norm().item() - n) <= 1e-4 * max(n, 1e-3), (k, gk.norm().item(), n)
        if ("grad:" + k) in g:
            assert _rel(gk, g["grad:" + k]) < 1e-4, k


@pytest.mark.parametrize("name", ["mmvae_tiny", "elbo_photo_cfg3", "mmvae_tiny_noconcat"])
def test_oracle_adamw_trajectory(name):
    g = load_golden(name)
    c = g["config"]
    cfg = oracle_cfg(c)
    p = O.make_params(cfg, fill_rule.fill, requires_grad=True)
    x = golden_x(g)
    st = O.AdamWState(lr=1e-3)
    n_u = 2 if c["kind"] == "mmvae" else 1
    for s, ref in enumerate(g["traj_losses"]):
        us = [torch.from_numpy(g[f"traj_u{s}_{i}"]) for i in range(n_u)]
        for v in p.values():
            v.grad = None
        loss, _, _ = _loss(g, cfg, p, x, us)
        loss.backward()
        assert abs(loss.item() - ref) / abs(ref) < 1e-5, (s, loss.item(), ref)
        O.adamw_step(p, {k: v.grad for k, v in p.items() if v.requires_grad}, st)
    ref_norms = json.loads(str(g["traj_param_norms"]))
    for k, n in ref_norms.items():
        if k.endswith("in_proj_bias"):
            # the key-bias slice has an analytically zero gradient (softmax is
            # shift invariant per query); Adam normalises its rounding noise to
            # +-lr steps, so it is chaotic in any implementation.  Skipped.
            continue
        assert abs(p[k].detach().norm().item() - n) <= 1e-5 * max(n, 1.0), k


@pytest.mark.parametrize("name", ["mmvae_tiny", "mmvae_cfg5"])
def test_oracle_generate_matches_reference(name):
    """photospecMMVAE.generate (mmVAE.py:108-118) and SpectraVAE.generate
    (SpectraVAE.py:198-206) with the reference's recorded prior draws."""
    g = load_golden("gen_" + name)
    c = g["config"]
    cfg = oracle_cfg(c)
    p = O.make_params(cfg, fill_rule.fill)
    x = golden_x(load_golden(name))
    N = int(g["N"])
    with torch.no_grad():
        gen = O.mmvae_generate(p, cfg, x, N, torch.from_numpy(g["u_gen"]))
        sgen = O.spectra_generate(p, "vaes.1.", cfg.spec, tuple(t[:1] for t in x[1]), N,
                                  torch.from_numpy(g["u_sgen"]))
    for d in range(2):
        assert gen[d].shape == g[f"gen{d}"].shape
        assert _rel(gen[d], g[f"gen{d}"]) < 1e-5, d
    assert sgen.shape == g["sgen"].shape and _rel(sgen, g["sgen"]) < 1e-5
