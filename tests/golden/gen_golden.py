"""Generate golden fixtures by running the REFERENCE VAESNe package on CPU.

Run (this container only; /root/reference does not exist on the GPU box):
    cd /tmp && PYTHONPATH=/root/reference/package PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_golden.py /root/repo/tests/golden

The reference is imported from its read-only tree and never copied; only the
numbers it produces are written (small .npz fixtures, inputs + outputs).
``/root/repo`` must NOT be on sys.path (the build is also called VAESNe).

Determinism recipe: every module is built with dropout=0,
so one loss evaluation consumes exactly one uniform draw per VAE
(Laplace.rsample, torch/distributions/laplace.py:83), photometry first.  We
record those draws by re-seeding and replaying them, so the oracle and the
HIP build can inject the identical noise.
"""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
assert not any(os.path.abspath(p) == "/root/repo" for p in sys.path if p), "repo on sys.path"

spec = importlib.util.spec_from_file_location("fill_rule", os.path.join(HERE, "fill_rule.py"))
fill_rule = importlib.util.module_from_spec(spec)
spec.loader.exec_module(fill_rule)

from VAESNe.PhotometricVAE import PhotometricVAE, BrightPhotometricVAE  # noqa: E402  (reference)
from VAESNe.SpectraVAE import SpectraVAE, BrightSpectraVAE              # noqa: E402
from VAESNe.ImageVAE import HostImgVAE                                  # noqa: E402
from VAESNe.mmVAE import photospecMMVAE           # noqa: E402
from VAESNe.losses import m_iwae, _m_iwae, elbo   # noqa: E402

torch.set_num_threads(8)

CASES = {
    # name: kind, sizes, model kwargs
    "mmvae_tiny": dict(kind="mmvae", B=2, K=2, Lp=16, Ls=128, nb=6, layers=1, Lz=4, Dz=4,
                       beta=1.0, selfattn=False, concat=True, steps=3),
    "mmvae_tiny_noconcat": dict(kind="mmvae", B=2, K=3, Lp=12, Ls=64, nb=3, layers=2, Lz=4, Dz=2,
                                beta=0.7, selfattn=True, concat=False, steps=2),
    "mmvae_cfg4": dict(kind="mmvae", B=4, K=2, Lp=60, Ls=982, nb=6, layers=4, Lz=4, Dz=4,
                       beta=1.0, selfattn=False, concat=True, steps=3),
    "mmvae_cfg5": dict(kind="mmvae", B=2, K=8, Lp=60, Ls=982, nb=2, layers=4, Lz=4, Dz=4,
                       beta=0.5, selfattn=True, concat=True, steps=2),
    "elbo_spec_cfg2": dict(kind="spec", B=4, K=1, Ls=982, layers=4, Lz=4, Dz=4, beta=1.0,
                           selfattn=False, concat=True, steps=3),
    "elbo_photo_cfg3": dict(kind="photo", B=4, K=1, Lp=60, nb=2, layers=4, Lz=4, Dz=2, beta=0.5,
                            selfattn=False, concat=True, steps=3),
    "elbo_spec_tiny_K3": dict(kind="spec", B=3, K=3, Ls=50, layers=2, Lz=4, Dz=3, beta=2.0,
                              selfattn=True, concat=True, steps=2),
    # the exact benchmarked configuration (bench.py: cannon/ZTF_photospect.py per GPU)
    "mmvae_cfg5_b16": dict(kind="mmvae", B=16, K=8, Lp=60, Ls=982, nb=2, layers=4, Lz=4, Dz=4,
                           beta=0.5, selfattn=True, concat=True, steps=1),
    # Bright* VAEs (PhotometricVAE.py:226-355, SpectraVAE.py:211-332)
    "mmvae_bright": dict(kind="mmvae", bright=True, B=3, K=2, Lp=60, Ls=982, nb=2, layers=2, Lz=4,
                         Dz=4, beta=0.5, selfattn=True, concat=True, steps=2),
    "elbo_bright_spec": dict(kind="spec", bright=True, B=3, K=2, Ls=300, layers=2, Lz=4, Dz=3,
                             beta=1.0, selfattn=False, concat=True, steps=2),
    "elbo_bright_photo": dict(kind="photo", bright=True, B=4, K=1, Lp=60, nb=6, layers=2, Lz=4,
                              Dz=2, beta=0.5, selfattn=False, concat=True, steps=2),
    # BASELINE config 1: cannon/mnist.py HostImgVAE (host path), B=2 of its B=32
    "image_cfg1": dict(kind="image", B=2, K=1, img=60, C=1, patch=3, layers=4, Lz=4, Dz=4,
                       beta=0.1, selfattn=False, steps=2),
}

# Reference-initialised checkpoints: the model built right after torch.manual_seed(0)
# exactly as a script does (no parameter fill), its state_dict saved with
# torch.save (tensors only, loadable with weights_only=True), plus the loss of that
# model on the case's inputs / noise.
CKPT_CASES = ["mmvae_cfg5", "mmvae_bright", "image_cfg1"]

FULL_GRAD_SUFFIXES = [
    "dec.generativetransformer.transformerblocks.0.self_attn.in_proj_weight",
    "dec.generativetransformer.transformerblocks.0.layernorm1.weight",
    "dec.generativetransformer.get_flux.fc2.weight",
    "dec.generativetransformer.get_photo.fc2.weight",
    "enc.inference_transformer.initbottleneck",
    "enc.inference_transformer.transformerblocks.0.cross_attn.out_proj.weight",
    "enc.inference_transformer.bandembd.weight",
    "dec.generativetransformer.bandembd.weight",
    "brightnessfc.mlp.0.weight",
    "brightnessfc.mlp.2.bias",
    "enc.inference_transformer.patch_embed.proj.weight",
    "dec.generativetransformer.final_refine.0.weight",
    "dec.generativetransformer.final_refine.2.weight",
    "dec.generativetransformer.decoder.weight",
]


def construct(c):
    """The reference model for config c (random init; dropout 0)."""
    if c["kind"] == "image":
        return HostImgVAE(img_size=c["img"], latent_len=c["Lz"], latent_dim=c["Dz"],
                          patch_size=c["patch"], in_channels=c["C"], focal_loc=False, model_dim=32,
                          num_heads=4, ff_dim=32, num_layers=c["layers"], dropout=0.0,
                          selfattn=c["selfattn"], beta=c["beta"])
    common = dict(latent_len=c["Lz"], latent_dim=c["Dz"], model_dim=32, num_heads=4, ff_dim=32,
                  num_layers=c["layers"], dropout=0.0)
    bright = c.get("bright", False)
    if bright:
        assert c["concat"], "Bright* VAEs build their encoders with concat=True"
        P, S = BrightPhotometricVAE, BrightSpectraVAE
    else:
        common["concat"] = c["concat"]
        P, S = PhotometricVAE, SpectraVAE
    if c["kind"] == "mmvae":
        photo = P(num_bands=c["nb"], selfattn=False, **common)
        specv = S(selfattn=c["selfattn"], **common)
        return photospecMMVAE(vaes=[photo, specv], beta=c["beta"])
    if c["kind"] == "spec":
        return S(selfattn=c["selfattn"], beta=c["beta"], **common)
    return P(num_bands=c["nb"], selfattn=c["selfattn"], beta=c["beta"], **common)


def build(c):
    model = construct(c)
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        f = fill_rule.fill(k, tuple(v.shape))
        new[k] = v.clone() if f is None else torch.from_numpy(f)
    model.load_state_dict(new)
    model.train()
    return model


def inputs(c, seed=1234):
    rng = np.random.default_rng(seed)
    out = {}
    if c["kind"] in ("mmvae", "photo"):
        f, t, b, m = fill_rule.photo_inputs(rng, c["B"], c["Lp"], c["nb"])
        out.update(pflux=f, ptime=t, pband=b, pmask=m)
    if c["kind"] in ("mmvae", "spec"):
        f, w, ph, m = fill_rule.spec_inputs(rng, c["B"], c["Ls"])
        out.update(sflux=f, swave=w, sphase=ph, smask=m)
    if c["kind"] == "image":
        img, label = fill_rule.image_inputs(rng, c["B"], c["C"], c["img"])
        out.update(image=img, label=label)
    return out


def to_x(c, arr):
    P = lambda: (torch.from_numpy(arr["pflux"]), torch.from_numpy(arr["ptime"]),
                 torch.from_numpy(arr["pband"]), torch.from_numpy(arr["pmask"]))
    S = lambda: (torch.from_numpy(arr["sflux"]), torch.from_numpy(arr["swave"]),
                 torch.from_numpy(arr["sphase"]), torch.from_numpy(arr["smask"]))
    if c["kind"] == "image":
        return (torch.from_numpy(arr["image"]), torch.from_numpy(arr["label"]))
    if c["kind"] == "mmvae":
        return [P(), S()]
    return S() if c["kind"] == "spec" else P()


def draws(c, seed):
    """Replay the uniform draws a loss evaluation consumes after manual_seed(seed)."""
    torch.manual_seed(seed)
    eps = torch.finfo(torch.float32).eps
    shape = (c["K"], c["B"], c["Lz"], c["Dz"])
    n = 2 if c["kind"] == "mmvae" else 1
    return [torch.empty(shape).uniform_(eps - 1, 1) for _ in range(n)]


def loss_fn(c, model, x):
    if c["kind"] == "mmvae":
        return m_iwae(model, x, K=c["K"])
    return elbo(model, x, K=c["K"])


def run_ckpt(name, c, outdir):
    """ckpt_<name>.pt: state_dict of the reference model constructed after
    torch.manual_seed(0) (default init); ckpt_<name>.npz: its loss on the case's
    inputs with injected noise."""
    torch.manual_seed(0)
    model = construct(c)
    model.train()
    torch.save(model.state_dict(), os.path.join(outdir, f"ckpt_{name}.pt"))
    x = to_x(c, inputs(c))
    seed0 = 11
    out = {f"u{i}": u.numpy() for i, u in enumerate(draws(c, seed0))}
    torch.manual_seed(seed0)
    with torch.no_grad():
        loss = -loss_fn(c, model, x)
    out["loss"] = np.array(loss.item(), dtype=np.float64)
    out["config"] = np.array(json.dumps(c))
    np.savez_compressed(os.path.join(outdir, f"ckpt_{name}.npz"), **out)
    print(f"ckpt_{name}: loss={loss.item():.6f}")


def run_case(name, c, outdir):
    model = build(c)
    arr = inputs(c)
    x = to_x(c, arr)
    out = dict(arr)
    out["config"] = np.array(json.dumps(c))
    seed0 = 7
    us = draws(c, seed0)
    for i, u in enumerate(us):
        out[f"u{i}"] = u.numpy()

    # forward pieces
    torch.manual_seed(seed0)
    with torch.no_grad():
        if c["kind"] == "mmvae":
            qz, px, zss = model(x, K=c["K"])
            for m in range(2):
                out[f"mu{m}"] = qz[m].loc.numpy()
                out[f"scale{m}"] = qz[m].scale.numpy()
                out[f"zs{m}"] = zss[m].numpy()
                for d in range(2):
                    out[f"loc{m}{d}"] = px[m][d].loc.numpy()
                    out[f"pxscale{m}{d}"] = px[m][d].scale.numpy()
            torch.manual_seed(seed0)
            out["lw"] = _m_iwae(model, x, K=c["K"]).numpy()
        elif c["kind"] == "image":
            q, pxz, zs = model(x, K=c["K"])
            out["mu0"], out["scale0"], out["zs0"] = q.loc.numpy(), q.scale.numpy(), zs.numpy()
            out["loc00"] = pxz.loc.numpy()
        else:
            q, pxz, zs = model(x, K=c["K"])
            out["mu0"], out["scale0"], out["zs0"] = q.loc.numpy(), q.scale.numpy(), zs.numpy()
            out["loc00"], out["pxscale00"] = pxz.loc.numpy(), pxz.scale.numpy()
    # value + gradient
    torch.manual_seed(seed0)
    loss = -loss_fn(c, model, x)
    loss.backward()
    out["loss"] = np.array(loss.item(), dtype=np.float64)
    names, norms = [], []
    for k, prm in model.named_parameters():
        if prm.grad is None:
            continue
        names.append(k)
        norms.append(prm.grad.norm().item())
        if any(k.endswith(s) for s in FULL_GRAD_SUFFIXES) or name == "mmvae_tiny":
            out["grad:" + k] = prm.grad.numpy().copy()
    out["grad_names"] = np.array(json.dumps(names))
    out["grad_norms"] = np.array(norms, dtype=np.float64)

    # AdamW trajectory from the filled params (fresh model)
    model = build(c)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    losses = []
    for s in range(c["steps"]):
        seed = 100 + s
        for i, u in enumerate(draws(c, seed)):
            out[f"traj_u{s}_{i}"] = u.numpy()
        torch.manual_seed(seed)
        opt.zero_grad()
        loss = -loss_fn(c, model, x)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    out["traj_losses"] = np.array(losses, dtype=np.float64)
    pn = {k: v.norm().item() for k, v in model.state_dict().items()}
    out["traj_param_norms"] = np.array(json.dumps(pn))
    path = os.path.join(outdir, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: loss={out['loss']:.6f} traj={losses} -> {path}")


# §8(f) 1: generation from the prior (mmVAE.py:108-118, SpectraVAE.py:198-206); each
# consumes ONE uniform draw (Laplace.rsample of the prior), recorded by replay.
GEN_CASES = ["mmvae_tiny", "mmvae_cfg5"]


def run_generate(name, c, outdir, N=3):
    """gen_<name>.npz: photospecMMVAE.generate(N, x) (prior draws [N, B, Lz, Dz] decoded
    by both modalities) and SpectraVAE.generate(N, x1[:1]) (draws [N, 1, Lz, Dz]; the
    reference's decode needs a single conditioning spectrum there) of the filled model."""
    model = build(c)
    x = to_x(c, inputs(c))
    eps = torch.finfo(torch.float32).eps
    out = {"config": np.array(json.dumps(c)), "N": np.array(N)}
    B = x[0][0].shape[0]
    torch.manual_seed(21)
    out["u_gen"] = torch.empty(N, B, c["Lz"], c["Dz"]).uniform_(eps - 1, 1).numpy()
    torch.manual_seed(21)
    gen = model.generate(N, x)
    out["gen0"], out["gen1"] = gen[0].numpy(), gen[1].numpy()
    x1 = tuple(t[:1] for t in x[1])
    torch.manual_seed(22)
    out["u_sgen"] = torch.empty(N, 1, c["Lz"], c["Dz"]).uniform_(eps - 1, 1).numpy()
    torch.manual_seed(22)
    out["sgen"] = model.vaes[1].generate(N, x1).numpy()
    path = os.path.join(outdir, f"gen_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"gen_{name}: gen0 {out['gen0'].shape} gen1 {out['gen1'].shape} "
          f"sgen {out['sgen'].shape} -> {path}")


# Whole-module pickles (torch.save(model), the form photometry2goldstein_mmvae.py:36-37
# and the other cannon scripts load): the filled reference model of the case, so its
# loss is the case's recorded `loss` (seed 7 noise u0/u1).  Loading them executes
# pickle code, so they are our own generated files, loaded only by tests.
PICKLE_CASES = ["mmvae_tiny", "mmvae_tiny_noconcat", "elbo_spec_tiny_K3"]


def run_pickle(name, c, outdir):
    model = build(c)
    path = os.path.join(outdir, f"pkl_{name}.pt")
    torch.save(model, path)
    print(f"pkl_{name}: whole-module pickle of {type(model).__name__} -> {path}")


if __name__ == "__main__":
    outdir = sys.argv[1] if len(sys.argv) > 1 else HERE
    only = sys.argv[2:]
    for name, c in CASES.items():
        if only and name not in only:
            continue
        run_case(name, c, outdir)
    for name in CKPT_CASES:
        if only and ("ckpt_" + name) not in only:
            continue
        run_ckpt(name, CASES[name], outdir)
    for name in GEN_CASES:
        if only and ("gen_" + name) not in only:
            continue
        run_generate(name, CASES[name], outdir)
    for name in PICKLE_CASES:
        if only and ("pkl_" + name) not in only:
            continue
        run_pickle(name, CASES[name], outdir)
