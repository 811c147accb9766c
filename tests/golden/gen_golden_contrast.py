"""Golden fixtures for the contrastive pretraining and regression heads (§8(f) row 4),
made by running the REFERENCE VAESNe package on CPU.

Run (this container only; /root/reference does not exist on the GPU box):
    cd /tmp && PYTHONPATH=/root/reference/package PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_golden_contrast.py /root/repo/tests/golden

Same rules as gen_golden.py: parameters from fill_rule.fill by state_dict key,
inputs from fill_rule's synthetic recipes, dropout 0, only numbers written.
Cases:
  contrast_*  ContraPhotSpec (contrastiveNets.py:20-101) + negInfoNCE
              (losses.py:98-110): projections, loss, every parameter gradient,
              an AdamW trajectory, and contras{photo,spec}regressionHead outputs.
  end2end_*   {photo,spec}end2endregression (regression.py:69-144): outputs and
              every parameter gradient of an MSE loss against a fixed target.
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

from VAESNe.contrastiveNets import ContraPhotSpec  # noqa: E402  (reference package)
from VAESNe.losses import negInfoNCE               # noqa: E402
from VAESNe.regression import (contrasphotoregressionHead, contrasspecregressionHead,  # noqa: E402
                               photoend2endregression, specend2endregression)

torch.set_num_threads(8)

CASES = {
    "contrast_tiny": dict(kind="contrast", B=6, Lp=16, Ls=64, nb=3, layers=2, Lz=4, Dz=4, proj=8,
                          selfattn=False, T=0.1, steps=2),
    "contrast_selfattn": dict(kind="contrast", B=5, Lp=12, Ls=50, nb=2, layers=1, Lz=2, Dz=3,
                              proj=5, selfattn=True, T=0.07, steps=2),
    "end2end_photo": dict(kind="end2end_photo", B=4, Lp=20, nb=2, layers=2, Lz=4, Dz=4, out=3,
                          hidden=[16, 16], selfattn=False),
    "end2end_spec": dict(kind="end2end_spec", B=3, Ls=70, layers=2, Lz=4, Dz=2, out=2,
                         hidden=[8, 8, 8], selfattn=True),
}


def fill(model):
    new = {}
    for k, v in model.state_dict().items():
        f = fill_rule.fill(k, tuple(v.shape))
        new[k] = v.clone() if f is None else torch.from_numpy(f)
    model.load_state_dict(new)
    model.train()
    return model


def build(c):
    if c["kind"] == "contrast":
        return fill(ContraPhotSpec(
            latent_len=c["Lz"], latent_dim=c["Dz"], proj_dim=c["proj"], num_bands=c["nb"],
            photo_model_dim=32, photo_num_heads=4, photo_ff_dim=32, photo_num_layers=c["layers"],
            photo_dropout=0.0, spec_model_dim=32, spec_num_heads=4, spec_num_layers=c["layers"],
            spec_ff_dim=32, spec_dropout=0.0, selfattn=c["selfattn"]))
    if c["kind"] == "end2end_photo":
        return fill(photoend2endregression(c["out"], num_bands=c["nb"], latent_len=c["Lz"],
                                           latent_dim=c["Dz"], num_layers=c["layers"],
                                           dropout=0.0, selfattn=c["selfattn"],
                                           MLPlatent=c["hidden"]))
    return fill(specend2endregression(c["out"], latent_len=c["Lz"], latent_dim=c["Dz"],
                                      num_layers=c["layers"], dropout=0.0,
                                      selfattn=c["selfattn"], MLPlatent=c["hidden"]))


def inputs(c, seed=1234):
    rng = np.random.default_rng(seed)
    out = {}
    if c["kind"] in ("contrast", "end2end_photo"):
        f, t, b, m = fill_rule.photo_inputs(rng, c["B"], c["Lp"], c["nb"])
        out.update(pflux=f, ptime=t, pband=b, pmask=m)
    if c["kind"] in ("contrast", "end2end_spec"):
        f, w, ph, m = fill_rule.spec_inputs(rng, c["B"], c["Ls"])
        out.update(sflux=f, swave=w, sphase=ph, smask=m)
    return out


def to_x(c, arr):
    P = tuple(torch.from_numpy(arr[k]) for k in ("pflux", "ptime", "pband", "pmask")) \
        if "pflux" in arr else None
    S = tuple(torch.from_numpy(arr[k]) for k in ("sflux", "swave", "sphase", "smask")) \
        if "sflux" in arr else None
    if c["kind"] == "contrast":
        return [P, S]
    return P if c["kind"] == "end2end_photo" else S


def grads(model, out, prefix="grad:"):
    names = []
    for k, prm in model.named_parameters():
        if prm.grad is not None:
            names.append(k)
            out[prefix + k] = prm.grad.numpy().copy()
    out["grad_names"] = np.array(json.dumps(names))


def run_case(name, c, outdir):
    arr = inputs(c)
    x = to_x(c, arr)
    out = dict(arr)
    out["config"] = np.array(json.dumps(c))
    model = build(c)
    if c["kind"] == "contrast":
        with torch.no_grad():
            z1, z2 = model(x)
        out["z1"], out["z2"] = z1.numpy(), z2.numpy()
        loss = -negInfoNCE(model, x, temperature=c["T"])   # training_step's sign
        loss.backward()
        out["loss"] = np.array(loss.item(), dtype=np.float64)
        grads(model, out)
        # frozen-encoder regression heads on the same (filled) network
        torch.manual_seed(3)
        for nm, cls, xx in (("photohead", contrasphotoregressionHead, x[0]),
                            ("spechead", contrasspecregressionHead, x[1])):
            net = build(c)
            head = cls(net, outdim=3, MLPlatent=[16, 16])
            for k, v in head.outfc.state_dict().items():
                out[f"{nm}:{k}"] = v.numpy().copy()
            with torch.no_grad():
                out[f"{nm}_y"] = head(xx).numpy()
        # AdamW trajectory (lr as cannon/test_photospectra_contrast.py:91)
        model = build(c)
        opt = torch.optim.AdamW(model.parameters(), lr=2.5e-4)
        losses = []
        for _ in range(c["steps"]):
            opt.zero_grad()
            loss = -negInfoNCE(model, x, temperature=c["T"])
            loss.backward()
            opt.step()
            losses.append(loss.item())
        out["traj_losses"] = np.array(losses, dtype=np.float64)
    else:
        y = model(x)
        tgt = np.random.default_rng(99).standard_normal(tuple(y.shape)).astype(np.float32)
        out["target"] = tgt
        out["y"] = y.detach().numpy()
        loss = torch.nn.MSELoss()(y, torch.from_numpy(tgt))   # spec2goldstein_end2end.py:77
        loss.backward()
        out["loss"] = np.array(loss.item(), dtype=np.float64)
        grads(model, out)
    path = os.path.join(outdir, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: loss={float(out['loss']):.6f} -> {path}")


if __name__ == "__main__":
    outdir = sys.argv[1] if len(sys.argv) > 1 else HERE
    only = sys.argv[2:]
    for name, c in CASES.items():
        if only and name not in only:
            continue
        run_case(name, c, outdir)
