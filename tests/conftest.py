import importlib.util
import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "vaesne-dev_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


def _load_fill_rule():
    spec = importlib.util.spec_from_file_location("fill_rule", os.path.join(GOLDEN, "fill_rule.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


fill_rule = _load_fill_rule()


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["config"] = json.loads(str(d["config"]))
    return d


GOLDEN_CASES = ["mmvae_tiny", "mmvae_tiny_noconcat", "mmvae_cfg4", "mmvae_cfg5",
                "elbo_spec_cfg2", "elbo_photo_cfg3", "elbo_spec_tiny_K3"]


def oracle_cfg(c):
    from oracle.vaesne_oracle import MMVAECfg, VaeCfg
    common = dict(latent_len=c["Lz"], latent_dim=c["Dz"], model_dim=32, num_heads=4, ff_dim=32,
                  num_layers=c["layers"], concat=c["concat"])
    if c["kind"] == "mmvae":
        return MMVAECfg(photo=VaeCfg("photo", num_bands=c["nb"], selfattn=False, **common),
                        spec=VaeCfg("spec", selfattn=c["selfattn"], **common), beta=c["beta"])
    if c["kind"] == "spec":
        return VaeCfg("spec", selfattn=c["selfattn"], beta=c["beta"], **common)
    return VaeCfg("photo", num_bands=c["nb"], selfattn=c["selfattn"], beta=c["beta"], **common)


def golden_x(g, device="cpu", dtype=torch.float32):
    c = g["config"]
    f = lambda k: torch.from_numpy(g[k]).to(device)
    fl = lambda k: torch.from_numpy(g[k]).to(device=device, dtype=dtype)
    P = lambda: (fl("pflux"), fl("ptime"), f("pband"), f("pmask"))
    S = lambda: (fl("sflux"), fl("swave"), fl("sphase"), f("smask"))
    if c["kind"] == "mmvae":
        return [P(), S()]
    return S() if c["kind"] == "spec" else P()


def has_gpu():
    return torch.cuda.is_available()


# ---------------------------------------------------------------------------
# the HIP build (package VAESNe under vaesne-dev_amd/)
# ---------------------------------------------------------------------------
def build_model(c, device="cuda", dropout=0.0):
    """The build's model for a golden config, parameters from the fill rule
    (same rule the golden generator applied to the reference)."""
    from VAESNe.PhotometricVAE import PhotometricVAE
    from VAESNe.SpectraVAE import SpectraVAE
    from VAESNe.mmVAE import photospecMMVAE
    common = dict(latent_len=c["Lz"], latent_dim=c["Dz"], model_dim=32, num_heads=4, ff_dim=32,
                  num_layers=c["layers"], dropout=dropout, concat=c["concat"])
    if c["kind"] == "mmvae":
        photo = PhotometricVAE(num_bands=c["nb"], selfattn=False, **common)
        spec = SpectraVAE(selfattn=c["selfattn"], **common)
        model = photospecMMVAE(vaes=[photo, spec], beta=c["beta"])
    elif c["kind"] == "spec":
        model = SpectraVAE(selfattn=c["selfattn"], beta=c["beta"], **common)
    else:
        model = PhotometricVAE(num_bands=c["nb"], selfattn=c["selfattn"], beta=c["beta"], **common)
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        f = fill_rule.fill(k, tuple(v.shape))
        new[k] = v.clone() if f is None else torch.from_numpy(f)
    model.load_state_dict(new)
    return model.to(device)


def golden_us(g):
    return [torch.from_numpy(g[k]) for k in sorted(k for k in g if k.startswith("u") and k[1:].isdigit())]
