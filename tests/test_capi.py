"""CPU-side checks of the drop-in boundary: the C-ABI library exports exactly
what include/vaesne_hip.h declares, the ctypes table matches the header, the
build's modules reproduce the reference's state_dict layout, and the product
path refuses CPU tensors (no CPU fallback)."""
import os
import re

import pytest
import torch

from conftest import ORACLE_CASES, ROOT, build_model, load_golden, oracle_cfg
from oracle import vaesne_oracle as O

HEADER = os.path.join(ROOT, "include", "vaesne_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vaesne_\w+)\s*\(", src)))


def header_arity():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|int64_t)\s+(vaesne_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def test_library_exports_every_header_symbol():
    from VAESNe import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n


def test_ctypes_table_matches_header():
    from VAESNe import _lib
    ar = header_arity()
    assert set(ar) == set(_lib.SIGNATURES), set(ar) ^ set(_lib.SIGNATURES)
    for n, (_, args) in _lib.SIGNATURES.items():
        assert len(args) == ar[n], (n, len(args), ar[n])


@pytest.mark.parametrize("name", ORACLE_CASES)
def test_state_dict_layout_matches_reference(name):
    """Key names and shapes equal the reference module tree (as recorded by
    the oracle's param_shapes, itself checked against the golden grads)."""
    c = load_golden(name)["config"]
    model = build_model(c, device="cpu")
    sd = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    ref = O.param_shapes(oracle_cfg(c))
    assert sd == {k: tuple(v) for k, v in ref.items()}


def test_constructors_accept_script_length_kwargs():
    """cannon/ZTF_photospect.py:89,104 pass spectra_length / photometric_length."""
    from VAESNe.PhotometricVAE import PhotometricVAE
    from VAESNe.SpectraVAE import SpectraVAE
    SpectraVAE(latent_len=4, latent_dim=4, spectra_length=982)
    PhotometricVAE(num_bands=2, latent_len=4, latent_dim=4, model_dim=32, ff_dim=32,
                   photometric_length=60)


def test_cpu_tensors_are_refused():
    from VAESNe.SpectraVAE import SpectraVAE
    m = SpectraVAE(latent_len=4, latent_dim=4, num_layers=1)
    x = (torch.randn(2, 16), torch.linspace(-1, 1, 16).repeat(2, 1), torch.randn(2),
         torch.zeros(2, 16, dtype=torch.bool))
    with pytest.raises(RuntimeError, match="ROCm"):
        m(x, K=1)


def test_param_count_cfg4():
    from VAESNe.PhotometricVAE import PhotometricVAE
    from VAESNe.SpectraVAE import SpectraVAE
    from VAESNe.mmVAE import photospecMMVAE
    p = PhotometricVAE(num_bands=6, latent_len=4, latent_dim=4, model_dim=32, ff_dim=32)
    s = SpectraVAE(latent_len=4, latent_dim=4)
    m = photospecMMVAE([p, s])
    assert sum(x.numel() for x in m.parameters() if x.requires_grad) == 203018
    assert abs(m.vaes[0].llik_scaling - 982 / 60) < 1e-12 and m.vaes[1].llik_scaling == 1.0
