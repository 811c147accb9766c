"""Whole-module pickles written by the REFERENCE (torch.save(model), the form the cannon
scripts save and torch.load: cannon/test_spectra.py:94, try_spectra_model.py:29) load
into this package: the pickle names our classes by module path, its leaf layers are
torch nn.Linear / nn.MultiheadAttention and its sinusoidal embeddings hold a tensor
div_term (util_layers.py:122,138).  util_layers.ReferencePickle re-classes the leaves
and rebuilds the embeddings, so the loaded model IS a build model (same classes, same
state) — the GPU half (test_gpu_parity.py::test_reference_pickle_loss) runs it.

The fixtures tests/golden/pkl_*.pt are our own generated files (gen_golden.py
run_pickle: the reference's filled model of the case), loaded with weights_only=False
because a whole-module pickle cannot be loaded otherwise."""
import io
import os

import pytest
import torch

from conftest import ROOT, build_model, load_golden

PICKLE_CASES = ["mmvae_tiny", "mmvae_tiny_noconcat", "elbo_spec_tiny_K3"]


def load_reference_pickle(name, map_location="cpu"):
    path = os.path.join(ROOT, "tests", "golden", f"pkl_{name}.pt")
    return torch.load(path, map_location=map_location, weights_only=False)


def _same_structure(a, b):
    for (n1, m1), (n2, m2) in zip(a.named_modules(), b.named_modules(), strict=True):
        assert n1 == n2
        assert type(m1) is type(m2), (n1, type(m1), type(m2))
        pub = lambda m: {k for k in m.__dict__ if not k.startswith("_")}
        assert pub(m1) == pub(m2), (n1, pub(m1) ^ pub(m2))
        assert ("_div" in m1.__dict__) == ("_div" in m2.__dict__), n1


@pytest.mark.parametrize("name", PICKLE_CASES)
def test_reference_pickle_loads_as_build_model(name):
    model = load_reference_pickle(name)
    ours = build_model(load_golden(name)["config"], device="cpu")
    _same_structure(model, ours)
    sa, sb = model.state_dict(), ours.state_dict()
    assert list(sa) == list(sb)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for m1, m2 in zip(model.modules(), ours.modules()):
        if "_div" in m2.__dict__:
            assert torch.equal(m1.div_term, m2.div_term)
            assert "div_term" not in m1.__dict__


def test_build_model_pickle_round_trip():
    """torch.save of a build model (as the scripts do after training) loads back with
    the same classes and state; the per-device div_term cache is not pickled."""
    ours = build_model(load_golden("mmvae_tiny")["config"], device="cpu")
    for m in ours.modules():
        if "_div" in m.__dict__:
            m._div._dev["meta"] = torch.empty(0, device="meta")
    buf = io.BytesIO()
    torch.save(ours, buf)
    buf.seek(0)
    back = torch.load(buf, weights_only=False)
    _same_structure(back, ours)
    for m in back.modules():
        if "_div" in m.__dict__:
            assert m._div._dev == {}
    for (k, a), (_, b) in zip(back.state_dict().items(), ours.state_dict().items()):
        assert torch.equal(a, b), k
