"""training_step's captured steps (VAESNe._stepgraph) against the eager loop.

The script's literal loop (cannon/ZTF_photospect.py:119-128: training_step with
torch.optim.AdamW over a DataLoader of multimodalDataset batches, m_iwae K=8, dropout
0.1) runs twice from the same initial state: every batch eager (_config.step_graph
off) and with the forward + backward captured after two warm-up batches and replayed.
Each batch draws its noise and dropout masks under the same call ids and device
counter either way, so parameters and losses must agree BITWISE -- including the
ragged last batch of an epoch (a second signature), a loss function whose
closure value changes between epochs (a new capture), and a loss function that
cannot be captured (it synchronises: it falls back to eager)."""
import os
import sys

import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(graph, monkeypatch, epochs=3, fn_of_epoch=None, B=4, n=11):
    sys.path.insert(0, ROOT)
    import bench
    from VAESNe import _config, _stepgraph, rng
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    from VAESNe.training_util import training_step
    monkeypatch.setattr(_config, "step_graph", graph)
    torch.manual_seed(0)
    model = bench.make_model(DEV, 0.1)
    rng.manual_seed(99)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    x = bench.synthetic_batch(n, 7, "cpu")            # 11 pairs: batches of 4, 4, 3
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=B, shuffle=False)
    losses = []
    for ep in range(epochs):
        fn = fn_of_epoch(ep) if fn_of_epoch else (lambda m, xx: m_iwae(m, xx, K=3))
        losses.append(training_step(model, opt, loader, loss_fn=fn, multimodal=True))
    torch.cuda.synchronize()
    graphs = len(_stepgraph._CACHE.get(model, {}))
    n_captured = sum(e.graph is not None for e in _stepgraph._CACHE.get(model, {}).values())
    params = [p.detach().clone() for p in model.parameters()]
    _stepgraph.clear()
    return params, losses, graphs, n_captured


def _same(a, b):
    pa, la = a[0], a[1]
    pb, lb = b[0], b[1]
    assert la == lb, (la, lb)
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


def test_captured_training_step_bitwise_equals_eager(monkeypatch):
    eager = _run(False, monkeypatch)
    graph = _run(True, monkeypatch)
    _same(eager, graph)
    assert eager[3] == 0
    # batches of 4 and the ragged 3: two signatures, both captured by epoch 3
    assert graph[2] == 2 and graph[3] == 2


def test_closure_change_recaptures(monkeypatch):
    from VAESNe.losses import m_iwae

    def fn_of_epoch(ep):
        K = 2 if ep < 2 else 3            # a script changing K between epochs
        return lambda m, xx: m_iwae(m, xx, K=K)
    eager = _run(False, monkeypatch, epochs=4, fn_of_epoch=fn_of_epoch)
    graph = _run(True, monkeypatch, epochs=4, fn_of_epoch=fn_of_epoch)
    _same(eager, graph)
    assert graph[2] == 3                   # K=2 (4 and 3 pairs) + K=3 (4 pairs)


def test_uncapturable_loss_runs_eagerly(monkeypatch):
    from VAESNe.losses import m_iwae

    def fn_of_epoch(ep):
        def fn(m, xx):
            loss = m_iwae(m, xx, K=3)
            if not torch.isfinite(loss).item():      # a host sync: not capturable
                raise RuntimeError("non-finite")
            return loss
        return fn
    eager = _run(False, monkeypatch, fn_of_epoch=fn_of_epoch)
    graph = _run(True, monkeypatch, fn_of_epoch=fn_of_epoch)
    _same(eager, graph)
    assert graph[3] == 0
