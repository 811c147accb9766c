"""The captured-step signature of training_step (VAESNe._stepgraph), on the CPU: what
makes two batches replay the same hipGraph and what forces a new capture."""
import os

import torch
from torch import nn

from VAESNe import _stepgraph as SG


def _fn(K):
    return lambda m, x: (m, x, K)


GLOBAL_K = 8


def _uses_global(m, x):
    return (m, x, GLOBAL_K)


def test_closure_values_and_code_key_the_loss_function():
    a, b, c = _fn(2), _fn(2), _fn(3)
    assert a is not b
    assert SG._fn_key(a) == SG._fn_key(b)          # a new lambda per epoch, same K: same graph
    assert SG._fn_key(a) != SG._fn_key(c)          # K changed: new capture
    assert SG._fn_key(a) != SG._fn_key(lambda m, x: (m, x, 2))   # other code


def test_scalar_globals_key_the_loss_function():
    global GLOBAL_K
    k0 = SG._fn_key(_uses_global)
    GLOBAL_K = 4
    try:
        assert SG._fn_key(_uses_global) != k0
    finally:
        GLOBAL_K = 8
    assert SG._fn_key(_uses_global) == k0


def test_module_scalars_and_parameters_key_the_network():
    net = nn.Sequential(nn.Linear(3, 4), nn.Dropout(0.1))
    net.llik_scaling = 2.0
    x = [torch.zeros(2, 3)]
    params = list(net.parameters())
    s0 = SG._signature(net, _fn(1), x, False, params)
    assert SG._signature(net, _fn(1), x, False, params) == s0
    net[1].p = 0.2                                  # dropout changed
    assert SG._signature(net, _fn(1), x, False, params) != s0
    net[1].p = 0.1
    net.llik_scaling = 1.0                          # beta annealing
    assert SG._signature(net, _fn(1), x, False, params) != s0
    net.llik_scaling = 2.0
    net.eval()                                      # training flags
    assert SG._signature(net, _fn(1), x, False, params) != s0
    net.train()
    assert SG._signature(net, _fn(1), [torch.zeros(5, 3)], False, params) != s0   # ragged batch
    net[0].weight.requires_grad_(False)             # frozen parameter
    assert SG._signature(net, _fn(1), x, False, params) != s0


def test_numpy_and_tensor_attributes_key_the_network():
    """values baked into a captured graph as kernel arguments must be in
    the signature whatever their Python type -- numpy scalars (llik_scaling =
    1 / np.float64(beta)), numpy globals of the loss function -- and a tensor attribute
    re-bound to another tensor is a new signature."""
    import numpy as np
    net = nn.Sequential(nn.Linear(3, 4))
    net.llik_scaling = 1.0 / np.float64(0.5)
    x = [torch.zeros(2, 3)]
    params = list(net.parameters())
    s0 = SG._signature(net, _fn(1), x, False, params)
    net.llik_scaling = 1.0 / np.float64(0.25)       # beta annealing with a numpy beta
    assert SG._signature(net, _fn(1), x, False, params) != s0
    net.llik_scaling = 1.0 / np.float64(0.5)
    assert SG._signature(net, _fn(1), x, False, params) == s0
    net.scale = torch.ones(())
    s1 = SG._signature(net, _fn(1), x, False, params)
    net.scale.mul_(2)                               # in place: the graph reads it live
    assert SG._signature(net, _fn(1), x, False, params) == s1
    old = net.scale                                 # (kept alive: a distinct storage)
    net.scale = torch.ones(())                      # re-bound: a new signature
    assert SG._signature(net, _fn(1), x, False, params) != s1 and old is not net.scale
    net._private = np.float64(3.0)                  # private attributes never key
    assert SG._signature(net, _fn(1), x, False, params) == SG._signature(net, _fn(1), x, False, params)
    assert SG._fn_key(_fn(np.int64(2))) != SG._fn_key(_fn(np.int64(3)))
    assert SG._fn_key(_fn(np.int64(2))) == SG._fn_key(_fn(np.int64(2)))


def test_walk_matches_module_and_parameter_order():
    """_walk's single traversal gives Module.modules()' scalars and Module.parameters()
    in their orders, shared submodules / parameters once."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    shared = nn.Linear(2, 2)
    nets = [nn.Sequential(nn.Linear(3, 4), nn.Sequential(nn.Dropout(0.2), shared), shared),
            bench.make_model("cpu", 0.1)]
    for net in nets:
        scal, params = SG._walk(net)
        assert [id(p) for p in params] == [id(p) for p in net.parameters()]
        ref = tuple((k, SG._scalar_key(v)) for m in net.modules() for k, v in m.__dict__.items()
                    if k[0] != "_" and SG._scalar_key(v) is not SG._SKIP)
        assert scal == ref


def test_host_tensors_and_parity_rng_modes_run_eagerly():
    from VAESNe import rng
    net = nn.Linear(3, 4)
    assert SG.step(net, _fn(1), (torch.zeros(2, 3),), False) is None   # host batch: eager
    assert not SG.eligible("cpu")
    with rng.inject_uniform([torch.zeros(1)]):
        assert not rng.capturable()
    rng.set_mode("torch_cpu")
    try:
        assert not rng.capturable()
    finally:
        rng.set_mode("device")
    assert rng.capturable()


def test_unflat_restores_the_multimodal_structure():
    x = [(torch.zeros(1), torch.ones(1)), (torch.full((1,), 2.0),)]
    flat = SG._flat(x, True)
    assert len(flat) == 3
    back = SG._unflat(flat, x, True)
    assert isinstance(back, list) and len(back[0]) == 2 and len(back[1]) == 1
    assert back[1][0] is flat[2]


def test_capture_topology_rule():
    """ADVICE / VERDICT r03: the fork / join shapes that crash hipStreamEndCapture
    (tools/capture_patterns.py, profiles/r03_v4/capture_patterns.txt) raise
    CaptureTopologyError before the offending wait; the product's shapes (side streams
    forked from and joined into the origin) pass."""
    import pytest
    from VAESNe._capture import CaptureTopologyError, check_edges
    O, S, P, Q = 1, 2, 3, 4

    def edges(pattern):
        # "w X Y": X waits on Y (Y records an event, X waits on it); "k X": ignored
        out, n = [], 0
        for op in pattern.split("|"):
            f = op.split()
            if f[0] == "w":
                n += 1
                out += [("record", n, {"O": O, "S": S, "P": P, "Q": Q}[f[2]]),
                        ("wait", n, {"O": O, "S": S, "P": P, "Q": Q}[f[1]])]
        return out
    ok = ["w S O|k S|w O S", "w S O|w P O|k S|k P|w O S|w O P",
          "w S O|w P O|w Q O|k S|w O S|k O|w S O|k S|w O S"]
    crash = {   # each crashed (rc -11) in the r03 probe
        "nested": "w S O|w P S|k P|w S P|k S|w O S",
        "sibling_mutual": "w S O|w P O|k S|k P|w S P|k S|w P S|k P|w O S|w O P",
        "sibling_back": "w S O|w P O|k P|w S P|k S|w P S|k P|w O S|w O P",
        "child_waits_origin": "w S O|w P S|k P|w S P|k O|w P O|k P|w O P|w O S",
    }
    for p in ok:
        check_edges(O, edges(p))
    for name, p in crash.items():
        with pytest.raises(CaptureTopologyError):
            check_edges(O, edges(p))
    check_edges(O, [("wait", 99, S)])          # an event recorded before the capture
