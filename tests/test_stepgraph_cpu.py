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
        ref = tuple(v for m in net.modules() for v in m.__dict__.values()
                    if type(v) in SG._SCALARS)
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
