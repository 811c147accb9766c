"""Captured training steps for `training_step` (the cannon scripts' own loop).

The scripts call `training_step(model, AdamW, loader, loss_fn=lambda m, x:
m_iwae(m, x, K=K), multimodal=True)` (cannon/ZTF_photospect.py:119-128): an eager
loop that launches every forward and backward kernel from Python, one batch at a
time.  At the reference's batch (16 pairs) the host side of ~450 launches per step
costs several times the GPU time of the step.  Here the forward + backward of a
batch signature is captured ONCE as a hipGraph and replayed for every later batch
of that signature: the batch is copied into the graph's static inputs, the graph
replays, the parameter gradients appear in the tensors the capture allocated, and
the user's optimizer steps eagerly on them, exactly as before.

Signature (everything the captured arithmetic depends on): the loss function's code,
closure values and the scalar globals it names (e.g. a script's `K`), the input
shapes / dtypes, every parameter's storage and requires_grad, and every module's
scalar attributes (training flags, dropout p, llik_scaling, ...).  A change of any
of them is a new signature; up to MAX_GRAPHS are kept per network (a loader's full
batches + its ragged last batch).  A signature is captured after WARMUP eager
batches; a capture that fails (a loss function that synchronises, say) marks the
signature eager for good.

Not captured (always eager): injected or torch-CPU-generator noise
(rng.inject_uniform / rng.set_mode("torch_cpu"): the parity paths), host tensors,
VAESNE_STEP_GRAPH=0.  Randomness: training_step restarts the RNG call ids at every
batch and advances the device counter after it, so a replayed batch draws exactly
what the same batch would draw eagerly (tests/test_gpu_stepgraph.py: bitwise).
"""
from __future__ import annotations

import numbers
import sys
import weakref

import numpy as np
import torch

from . import _config, _defer, rng, training_util
from ._capture import guarded as _guarded

WARMUP = 2
MAX_GRAPHS = 3

_SKIP = object()


def _scalar_key(v, depth=0):
    """The value key of a number (Python or numpy: an llik_scaling of 1/np.float64(beta)),
    string, None or a tuple / list of them; a tensor by its storage, shape and dtype (a
    graph reads the memory it was captured on, so re-binding the attribute to another
    tensor is a new signature while in-place updates need none); _SKIP otherwise."""
    if v is None or isinstance(v, (str, bool)):
        return v
    if isinstance(v, numbers.Number):
        if isinstance(v, np.generic):
            return (type(v).__name__, v.item())
        return (type(v).__name__, v)
    if isinstance(v, torch.Tensor):
        return ("tensor", v.data_ptr(), tuple(v.shape), v.dtype, v.device)
    if isinstance(v, (tuple, list)) and depth < 2 and len(v) <= 16:
        ks = tuple(_scalar_key(e, depth + 1) for e in v)
        return _SKIP if any(k is _SKIP for k in ks) else (type(v).__name__,) + ks
    return _SKIP


class _Entry:
    __slots__ = ("seen", "graph", "static_x", "loss", "params", "grads", "failed")

    def __init__(self):
        self.seen, self.graph, self.static_x, self.loss = 0, None, None, None
        self.params, self.grads, self.failed = None, None, False


_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_warned = set()


def _value_key(v):
    """Numbers, strings, tensors and tuples of them by value (_scalar_key); anything
    else (functions, modules, containers) by identity."""
    k = _scalar_key(v)
    return ("id", id(v)) if k is _SKIP else k


def _fn_key(fn):
    code = getattr(fn, "__code__", None)
    if code is None:
        return ("obj", id(fn))
    cells = tuple(_value_key(c.cell_contents) for c in (fn.__closure__ or ()))
    g = getattr(fn, "__globals__", {})
    names = []
    for n in code.co_names:     # the scalar globals it names (a script's K, beta, ...)
        if n in g:
            k = _scalar_key(g[n])
            if k is not _SKIP:
                names.append((n, k))
    defaults = tuple(_value_key(d) for d in (fn.__defaults__ or ()))
    kw = tuple(sorted((k, _value_key(v)) for k, v in (fn.__kwdefaults__ or {}).items()))
    return (code, cells, tuple(names), defaults, kw, _value_key(getattr(fn, "__self__", None)))


def _module_scalars(network):
    return _walk(network)[0]


_WALKS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _walk(network):
    """(the modules' scalar attributes, the parameters) of `network`, revalidated against
    the previous batch's walk instead of recomputed when nothing changed (_walk_valid):
    the full walk costs ~1 ms per batch on the unchanged script's loop, the check a
    fraction of it."""
    w = _WALKS.get(network)
    if w is not None and _walk_valid(w):
        return w[0], w[1]
    scalars, params, mods = _walk_full(network)
    _WALKS[network] = (scalars, params, mods)
    return scalars, params


def _walk_valid(w):
    """Every module of the cached walk still has the same attribute names, the same
    child modules and parameters (identity), and every scalar attribute the same object
    or the same key."""
    for d, keys, children, prms, watch in w[2]:
        if len(d) != len(keys) or tuple(d) != keys:
            return False
        if tuple(map(id, d["_modules"].values())) != children \
                or tuple(map(id, d["_parameters"].values())) != prms:
            return False
        for name, obj, k in watch:
            v = d[name]
            if v is not obj and _scalar_key(v) != k:
                return False
    return True


def _walk_full(network):
    """(the modules' scalar attributes, the parameters) in ONE pre-order traversal: the
    orders of Module.modules() / Module.parameters() (shared modules and parameters
    once), without named_modules' prefix strings: ~5x cheaper per batch than the two
    walks it replaces.  Also what _walk_valid checks: per module its __dict__, attribute
    names, children, parameters and (name, object, key) of each scalar attribute."""
    scalars, params, mods = [], [], []
    seen_m, seen_p = set(), set()
    stack = [network]
    while stack:
        m = stack.pop()
        if id(m) in seen_m:
            continue
        seen_m.add(id(m))
        d = m.__dict__
        watch = []
        # public attributes only: private ones (`_qz_x_params`, set by every forward;
        # the module's own registries) are not hyperparameters
        for name, v in d.items():
            if name[0] != "_":
                k = _scalar_key(v)
                if k is not _SKIP:
                    scalars.append((name, k))
                    # a list can change in place: re-keyed every time (no identity shortcut)
                    watch.append((name, None if isinstance(v, list) else v, k))
        for prm in d["_parameters"].values():
            if prm is not None and id(prm) not in seen_p:
                seen_p.add(id(prm))
                params.append(prm)
        mods.append((d, tuple(d), tuple(map(id, d["_modules"].values())),
                     tuple(map(id, d["_parameters"].values())), tuple(watch)))
        stack.extend(c for c in reversed(list(d["_modules"].values())) if c is not None)
    return tuple(scalars), params, mods


def _flat(x, multimodal):
    return [t for m in x for t in m] if multimodal else list(x)


def _unflat(ts, x, multimodal):
    if not multimodal:
        return tuple(ts)
    out, i = [], 0
    for m in x:
        out.append(tuple(ts[i:i + len(m)]))
        i += len(m)
    return out


def eligible(device) -> bool:
    return (_config.step_graph and torch.device(device).type == "cuda" and rng.capturable()
            and torch.is_grad_enabled())


def _signature(network, loss_fn, xs, multimodal, params, scalars=None):
    if scalars is None:
        scalars = _module_scalars(network)
    return (_fn_key(loss_fn), multimodal, tuple((tuple(t.shape), t.dtype) for t in xs),
            tuple((p.data_ptr(), p.requires_grad) for p in params), scalars)


def step(network, loss_fn, x, multimodal):
    """The batch's objective value (a device scalar: the loss is its negation, as
    training_util.backward_negated(..., negate=False) returns it) with every parameter
    gradient set, from a replay of the captured step; None when this batch must run
    eagerly (warm-up, an uncapturable signature)."""
    xs = _flat(x, multimodal)
    if not all(t.is_cuda for t in xs):
        return None
    scalars, params = _walk(network)
    key = _signature(network, loss_fn, xs, multimodal, params, scalars)
    graphs = _CACHE.setdefault(network, {})
    ent = graphs.get(key)
    if ent is None:
        while len(graphs) >= MAX_GRAPHS:
            graphs.pop(next(iter(graphs)))
        ent = graphs[key] = _Entry()
    if ent.failed:
        return None
    if ent.graph is None:
        ent.seen += 1
        if ent.seen <= WARMUP:
            return None
        if not _capture(ent, network, loss_fn, x, xs, multimodal, params):
            return None
    for s, t in zip(ent.static_x, xs):
        s.copy_(t, non_blocking=True)
    ent.graph.replay()
    for p, g in zip(ent.params, ent.grads):
        p.grad = g
    return ent.loss


def _drop_autograd_refs(network):
    """The VAEs keep their last posterior parameters (the reference's _qz_x_params).
    Detached, they no longer hold the previous step's autograd graph alive: its
    AccumulateGrad nodes are bound to the eager step's stream and must not be reused
    by a capture (torch then syncs the capture with that stream and the capture
    breaks)."""
    for m in network.modules():
        q = getattr(m, "_qz_x_params", None)
        if isinstance(q, (tuple, list)):
            m._qz_x_params = type(q)(t.detach() if torch.is_tensor(t) else t for t in q)


def _capture(ent, network, loss_fn, x, xs, multimodal, params) -> bool:
    static_x = [t.clone() for t in xs]
    sx = _unflat(static_x, x, multimodal)
    _drop_autograd_refs(network)
    for p in params:
        p.grad = None                     # gradients are allocated in the graph's pool
    g = torch.cuda.CUDAGraph()
    try:
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            with _guarded(), _defer.deferred():
                sloss = training_util.backward_negated(loss_fn(network, sx), negate=False)
    except Exception as e:   # noqa: BLE001 -- any capture failure: this signature stays eager
        ent.failed = True
        for p in params:
            p.grad = None
        torch.cuda.synchronize()
        rng.reset_call_ids()      # the eager rerun of this batch draws what it would have
        if type(e).__name__ not in _warned:
            _warned.add(type(e).__name__)
            print(f"[VAESNe] training_step: the step could not be captured as a hipGraph "
                  f"({type(e).__name__}: {e}); running it eagerly", file=sys.stderr)
        return False
    _drop_autograd_refs(network)
    ent.graph, ent.static_x, ent.loss = g, static_x, sloss
    ent.params = [p for p in params if p.grad is not None]
    ent.grads = [p.grad for p in ent.params]
    return True


def clear(network=None):
    """Drop the captured steps (of one network, or all)."""
    if network is None:
        _CACHE.clear()
    else:
        _CACHE.pop(network, None)
