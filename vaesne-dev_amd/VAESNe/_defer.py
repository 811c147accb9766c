"""Deferred parameter-gradient sums (include/vaesne_hip.h: vaesne_colsum_list).

Every parameter gradient of the step is a fixed-order column sum over
per-workgroup partials.  Launched right after its producer, each is one more
kernel (about 90 per training step) and, in a captured step, one more graph
node on the backward's dependency chains.  Inside `deferred()` (entered by
training_util.training_step and the bench step around forward + backward) the
producers append their sums to one list instead, and an autograd final callback
launches them all when the backward pass ends (vaesne_colsum_flush: one or two
launches), before anything can read a parameter gradient.

A deferred gradient holds no values until the flush, so nothing may read it
before: an op defers only if each parameter it produces a gradient for was
used by exactly one VAESNe op in the forward (counted here), has .grad None
(no accumulation into an existing gradient) and carries no tensor hooks.  A
parameter that ALSO feeds a plain torch op would have its two gradients summed
by autograd before the flush: the flush detects that (the parameter's .grad is
not the deferred tensor, or was modified in place) and raises; run such models
outside `deferred()` (the per-op sums are then launched at once, as always).
"""
from __future__ import annotations

import contextlib
import ctypes as C

import torch

from . import _config, _stamps
from ._lib import lib


class Entry(C.Structure):
    _fields_ = [("partial", C.c_void_p), ("ld", C.c_int64), ("groups", C.c_int),
                ("cols", C.c_int), ("out", C.c_void_p), ("accum", C.c_int)]


class List(C.Structure):
    _fields_ = [("entries", C.POINTER(Entry)), ("count", C.c_int), ("capacity", C.c_int)]


CAPACITY = 2048
_MAX_ENTRIES_PER_CALL = 8        # vaesne_*_bwd append at most 7 sums per call


class _State:
    def __init__(self):
        self.depth = 0
        self.uses = {}
        self.store = (Entry * CAPACITY)()
        self.clist = List(C.cast(self.store, C.POINTER(Entry)), 0, CAPACITY)
        self.pending = []        # (param, output data_ptr, output version) to verify
        self.keep = []           # partial buffers alive until the flush
        self.streams = []
        self.armed = False


_S = _State()


def active() -> bool:
    return _S.depth > 0


@contextlib.contextmanager
def deferred(enabled=None):
    """Defer the parameter-gradient sums of the backward passes run inside
    (enabled None: _config.defer_grads, on unless VAESNE_DEFER_GRADS=0)."""
    if enabled is None:
        enabled = _config.defer_grads
    if not enabled:
        yield
        return
    _S.depth += 1
    if _S.depth == 1:
        _S.uses.clear()
    try:
        yield
    finally:
        _S.depth -= 1
        if _S.depth == 0:
            _S.uses.clear()
            if _S.armed or _S.clist.count or _S.pending:
                # a backward raised before its final callback (the flush) ran: drop
                # the queued sums, so the next backward arms a fresh flush and never
                # touches the freed partial buffers of this one.  The gradients it
                # had deferred hold no values: the caller's next zero_grad (or the
                # exception) discards them.
                _reset()


def _reset():
    _S.clist.count = 0
    _S.pending, _S.keep, _S.streams = [], [], []
    _S.armed = False


def count_uses(*params):
    """Forward side: record one use of each parameter tensor (deferral only)."""
    if _S.depth == 0:
        return
    for p in params:
        if p is not None and p.requires_grad and p.is_leaf:
            _S.uses[id(p)] = _S.uses.get(id(p), 0) + 1


def _deferrable(p) -> bool:
    return (p.is_leaf and p.grad is None and _S.uses.get(id(p), 0) == 1
            and not p._backward_hooks
            and not getattr(p, "_post_accumulate_grad_hooks", None))


def target(params, outputs, keep=(), entries=_MAX_ENTRIES_PER_CALL):
    """Backward side: the list to append this op's sums to (a ctypes pointer), or
    None to launch them now.  `params[i]` receives `outputs[i]` (None entries
    skipped); `keep` = the partial buffers the sums read; `entries` = the most sums
    the op appends."""
    if _S.depth == 0 or _S.clist.count + entries > CAPACITY:
        return None
    pairs = [(p, o) for p, o in zip(params, outputs) if p is not None and o is not None]
    if not pairs or not all(_deferrable(p) for p, _ in pairs):
        return None
    if not _S.armed:
        torch.autograd.Variable._execution_engine.queue_callback(flush)
        _S.armed = True
    st = torch.cuda.current_stream()
    if all(st != s for s in _S.streams):
        _S.streams.append(st)
    # no reference to the outputs is kept: autograd must be able to steal them
    # into .grad (an extra reference would make AccumulateGrad copy them, i.e.
    # read them before the flush)
    _S.pending.append([(p, o.data_ptr(), o._version) for p, o in pairs])
    _S.keep.extend(keep)
    return C.byref(_S.clist)


def flush():
    """Launch every pending sum on the current stream (after all producer streams)."""
    _S.armed = False
    if _S.clist.count == 0 and not _S.pending:
        return
    cur = torch.cuda.current_stream()
    for s in _S.streams:
        if s != cur:
            cur.wait_stream(s)
    _stamps.mark("flush")
    lib.colsum_flush(C.byref(_S.clist), cur.cuda_stream)
    for t in _S.keep:
        t.record_stream(cur)
    pending = _S.pending
    _S.pending, _S.keep, _S.streams = [], [], []
    for group in pending:
        for p, ptr_, ver in group:
            g = p.grad
            if g is None:
                continue     # torch.autograd.grad: the gradient went to the caller
            if g.data_ptr() == ptr_ and g._version == ver:
                g.record_stream(cur)   # written on `cur` by the flush
            else:
                raise RuntimeError(
                    "VAESNe deferred gradient sums: a parameter received a second gradient "
                    "outside the VAESNe ops (e.g. a plain torch op on the parameter) before "
                    "the sums were launched; run this model outside VAESNe._defer.deferred()")
