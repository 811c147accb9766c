"""Refuse, with an error, the stream topologies that crash a hipGraph capture.

On this ROCm a stream other than the capture's origin that waits on another captured
stream is filed under that stream, and hipStreamEndCapture walks those files
recursively: two non-origin streams that wait on each other -- directly, or through
autograd, which replays each op's backward on its forward stream and so reverses
every cross-stream edge of the forward -- recurse until the host stack overflows
(tools/capture_patterns.py: 7 of 9 fork / join shapes end in SIGSEGV inside
hipStreamEndCapture; DESIGN.md "The backward tail and the graph executor").

The product's captures (training_step's step graphs, bench.py's step) fork every
side stream from the origin and join it back into the origin only.  `guarded()`
holds a capture to that rule: while it is active, every event recorded and every
event waited on (Stream.wait_stream / wait_event, Event.wait) is checked, and a wait
of one non-origin stream on another raises CaptureTopologyError BEFORE the wait is
issued -- the capture then ends unjoined (an ordinary HIP error) instead of taking
the process down.  A future stream change, or a VAESNE_CTX_STREAMS setting that
nests a fork, fails loudly here."""
from __future__ import annotations

import contextlib

import torch


class CaptureTopologyError(RuntimeError):
    pass


def check_wait(origin, waiter, source):
    """The rule for one edge `waiter` waits on `source` (stream handles; source None:
    an event never recorded in this capture, e.g. one recorded before it)."""
    if source is None or waiter == source or waiter == origin or source == origin:
        return
    raise CaptureTopologyError(
        f"hipGraph capture: side stream {waiter:#x} would wait on side stream {source:#x}; "
        "side streams may only fork from and join into the capture's origin stream "
        "(a nested or mutual wait crashes hipStreamEndCapture on this ROCm)")


def check_edges(origin, edges):
    """Replay an edge list: ("record", event, stream) / ("wait", event, stream)."""
    where = {}
    for op, ev, st in edges:
        if op == "record":
            where[ev] = st
        else:
            check_wait(origin, st, where.get(ev))


_active = []


@contextlib.contextmanager
def guarded(origin=None):
    """Check every cross-stream edge created inside the block (see module doc)."""
    if not torch.cuda.is_available():
        yield
        return
    origin = (origin or torch.cuda.current_stream()).cuda_stream
    state = {"origin": origin, "where": {}}
    _active.append(state)
    E = torch.cuda.Event
    rec, wait = E.record, E.wait
    if len(_active) == 1:
        def record(self, stream=None):
            s = stream if stream is not None else torch.cuda.current_stream()
            if _active:
                _active[-1]["where"][id(self)] = (self, s.cuda_stream)
            return rec(self, stream)

        def wait_(self, stream=None):
            s = stream if stream is not None else torch.cuda.current_stream()
            if _active:
                st = _active[-1]
                src = st["where"].get(id(self))
                check_wait(st["origin"], s.cuda_stream,
                           src[1] if src is not None and src[0] is self else None)
            return wait(self, stream)
        E.record, E.wait = record, wait_
    try:
        yield
    finally:
        _active.pop()
        if not _active:
            E.record, E.wait = rec, wait
