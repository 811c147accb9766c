"""Diagnostic (not product): a stream-ordering checker for one eager training step of the
bench model.  It extends torch.cuda._sanitizer's happens-before bookkeeping (HIP events /
stream waits seen through torch's GPU trace hooks) with

* the VAESNe launches: every _ops entry point and every autograd Function's forward and
  backward count as one kernel that reads its tensor inputs (and saved tensors) and writes
  its tensor outputs, on the stream current at the call;
* memory reuse: when the caching allocator hands out a block, every access to the freed
  tensor that lived there from a stream other than the allocating one must be ordered
  before the allocating stream's current point, unless the tensor was record_stream'ed
  to that stream.

Accesses are keyed by storage (untyped_storage base pointer and size)."""
import collections
import functools
import inspect
import os
import re
import sys
import traceback

import torch
import torch.cuda._gpu_trace as gpu_trace
from torch.cuda._sanitizer import StreamSynchronizations
from torch.utils import _pytree as pytree
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _defer, _ops, rng, training_util  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

Acc = collections.namedtuple("Acc", "stream seq op where")
FACTORY = re.compile("(new_.*|.*_like|empty.*)")


def _where():
    st = [f for f in traceback.extract_stack()[:-3] if "diag_stream_sanitizer" not in f.filename
          and "torch/" not in f.filename]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-4:][::-1])


class Checker:
    def __init__(self):
        self.syncs = StreamSynchronizations()
        self.seq = 0
        self.live = {}          # base ptr -> [nbytes, last write Acc, reads since, recorded set]
        self.dead = []          # (base, nbytes, accesses, recorded set)
        self.reports = collections.OrderedDict()
        self.enabled = False

    def _ordered(self, stream, acc):
        return acc.stream == stream or self.syncs.is_ordered_after(stream, acc.seq, acc.stream)

    def _report(self, kind, cur, prev):
        key = (kind, cur.op, prev.op, cur.where, prev.where)
        self.reports[key] = self.reports.get(key, 0) + 1

    def launch(self, reads, writes, op):
        if not self.enabled:
            return
        stream = torch.cuda.current_stream().cuda_stream
        self.seq += 1
        self.syncs.update_seq_num(stream, self.seq)
        where = _where()
        cur = Acc(stream, self.seq, op, where)
        for t in reads:
            e = self._entry(t)
            if e[1] is not None and not self._ordered(stream, e[1]):
                self._report("read-after-write", cur, e[1])
            e[2].append(cur)
        for t in writes:
            e = self._entry(t)
            for prev in (e[2] if e[2] else ([e[1]] if e[1] is not None else [])):
                if not self._ordered(stream, prev):
                    self._report("write-after-" + ("read" if e[2] else "write"), cur, prev)
            e[1], e[2] = cur, []

    def _entry(self, t):
        s = t.untyped_storage()
        base = s.data_ptr()
        e = self.live.get(base)
        if e is None:
            e = self.live[base] = [s.nbytes(), None, [], set()]
        else:
            e[0] = max(e[0], s.nbytes())
        return e

    def autograd_join(self, grads):
        """autograd makes a node's stream wait for the streams that produced its incoming
        gradients (events the GPU trace hooks may not show): merge those streams' states"""
        if not self.enabled:
            return
        stream = torch.cuda.current_stream().cuda_stream
        for t in grads:
            w = self._entry(t)[1]
            if w is not None and w.stream != stream:
                self.syncs._ensure_stream_exists(stream)
                self.syncs._ensure_stream_exists(w.stream)
                self.syncs._state_wait_for_other(self.syncs.current_sync_states[stream],
                                                 self.syncs.current_sync_states[w.stream])

    def record_stream(self, t, stream):
        if self.enabled and t.is_cuda:
            self._entry(t)[3].add(stream.cuda_stream)

    # GPU trace callbacks
    def on_free(self, ptr):
        e = self.live.pop(ptr, None)
        if e is not None:
            accs = ([e[1]] if e[1] is not None else []) + e[2]
            self.dead.append((ptr, e[0], accs, e[3]))

    def on_alloc(self, ptr):
        if not self.enabled:
            return
        stream = torch.cuda.current_stream().cuda_stream
        keep = []
        for d in self.dead:
            base, n, accs, rec = d
            if base <= ptr < base + n:
                for a in accs:
                    if a.stream != stream and a.stream not in rec and not self._ordered(stream, a):
                        self._report("reuse-before-other-stream-done",
                                     Acc(stream, self.seq, "alloc", _where()), a)
                        print(f"REUSE on {sname(stream)} of [{base:#x} +{n}] last used on {sname(a.stream)} "
                              f"by {a.op}; all accesses: "
                              + "; ".join(f"{x.op}@{sname(x.stream)}" for x in accs)
                              + f"; recorded to {[sname(r) for r in rec]}")
            else:
                keep.append(d)
        self.dead = keep


NAMES = {}


def sname(h):
    return NAMES.get(h, hex(h))


def fill_names():
    from VAESNe import mmVAE, util_layers
    NAMES[torch.cuda.default_stream().cuda_stream] = "main"
    for st in mmVAE._SIDE.values():
        NAMES[st.cuda_stream] = "side"
    for d in util_layers._CTX_STREAMS.values():
        for i, st in d.items():
            NAMES[st.cuda_stream] = f"cs{i}"


CHK = Checker()
gpu_trace.register_callback_for_event_record(lambda ev, st: CHK.syncs.record_state(ev, st))
gpu_trace.register_callback_for_event_wait(lambda ev, st: CHK.syncs.stream_wait_for_event(st, ev))
gpu_trace.register_callback_for_memory_allocation(CHK.on_alloc)
gpu_trace.register_callback_for_memory_deallocation(CHK.on_free)
gpu_trace.register_callback_for_device_synchronization(lambda: CHK.syncs.sync_all_streams())
gpu_trace.register_callback_for_stream_synchronization(lambda st: CHK.syncs.all_streams_wait_for_stream(st))
gpu_trace.register_callback_for_event_synchronization(lambda ev: CHK.syncs.all_streams_wait_for_event(ev))
gpu_trace.register_callback_for_event_creation(lambda ev: CHK.syncs.create_event(ev))
gpu_trace.register_callback_for_event_deletion(lambda ev: CHK.syncs.delete_event(ev))
gpu_trace.register_callback_for_stream_creation(lambda st: CHK.syncs.create_stream(st))
torch._C._activate_gpu_trace()

_orig_record = torch.Tensor.record_stream


def _record_stream(self, stream):
    CHK.record_stream(self, stream)
    return _orig_record(self, stream)


torch.Tensor.record_stream = _record_stream


def _cuda_tensors(obj):
    out = []
    pytree.tree_map_(lambda v: out.append(v) if isinstance(v, torch.Tensor) and v.is_cuda else None, obj)
    return out


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        reads, writes = [], []
        schema = func._schema
        if schema.name == "aten::record_stream" or FACTORY.match(schema.name.split("::")[-1]):
            return out
        for i, arg in enumerate(schema.arguments):
            v = args[i] if i < len(args) else kwargs.get(arg.name)
            ts = _cuda_tensors(v)
            if arg.alias_info is not None and arg.alias_info.is_write:
                writes += ts
            elif arg.alias_info is None:
                reads += ts
        name = schema.name
        if not (name.endswith("empty") or "empty" in name or name in ("aten::view", "aten::_unsafe_view")):
            outs = _cuda_tensors(out)
            ret_views = any(r.alias_info is not None and not r.alias_info.is_write for r in schema.returns)
            if not ret_views:
                writes += outs
        CHK.launch(reads, writes, name)
        return out


def wrap_fn(name, f):
    @functools.wraps(f)
    def g(*a, **k):
        ins = _cuda_tensors((a, k))
        out = f(*a, **k)
        CHK.launch(ins, _cuda_tensors(out), name)
        return out
    return g


def wrap_bwd(name, f):
    def g(ctx, *grads):
        saved = list(getattr(ctx, "saved_tensors", ()) or ())
        CHK.autograd_join(_cuda_tensors(grads))
        out = f(ctx, *grads)
        CHK.launch(_cuda_tensors((grads, saved)), _cuda_tensors(out), name + ".backward")
        return out
    return g


for n_, v in list(vars(_ops).items()):
    if inspect.isclass(v) and issubclass(v, torch.autograd.Function) and v is not torch.autograd.Function:
        fwd = v.forward
        v.forward = staticmethod(wrap_fn(n_ + ".forward", fwd))
        v.backward = staticmethod(wrap_bwd(n_, v.backward))

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.1")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
fn = lambda m, xx: m_iwae(m, xx, K=3)


def step():
    rng.manual_seed(99)
    rng.reset_call_ids()
    for p in model.parameters():
        p.grad = None
    with _defer.deferred():
        v = training_util.backward_negated(fn(model, x), negate=False)
    torch.cuda.synchronize()
    return v


step()
torch.cuda.synchronize()
fill_names()
print("streams", NAMES)
CHK.enabled = True
if os.environ.get("CAPTURE"):
    from VAESNe import _stepgraph
    from VAESNe._capture import guarded
    _stepgraph._drop_autograd_refs(model)
    for p in model.parameters():
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        NAMES[torch.cuda.current_stream().cuda_stream] = "capture"
        with guarded(), Mode():
            rng.reset_call_ids()
            with _defer.deferred():
                training_util.backward_negated(fn(model, x), negate=False)
else:
    with Mode():
        step()
CHK.enabled = False
print(f"{len(CHK.reports)} distinct reports")
for (kind, cop, pop, cw, pw), n in list(CHK.reports.items())[:int(os.environ.get("SHOW", "40"))]:
    print(f"[{n}x] {kind}: {cop} @ {cw}\n        after {pop} @ {pw}")
