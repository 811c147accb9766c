"""Diagnostic (not product): eager step vs the same step captured and replayed, with every
_ops entry point wrapped to snapshot (clone, on the calling stream) its tensor inputs
before and its tensor outputs after the call.  Prints the first calls whose snapshots
differ between the eager run and a replay: the first differing OUTPUT whose inputs
agree names the launch that went wrong."""
import inspect
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _defer, _ops, _stepgraph, rng, training_util  # noqa: E402
from VAESNe._capture import guarded  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.1")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
params = list(model.parameters())
fn = lambda m, xx: m_iwae(m, xx, K=3)

LOG = []
ON = [False]
SKIP = {"used_on", "stream", "ptr", "require_device", "launch_timer"}


def _flat(o):
    if torch.is_tensor(o):
        return [o]
    if isinstance(o, (tuple, list)):
        return [t for e in o for t in _flat(e)]
    return []


def wrap(name, f):
    def g(*a, **k):
        if not ON[0]:
            return f(*a, **k)
        sid = torch.cuda.current_stream().stream_id
        ins = [t.detach().clone() for t in _flat(list(a) + list(k.values())) if t.is_cuda]
        out = f(*a, **k)
        outs = [t.detach().clone() for t in _flat(out) if t.is_cuda]
        LOG.append((name, sid, ins, outs))
        return out
    return g


for n_, v in list(vars(_ops).items()):
    if n_.startswith("_") or n_ in SKIP:
        continue
    if inspect.isclass(v) and issubclass(v, torch.autograd.Function) and v is not torch.autograd.Function:
        v.apply = staticmethod(wrap(n_ + ".apply", v.apply))
    elif inspect.isfunction(v) and v.__module__ == _ops.__name__:
        setattr(_ops, n_, wrap(n_, v))
# the model modules imported the names directly: patch theirs too
import VAESNe  # noqa: E402
for modname, mod in list(sys.modules.items()):
    if not modname.startswith("VAESNe.") or mod is _ops:
        continue
    for n_, v in list(vars(mod).items()):
        if getattr(v, "__module__", None) == _ops.__name__ and inspect.isfunction(v) and n_ in vars(_ops):
            setattr(mod, n_, getattr(_ops, n_))


def step():
    with _defer.deferred():
        return training_util.backward_negated(fn(model, x), negate=False)


def eager():
    rng.manual_seed(99)
    rng.reset_call_ids()
    for p in params:
        p.grad = None
    v = step()
    torch.cuda.synchronize()
    return v.item()


eager()
LOG.clear()
ON[0] = True
ref_loss = eager()
ref = list(LOG)
LOG.clear()
_stepgraph._drop_autograd_refs(model)
for p in params:
    p.grad = None
rng.manual_seed(99)
rng.reset_call_ids()
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    with guarded():
        sloss = step()
cap = list(LOG)
ON[0] = False
print("calls eager", len(ref), "captured", len(cap))
for rep in range(int(os.environ.get("REPLAYS", "4"))):
    rng.manual_seed(99)
    g.replay()
    torch.cuda.synchronize()
    nd = 0
    for i, (a, b) in enumerate(zip(ref, cap)):
        if a[0] != b[0]:
            print(f"  call {i}: name mismatch {a[0]} vs {b[0]}")
            break
        di = [j for j, (u, w) in enumerate(zip(a[2], b[2])) if u.shape == w.shape and not torch.equal(u, w)]
        do = [(j, float((u - w).abs().max())) for j, (u, w) in enumerate(zip(a[3], b[3]))
              if u.shape == w.shape and not torch.equal(u, w)]
        if di or do:
            nd += 1
            if nd <= int(os.environ.get("SHOW", "6")):
                print(f"  replay {rep} call {i} {a[0]} stream {a[1]}/{b[1]}: inputs differ {di} "
                      f"outputs differ {do} shapes in {[tuple(t.shape) for t in a[2]]}")
    print(f"replay {rep}: loss {sloss.item()!r} vs {ref_loss!r}; {nd} calls differ")
