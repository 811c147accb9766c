"""Diagnostic (not product): find a launch inside the captured training step that reads a
buffer before this replay has written it (a missing dependency that reads the previous
replay's values).  Captures one forward + backward with every float tensor an aten op
creates held alive (VAESNE_DEFER_GRADS=0 is set here: held references defeat the deferred
gradient sums), fills all of them with NaN before a replay, and after it lists the held
tensors that still hold NaN, in creation order: the first of them whose creator fully
writes it names the consumer side of the race."""
import os
import sys
import traceback

os.environ.setdefault("VAESNE_DEFER_GRADS", "0")
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _defer, _stepgraph, rng, training_util  # noqa: E402
from VAESNe._capture import guarded  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.1")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
params = list(model.parameters())
names = [n for n, _ in model.named_parameters()]
fn = lambda m, xx: m_iwae(m, xx, K=3)
HELD = []
MAIN = torch.cuda.current_stream()


def _where():
    st = [f for f in traceback.extract_stack()[:-2] if "torch/" not in f.filename
          and "diag_poison" not in f.filename]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])


class Keep(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if any(r.alias_info is not None for r in func._schema.returns):
            return out            # a view or an in-place result: not a new buffer
        outs = out if isinstance(out, (tuple, list)) else [out]
        for t in outs:
            if torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32:
                side = "main" if torch.cuda.current_stream() == MAIN else "other"
                HELD.append((t, func._schema.name, side, _where()))
        return out


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
    return v.item(), [None if p.grad is None else p.grad.clone() for p in params]


eager()
ref = eager()
_stepgraph._drop_autograd_refs(model)
for p in params:
    p.grad = None
rng.manual_seed(99)
rng.reset_call_ids()
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    with guarded(), Keep():
        sloss = step()
grads = [p.grad for p in params]
print(f"held {len(HELD)} float tensors")
for rep in range(int(os.environ.get("REPLAYS", "3"))):
    for t, *_ in HELD:
        t.fill_(float("nan"))
    rng.manual_seed(99)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    nan = [(i, op, side, where, float(torch.isnan(t).float().mean()))
           for i, (t, op, side, where) in enumerate(HELD) if torch.isnan(t).any()]
    diff = [n for n, a, b in zip(names, ref[1], grads) if a is not None and not torch.equal(a, b)]
    print(f"replay {rep}: loss {sloss.item()!r} vs eager {ref[0]!r}; {len(diff)} grads differ; "
          f"{len(nan)} held tensors with NaN")
    for e in nan[:int(os.environ.get("SHOW", "12"))]:
        print("   ", e)
