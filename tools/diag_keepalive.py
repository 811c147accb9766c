"""Diagnostic (not product): eager step vs the same step captured and replayed, with every
tensor an aten op creates during the step kept alive until the end (KEEP=all), or only
those created while the current stream is the main / a side stream (KEEP=main|other),
or none (KEEP=none).  If keeping tensors alive removes an eager/replay mismatch, a
tensor's memory is handed to a new allocation while another stream still uses it."""
import os
import sys

import torch
from torch.utils._python_dispatch import TorchDispatchMode

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
KEEP = os.environ.get("KEEP", "all")
MAIN = torch.cuda.current_stream()
HELD = []


class Keep(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        st = torch.cuda.current_stream()
        on_main = st == MAIN
        if KEEP == "all" or (KEEP == "main" and on_main) or (KEEP == "other" and not on_main):
            outs = out if isinstance(out, (tuple, list)) else [out]
            HELD.extend(t for t in outs if torch.is_tensor(t) and t.is_cuda)
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
    with guarded():
        if KEEP == "none":
            sloss = step()
        else:
            with Keep():
                sloss = step()
grads = [p.grad for p in params]
print(f"KEEP={KEEP}: held {len(HELD)} tensors")
for rep in range(int(os.environ.get("REPLAYS", "5"))):
    rng.manual_seed(99)
    g.replay()
    torch.cuda.synchronize()
    diff = [n for n, a, b in zip(names, ref[1], grads) if a is not None and not torch.equal(a, b)]
    print(f"replay {rep}: loss {sloss.item()!r} vs eager {ref[0]!r}; {len(diff)} grads differ")
