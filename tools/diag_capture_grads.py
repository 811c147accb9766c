"""Diagnostic (not product): eager forward + backward of the bench model vs the same step
captured as a hipGraph and replayed (VAESNe._stepgraph's capture recipe), per-parameter
bitwise comparison of the gradients."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _defer, _lib, _stepgraph, rng, training_util  # noqa: E402
from VAESNe._capture import guarded  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.1")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
params = list(model.parameters())
names = [n for n, _ in model.named_parameters()]
fn = lambda m, xx: m_iwae(m, xx, K=3)
# stash every module output tensor of the spectra decoder / encoder (forward activations)
acts = {}


def hook(name):
    def f(mod, inp, out):
        if torch.is_tensor(out):
            acts[name] = out.detach().clone()
        elif isinstance(out, (tuple, list)):
            for i, o in enumerate(out):
                if torch.is_tensor(o):
                    acts[f"{name}[{i}]"] = o.detach().clone()
    return f


for n_, m_ in model.named_modules():
    if n_.count(".") <= 3 and n_:
        m_.register_forward_hook(hook(n_))


def eager():
    rng.manual_seed(99)
    rng.reset_call_ids()
    for p in params:
        p.grad = None
    with _defer.deferred():
        v = training_util.backward_negated(fn(model, x), negate=False)
    torch.cuda.synchronize()
    return v.item(), [None if p.grad is None else p.grad.clone() for p in params]


ref = eager()
ref_acts = {k: v.detach().clone() for k, v in acts.items()}
ref2 = eager()
print("eager twice equal:", ref[0] == ref2[0] and all(
    (a is None and b is None) or torch.equal(a, b) for a, b in zip(ref[1], ref2[1])))
_stepgraph._drop_autograd_refs(model)
for p in params:
    p.grad = None
rng.manual_seed(99)
rng.reset_call_ids()
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    with guarded(), _defer.deferred():
        sloss = training_util.backward_negated(fn(model, x), negate=False)
grads = [p.grad for p in params]
for rep in range(3):
    rng.manual_seed(99)
    g.replay()
    torch.cuda.synchronize()
    ad = [(k, float((acts[k] - v).abs().max())) for k, v in ref_acts.items()
          if k in acts and acts[k].shape == v.shape and not torch.equal(acts[k], v)]
    print(f"replay {rep}: forward activations differing: {len(ad)} of {len(ref_acts)}", ad[:10])
    diff = [(n, float((a - b).abs().max())) for n, a, b in zip(names, ref[1], grads)
            if a is not None and not torch.equal(a, b)]
    print(f"replay {rep}: loss {sloss.item()!r} vs eager {ref[0]!r}; {len(diff)} grads differ")
    same = [n for n, a, b in zip(names, ref[1], grads) if a is not None and torch.equal(a, b)]
    print("   equal:", len(same), same[:40])
    big = sorted(diff, key=lambda d: -d[1] / max(1e-30, float(ref[1][names.index(d[0])].abs().max())))
    for d in big[:8]:
        print("   ", d, "rel", d[1] / max(1e-30, float(ref[1][names.index(d[0])].abs().max())))
