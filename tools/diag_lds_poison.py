"""Diagnostic (not product): find kernels that read LDS they never wrote.  Every VAESNe
autograd op (forward and backward) runs right after a kernel that fills the LDS of every
CU with a NaN pattern (tools/probe/liblds_poison.so); the first op whose outputs hold a
NaN that the unpoisoned run does not is the reader."""
import ctypes
import inspect
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _defer, _ops, rng, training_util, _chain  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

P = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "liblds_poison.so"))
PATTERN = int(os.environ.get("PATTERN", str(0x7FC00000)), 0)
ON = [False]
FOUND = []


def poison():
    if ON[0]:
        assert P.lds_poison(ctypes.c_uint32(PATTERN), 2048,
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0


def _tensors(o):
    if torch.is_tensor(o):
        return [o]
    if isinstance(o, (tuple, list)):
        return [t for e in o for t in _tensors(e)]
    return []


def check(name, out):
    if not ON[0]:
        return
    torch.cuda.synchronize()
    for t in _tensors(out):
        if t.is_cuda and t.is_floating_point() and not torch.isfinite(t).all():
            FOUND.append(name)
            print("non-finite output of", name, tuple(t.shape), flush=True)
            return


def wrap(name, f):
    def g(*a, **k):
        poison()
        out = f(*a, **k)
        check(name, out)
        return out
    return g


for mod in (_ops, _chain):
    for n_, v in list(vars(mod).items()):
        if inspect.isclass(v) and issubclass(v, torch.autograd.Function) and v is not torch.autograd.Function:
            v.forward = staticmethod(wrap(n_ + ".forward", v.forward))
            v.backward = staticmethod(wrap(n_ + ".backward", v.backward))

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.1")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)


def step():
    rng.manual_seed(99)
    rng.reset_call_ids()
    for p in model.parameters():
        p.grad = None
    with _defer.deferred():
        v = training_util.backward_negated(m_iwae(model, x, K=3), negate=False)
    torch.cuda.synchronize()
    return v.item()


base = step()
ON[0] = True
pois = step()
print(f"loss unpoisoned {base!r} poisoned {pois!r}; ops with non-finite outputs: {FOUND[:10]}")
