"""Diagnostic (not product): the model's forward alone (no gradient), captured once as a
hipGraph, against eager forwards, with the parameters perturbed in place before every
replay (a launch that reads a buffer before this replay wrote it, or after a later
writer, then sees the previous replay's slightly different values)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import rng  # noqa: E402
from VAESNe._capture import guarded  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, float(os.environ.get("PDROP", "0.0")))
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
params = [p for p in model.parameters()]
K = 3


def flat(out):
    qz_xs, px_zs, zss = out
    ts = [q.loc for q in qz_xs] + [q.scale for q in qz_xs] + list(zss)
    ts += [t for t in px_zs.merged for t in t] if getattr(px_zs, "merged", None) else []
    return ts


def fwd():
    rng.manual_seed(99)
    rng.reset_call_ids()
    with torch.no_grad():
        return flat(model(x, K=K))


if os.environ.get("NOCACHE"):
    from VAESNe import _ops
    _ops._KBIAS_CACHE.clear()
    _ops._KBIAS_REP_CACHE.clear()
    _orig_append = list.append

    class _NoCache(list):
        def append(self, v):
            pass
    _ops._KBIAS_CACHE = _NoCache()
    _ops._KBIAS_REP_CACHE = _NoCache()
if os.environ.get("NO_SIDE") == "1":
    from VAESNe import mmVAE
    mmVAE._side_stream = lambda t: None
if os.environ.get("NO_CTX") == "1":
    from VAESNe import util_layers
    util_layers._ctx_stream = lambda t, i=0: None
if os.environ.get("NO_PREP"):
    # no latent-independent decoder prefix on the side stream: each decoder runs whole
    from VAESNe import SpectraVAE as _S, PhotometricVAE as _P
    for cls in [c for m in (_S, _P) for c in vars(m).values() if isinstance(c, type)]:
        if "decode_prepare" in vars(cls):
            delattr(cls, "decode_prepare")
if os.environ.get("SIDE_ONLY"):
    from VAESNe import mmVAE
    _B = mmVAE._Branches
    cnt = [0]

    class _Sel(_B):
        def __init__(self, side):
            cnt[0] += 1
            super().__init__(side if str((cnt[0] - 1) % 2 + 1) == os.environ["SIDE_ONLY"] else None)
    mmVAE._Branches = _Sel
fwd()
fwd()
torch.cuda.synchronize()
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
HELD = []


class Hold(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if any(r.alias_info is not None for r in func._schema.returns):
            return out
        for t in (out if isinstance(out, (tuple, list)) else [out]):
            if torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32:
                import traceback
                st = [f for f in traceback.extract_stack()[:-1] if "torch/" not in f.filename
                      and "diag_fwd" not in f.filename]
                HELD.append((t, func._schema.name + " " + " < ".join(
                    f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])))
        return out


import contextlib  # noqa: E402
MODE = os.environ.get("MODE", "")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    with guarded(), (Hold() if MODE else contextlib.nullcontext()):
        rng.reset_call_ids()
        with torch.no_grad():
            outs = flat(model(x, K=K))
names = ["qloc0", "qloc1", "qscale0", "qscale1", "z0", "z1", "ploc0", "pscale0", "ploc1", "pscale1"]
gen = torch.Generator(device=dev).manual_seed(5)
bad = 0
for r in range(int(os.environ.get("REPLAYS", "6"))):
    with torch.no_grad():
        for p in params:
            if p.dtype.is_floating_point:
                p.add_(1e-3 * torch.randn(p.shape, device=dev, generator=gen))
    ref = [t.clone() for t in fwd()]
    torch.cuda.synchronize()
    if MODE == "poison":
        lo, hi = (int(v) for v in os.environ.get("PRANGE", "0,100000").split(","))
        for t, _ in HELD[lo:hi]:
            t.fill_(float(os.environ.get("PVAL", "nan")))
    rng.manual_seed(99)
    g.replay()
    torch.cuda.synchronize()
    diff = [(n, float((a - b).abs().max())) for n, a, b in zip(names, ref, outs) if not torch.equal(a, b)]
    bad += bool(diff)
    print(f"replay {r}: {len(diff)} outputs differ {diff}")
    if os.environ.get("TWICE"):
        rng.manual_seed(99)
        g.replay()
        torch.cuda.synchronize()
        diff = [(n, float((a - b).abs().max())) for n, a, b in zip(names, ref, outs) if not torch.equal(a, b)]
        print(f"  same params, replayed again: {len(diff)} outputs differ {diff}")
print(f"{bad} differing replays; held {len(HELD)}")
if os.environ.get("SHOWHELD"):
    lo, hi = (int(v) for v in os.environ.get("PRANGE", "0,100000").split(","))
    for i, (t, n) in enumerate(HELD[lo:hi]):
        print("held", lo + i, n, tuple(t.shape))
