"""Diagnostic (not product): tests/test_gpu_stepgraph.py's eager-vs-captured training loop,
optionally with every CUDA tensor an aten op creates kept alive (KEEP=all|main|other|none;
main/other: only those created while the current stream is / is not the main stream).
KEEP=record|record_main|record_other: record the new tensors on every stream instead
(blocks with stream uses are not reused during a capture).  KEEP=all|main|other need
VAESNE_DEFER_GRADS=0 (held references defeat the deferred gradient sums)."""
import os
import sys

import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils.data import DataLoader, TensorDataset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _config, _stepgraph, rng  # noqa: E402
from VAESNe.data_util import multimodalDataset  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402
from VAESNe.training_util import training_step  # noqa: E402

DEV = torch.device("cuda", 0)
KEEP = os.environ.get("KEEP", "none")
MAIN = torch.cuda.current_stream()
HELD = []
CNT = [0]
SKIPPED = []
LO, HI = (int(v) for v in os.environ.get("RANGE", "0,0").split(","))


def _where():
    import traceback
    st = [f for f in traceback.extract_stack()[:-2] if "torch/" not in f.filename
          and "diag_stepgraph" not in f.filename]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])


def _streams():
    from VAESNe import mmVAE, util_layers
    sts = [MAIN] + list(mmVAE._SIDE.values())
    for d in util_layers._CTX_STREAMS.values():
        sts += list(d.values())
    return sts


class Keep(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        on_main = torch.cuda.current_stream() == MAIN
        if KEEP == "record_except" and func._schema.name != "aten::record_stream":
            # record every capture-time allocation except those with index in [LO, HI)
            if torch.cuda.is_current_stream_capturing():
                i = CNT[0]
                CNT[0] += 1
                skip = LO <= i < HI
                outs = out if isinstance(out, (tuple, list)) else [out]
                for t in outs:
                    if torch.is_tensor(t) and t.is_cuda:
                        if skip:
                            SKIPPED.append((i, func._schema.name, tuple(t.shape), _where()))
                        else:
                            for st in _streams():
                                t.record_stream(st)
            return out
        if KEEP.startswith("record") and func._schema.name != "aten::record_stream":
            if KEEP == "record" or (KEEP == "record_main") == on_main:
                outs = out if isinstance(out, (tuple, list)) else [out]
                for t in outs:
                    if torch.is_tensor(t) and t.is_cuda:
                        for st in _streams():
                            t.record_stream(st)
            return out
        if KEEP == "all" or (KEEP == "main" and on_main) or (KEEP == "other" and not on_main):
            outs = out if isinstance(out, (tuple, list)) else [out]
            HELD.extend(t for t in outs if torch.is_tensor(t) and t.is_cuda)
        return out


def run(graph, epochs=3, B=4, n=11):
    _config.step_graph = graph
    torch.manual_seed(0)
    model = bench.make_model(DEV, float(os.environ.get("PDROP", "0.1")))
    rng.manual_seed(99)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    x = bench.synthetic_batch(n, 7, "cpu")
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=B, shuffle=False)
    losses = []
    for ep in range(epochs):
        losses.append(training_step(model, opt, loader, loss_fn=lambda m, xx: m_iwae(m, xx, K=3),
                                    multimodal=True))
    torch.cuda.synchronize()
    params = [p.detach().clone() for p in model.parameters()]
    _stepgraph.clear()
    return params, losses


if os.environ.get("NO_SIDE") == "1":
    from VAESNe import mmVAE
    mmVAE._side_stream = lambda t: None
if os.environ.get("NO_CTX") == "1":
    from VAESNe import util_layers
    util_layers._ctx_stream = lambda t, i=0: None
if os.environ.get("SIDE_ONLY"):
    # keep the side stream in one of forward's two branch blocks only (1: encoders +
    # decoder prepare, 2: decoders)
    from VAESNe import mmVAE
    _B = mmVAE._Branches
    cnt = [0]

    class _Sel(_B):
        def __init__(self, side):
            cnt[0] += 1
            super().__init__(side if str((cnt[0] - 1) % 2 + 1) == os.environ["SIDE_ONLY"] else None)
    mmVAE._Branches = _Sel
if os.environ.get("POISON"):
    # hold every float tensor each capture creates; fill them with NaN before each replay
    _cap = _stepgraph._capture
    PO = {}

    class _Hold(TorchDispatchMode):
        def __init__(self, lst):
            super().__init__()
            self.lst = lst

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            if any(r.alias_info is not None for r in func._schema.returns):
                return out
            for t in (out if isinstance(out, (tuple, list)) else [out]):
                if (torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32
                        and torch.cuda.is_current_stream_capturing()):
                    self.lst.append((t, func._schema.name))
            return out

    def _capture(ent, *a, **k):
        lst = []
        with _Hold(lst):
            ok = _cap(ent, *a, **k)
        if ok:
            PO[id(ent.graph)] = lst
        return ok
    _stepgraph._capture = _capture
    _rep0 = torch.cuda.CUDAGraph.replay

    def _replay_p(self):
        lst = PO.get(id(self), [])
        if os.environ["POISON"] == "1":
            for t, _ in lst:
                t.fill_(float("nan"))
        _rep0(self)
        torch.cuda.synchronize()
        bad = [(i, n) for i, (t, n) in enumerate(lst) if torch.isnan(t).all()]
        print(f"replay: {len(lst)} held, {len(bad)} still all-NaN", bad[:6])
    torch.cuda.CUDAGraph.replay = _replay_p
if os.environ.get("SYNC"):
    _rep = torch.cuda.CUDAGraph.replay

    def _replay(self):
        if os.environ["SYNC"] in ("before", "both"):
            torch.cuda.synchronize()
        _rep(self)
        if os.environ["SYNC"] in ("after", "both"):
            torch.cuda.synchronize()
    torch.cuda.CUDAGraph.replay = _replay
eager = run(False)
if KEEP != "none":
    with Keep():
        graph = run(True)
else:
    graph = run(True)
nd = sum(not torch.equal(a, b) for a, b in zip(eager[0], graph[0]))
if os.environ.get("SHOW_SKIPPED"):
    for e in SKIPPED:
        print("skipped", e)
print(f"allocs {CNT[0]} KEEP={KEEP} held={len(HELD)} losses eager {eager[1]} graph {graph[1]}; {nd} params differ")
