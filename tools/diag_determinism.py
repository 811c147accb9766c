"""Diagnostic (not product): is the eager training step bitwise reproducible?  Runs the
bench model's forward + backward several times on the same inputs / draws and compares
gradients; VAESNE_STREAMS=0 in the environment gives the one-stream variant."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _lib, rng  # noqa: E402
from VAESNe.losses import m_iwae  # noqa: E402

dev = torch.device("cuda", 0)
geo = tuple(int(v) for v in os.environ.get("GEO", "0,0").split(","))
_lib.lib.attn_force_geometry(*geo)
torch.manual_seed(0)
model = bench.make_model(dev, 0.1)
x = bench.synthetic_batch(int(os.environ.get("B", "4")), 7, dev)
res = []
for rep in range(4):
    rng.manual_seed(99)
    for p in model.parameters():
        p.grad = None
    loss = -m_iwae(model, x, K=3)
    loss.backward()
    torch.cuda.synchronize()
    res.append((loss.item(), [p.grad.clone() if p.grad is not None else None for p in model.parameters()]))
names = [n for n, _ in model.named_parameters()]
for r in range(1, len(res)):
    diff = [n for n, a, b in zip(names, res[0][1], res[r][1])
            if a is not None and not torch.equal(a, b)]
    print(f"rep {r}: loss {res[r][0]!r} vs {res[0][0]!r}; differing grads: {len(diff)} {diff[:6]}")
