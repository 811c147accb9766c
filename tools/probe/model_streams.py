"""Probe (not product): the HIP stream handles the model's forward uses."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import mmVAE, util_layers  # noqa: E402
dev = torch.device("cuda", 0)
model = bench.make_model(dev, 0.0)
x = bench.synthetic_batch(4, 7, dev)
with torch.no_grad():
    model(x, K=3)
print("side", {k: hex(v.cuda_stream) for k, v in mmVAE._SIDE.items()})
print("ctx", {k: {i: hex(s.cuda_stream) for i, s in d.items()} for k, d in util_layers._CTX_STREAMS.items()})
