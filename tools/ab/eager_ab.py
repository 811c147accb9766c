"""A/B of the eager script loop (bench.training_step_script's 'eager' leg) between the
current training_util and a previous copy (tools/ab/training_util_prev.py), interleaved.
    python tools/ab/eager_ab.py"""
import importlib.util
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def load_prev():
    from VAESNe import training_util  # noqa: F401  (package context for relative imports)
    spec = importlib.util.spec_from_file_location(
        "VAESNe._training_util_prev", os.path.join(ROOT, "tools", "ab", "training_util_prev.py"))
    mod = importlib.util.module_from_spec(spec)
    mod.__package__ = "VAESNe"
    spec.loader.exec_module(mod)
    return mod.training_step


def run(ts, graph, batches=8, bs=16):
    from torch.utils.data import DataLoader, TensorDataset
    from VAESNe import _config, _stepgraph
    from VAESNe.data_util import multimodalDataset
    from VAESNe.losses import m_iwae
    dev = torch.device("cuda", 0)
    _config.step_graph = graph
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    opt = torch.optim.AdamW(model.parameters(), lr=bench.CFG["lr"])
    x = bench.synthetic_batch(bs * batches, 2024, "cpu")
    loader = DataLoader(multimodalDataset(TensorDataset(*x[0]), TensorDataset(*x[1])),
                        batch_size=bs, shuffle=False)
    fn = lambda m, xx: m_iwae(m, xx, K=bench.CFG["K"])
    ts(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    loss = ts(model, opt, loader, loss_fn=fn, multimodal=True)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / batches
    _stepgraph.clear(model)
    return dt * 1e3, math.isfinite(loss)


def main():
    from VAESNe.training_util import training_step as cur
    prev = load_prev()
    for rep in range(3):
        for name, ts in (("prev", prev), ("cur", cur)):
            for graph in (False, True):
                ms, ok = run(ts, graph)
                print(f"rep{rep} {name:5s} {'captured' if graph else 'eager':8s} {ms:7.3f} ms {ok}",
                      flush=True)


if __name__ == "__main__":
    main()
