"""Which Python lines launch the aten kernels (copies, cat, add, fill, neg, ...) left
between the HIP kernels of bench.py's training step?  Runs eager steps of bench.Step
under torch.profiler with Python stacks and prints, per aten op that launched a GPU
kernel, the count and the innermost frames of the package / bench.
    python tools/glue_probe.py > gpurun_out/glue.txt"""
import collections
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))

import bench  # noqa: E402

GLUE = ("aten::copy_", "aten::cat", "aten::add", "aten::add_", "aten::fill_", "aten::neg",
        "aten::zero_", "aten::mul", "aten::sub", "aten::sum", "aten::clone", "aten::contiguous",
        "aten::zeros", "aten::ones", "aten::full", "aten::stack", "aten::index", "aten::where")


class _Glue(torch.utils._python_dispatch.TorchDispatchMode):
    """Counts the aten ops on device tensors by the package / bench lines that issue them."""

    def __init__(self):
        super().__init__()
        self.where = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket.__name__)
        dev = any(isinstance(a, torch.Tensor) and a.is_cuda
                  for a in list(args) + list((kwargs or {}).values()))
        if dev and any(g in name for g in ("copy", "clone", "cat", "add", "fill", "neg", "zero",
                                           "mul", "sub", "sum", "stack", "where", "index",
                                           "contiguous", "expand", "repeat")):
            fr = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno} {f.name}"
                  for f in traceback.extract_stack()
                  if ("VAESNe" in f.filename or "bench.py" in f.filename)]
            node = torch._C._current_autograd_node()
            shp = ";".join(f"{tuple(a.shape)}/{a.stride()}" for a in args
                           if isinstance(a, torch.Tensor))[:120]
            self.where[(name, " <- ".join(reversed(fr[-3:])) +
                        (f" [node {node.name()}]" if node is not None else "") + f" {{{shp}}}")] += 1
        return func(*args, **(kwargs or {}))


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = bench.make_model(dev, bench.CFG["dropout"])
    x = bench.synthetic_batch(16, 0, dev)
    step = bench.Step(model, x, dev, 1, use_graph=False)
    for _ in range(3):
        step.eager()
    torch.cuda.synchronize()
    mode = _Glue()
    with mode:
        step.eager()
    torch.cuda.synchronize()
    for (name, fr), n in sorted(mode.where.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:14s} {fr}")


if __name__ == "__main__":
    main()
