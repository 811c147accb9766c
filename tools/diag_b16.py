"""Diagnostic: per-parameter gradient errors of the HIP build vs the reference's
golden gradient norms on a golden case (default mmvae_cfg5_b16), optionally with
the side streams off (VAESNE_STREAMS=0) and repeated to expose nondeterminism."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from conftest import build_model, golden_us, golden_x, load_golden  # noqa: E402


def run(name):
    from VAESNe import rng
    from VAESNe.losses import m_iwae
    g = load_golden(name)
    c = g["config"]
    model = build_model(c)
    model.train()
    x = golden_x(g, "cuda")
    with rng.inject_uniform(golden_us(g)):
        loss = -m_iwae(model, x, K=c["K"])
    loss.backward()
    torch.cuda.synchronize()
    params = dict(model.named_parameters())
    names = json.loads(str(g["grad_names"]))
    errs = []
    for k, n in zip(names, g["grad_norms"]):
        errs.append((abs(params[k].grad.norm().item() - n) / max(n, 1e-3), k, params[k].grad.norm().item(), n))
    errs.sort(reverse=True)
    return loss.item(), float(g["loss"]), errs, {k: p.grad.clone() for k, p in params.items() if p.grad is not None}


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "mmvae_cfg5_b16"
    print("VAESNE_STREAMS", os.environ.get("VAESNE_STREAMS", "1"), flush=True)
    prev = None
    for rep in range(2):
        l, ref, errs, grads = run(name)
        print(f"rep {rep} loss {l:.6f} ref {ref:.6f} rel {abs(l-ref)/abs(ref):.2e}")
        for e in errs[:8]:
            print("   %.3e %s build %.6g ref %.6g" % e)
        nbad = sum(1 for e in errs if e[0] > 1e-3)
        print("   keys over 1e-3:", nbad, "of", len(errs))
        if prev is not None:
            d = max(float((grads[k] - prev[k]).abs().max()) for k in grads if grads[k] is not None)
            print("   max |grad(rep1) - grad(rep0)| =", d)
        prev = grads
