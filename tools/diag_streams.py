"""Diagnostic: gradients with the side streams on vs off (same process, same
inputs / noise) on a golden case; per key, which rows differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from conftest import build_model, golden_us, golden_x, load_golden  # noqa: E402


def grads(name, streams, ctx_streams="2"):
    from VAESNe import rng
    from VAESNe.losses import m_iwae
    os.environ["VAESNE_STREAMS"] = streams
    os.environ["VAESNE_CTX_STREAMS"] = ctx_streams
    g = load_golden(name)
    c = g["config"]
    model = build_model(c)
    model.train()
    x = golden_x(g, "cuda")
    with rng.inject_uniform(golden_us(g)):
        loss = -m_iwae(model, x, K=c["K"])
    loss.backward()
    torch.cuda.synchronize()
    return {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "mmvae_cfg5_b16"
    ref = grads(name, "0")
    for cs in ("1", "2", "4"):
        got = grads(name, "1", cs)
        print(f"== ctx streams {cs}")
        for k in ref:
            d = (got[k] - ref[k]).abs()
            if d.max() > 1e-3 * ref[k].abs().max():
                rows = (d.reshape(d.shape[0], -1).max(1).values > 1e-3 * ref[k].abs().max()).nonzero().flatten().tolist()
                print(f"  {k}: max diff {d.max():.4g} (ref max {ref[k].abs().max():.4g}); rows {rows[:8]}..{rows[-3:]} n={len(rows)}")
