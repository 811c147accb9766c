"""Encoder context self-attention (cfg 5: B=16 sequences x 983 tokens, 4 heads, dh 8,
dropout 0.1): four per-block launches of B=16 against one batch-stacked launch of B=64."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "vaesne-dev_amd"))
import torch
from VAESNe import _ops

dev = "cuda"
L, E, H = 983, 32, 4
g = torch.Generator(device=dev).manual_seed(0)


def case(B, reps):
    qkv = torch.randn(B, L, 3 * E, device=dev, generator=g).requires_grad_(True)
    mask = torch.rand(B, L, device=dev, generator=g) < 0.05
    mask[:, 0] = False
    kb = _ops.key_bias_of(mask)
    do = torch.randn(B, L, E, device=dev, generator=g)

    def run():
        for _ in range(reps):
            o = _ops.self_attention(qkv, None, H, 0.1, kbias=kb)
            (dq,) = torch.autograd.grad(o, qkv, do)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    t0.record()
    for _ in range(n):
        run()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / n


for rep in range(2):
    a = case(16, 4)
    b = case(64, 1)
    print(f"4 x B=16: {a * 1e3:.1f} us   1 x B=64: {b * 1e3:.1f} us", flush=True)
