"""Diagnostic (not product): two head_dim-8 attention forwards captured on two streams of
one hipGraph and replayed concurrently, against their eager one-stream results."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
from VAESNe import _lib, rng  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.lib
H, dh = 4, 8
E = H * dh
st = rng.state(dev)


def make(N, L, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    qkv = torch.randn(N, L, 3 * E, device=dev, generator=g)
    kb = torch.where(torch.rand(N, L, device=dev, generator=g) < 0.05, float("-inf"), 0.0)
    kb[:, 0] = 0.0
    o = torch.zeros(N, L, E, device=dev)
    lse = torch.zeros(N, H, L, device=dev)
    bits = torch.zeros(lib.attn_keep_bits_size(N, H, L, L) // 4, dtype=torch.int32, device=dev)
    b, s3 = qkv.data_ptr(), L * 3 * E

    def fwd(p):
        lib.attn_fwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E, kb.data_ptr(), L,
                     o.data_ptr(), L * E, E, lse.data_ptr(), N, H, L, L, dh, p, st.data_ptr(), 7,
                     bits.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    return fwd, (o, lse)


p = float(os.environ.get("PDROP", "0"))
lib.attn_force_geometry(*(int(v) for v in os.environ.get("GEO", "0,0").split(",")))
fa, outa = make(256, 982, 1)
fb, outb = make(256, 60, 2)
fa(p); fb(p)
torch.cuda.synchronize()
for rep in range(3):   # eager again, and two streams eagerly
    fa(p)
    torch.cuda.synchronize()
    print("eager rerun A equal:", [torch.equal(x, y.clone()) for x, y in zip(outa, outa)])
refa = [t.clone() for t in outa]
refb = [t.clone() for t in outb]
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
sa.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=sa):
    sb.wait_stream(sa)
    fa(p)
    with torch.cuda.stream(sb):
        for _ in range(3):
            fb(p)
    for _ in range(2):
        fa(p)
    sa.wait_stream(sb)
torch.cuda.synchronize()
for rep in range(6):
    for t in outa + outb:
        t.zero_()
    g.replay()
    torch.cuda.synchronize()
    print(f"replay {rep}: A equal {[torch.equal(a, b) for a, b in zip(refa, outa)]} "
          f"max {max(float((a - b).abs().max()) for a, b in zip(refa, outa)):.3g}; "
          f"B equal {[torch.equal(a, b) for a, b in zip(refb, outb)]}")
