"""debug: the split-f16 repeated-sequence backward against the plain one, per output"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
import torch
import test_gpu_rep_sf16 as T
for (Bd, R, L, pm, p) in [(1, 1, 37, 0.0, 0.1), (1, 2, 37, 0.0, 0.1), (1, 1, 300, 0.0, 0.1), (2, 16, 982, 0.05, 0.1)]:
    qkv, kb, do = T._inputs(Bd, R, L, pm, 3)
    N = R * Bd
    o, lse, bits, st = T._rep_fwd(qkv, kb, Bd, R, L, p, 5)
    rc, dx = T._rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)
    kbf = None if kb is None else kb.repeat(R, 1).contiguous()
    _, _, _, dpl = T._plain(qkv.repeat(R, 1, 1).contiguous(), kbf, do, N, L, p, 5, st)
    torch.cuda.synchronize()
    ds = dpl.view(R, Bd, L, 3 * T.E).sum(0)
    E = T.E
    for name, sl in (("dq", slice(0, E)), ("dk", slice(E, 2 * E)), ("dv", slice(2 * E, 3 * E))):
        a, b = dx[..., sl], ds[..., sl]
        print(Bd, R, L, name, "rel", T._rel(a, b), "n7", int((a == 7.0).sum()), "maxa", a.abs().max().item(), "maxb", b.abs().max().item())
        if name == "dq":
            err = (a - b).abs().amax(-1)   # [Bd, L]
            bad = (err > 1e-3 * b.abs().max()).nonzero()
            print("   bad rows", bad[:10].tolist(), len(bad))
