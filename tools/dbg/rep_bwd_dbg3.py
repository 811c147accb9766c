"""debug: where the rep backward's dV differs from fp64"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
import torch
import test_gpu_rep_sf16 as T
from test_gpu_sf16 import _decode_bits
E, H = T.E, T.H
for (Bd, R, L, p) in [(1, 1, 37, 0.1), (1, 1, 37, 0.0), (1, 4, 300, 0.1)]:
    qkv, kb, do = T._inputs(Bd, R, L, 0.0, 3)
    N = R * Bd
    o, lse, bits, st = T._rep_fwd(qkv, kb, Bd, R, L, p, 5)
    if p > 0:
        rc, dx = T._rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)
    _, _, _, dpl = T._plain(qkv.repeat(R, 1, 1).contiguous(), None, do, N, L, p, 5, st)
    torch.cuda.synchronize()
    if p == 0:
        dx = dpl.view(R, Bd, L, 3 * E).sum(0)
    keep = _decode_bits(bits, N, L, L, True) if p > 0 else torch.ones(N, H, L, L, dtype=torch.bool)
    ro, rdx = T._dense64_rep(qkv, kb, do, keep, Bd, R, L, p)
    dsum = dpl.view(R, Bd, L, 3 * E).double().sum(0).cpu()
    a = dx.double().cpu()[..., 2 * E:]; b = rdx[..., 2 * E:]; c = dsum[..., 2 * E:]
    err = (a - b).abs(); errp = (c - b).abs()
    i = int(err.argmax())
    print(Bd, R, L, p, "rep dv maxerr", err.max().item(), "plain", errp.max().item(), "ref max", b.abs().max().item(),
          "at", [i // (L * E), (i // E) % L, i % E], "val", a.flatten()[i].item(), b.flatten()[i].item())
    # error per feature / per key
    print("   rep   err by feature", " ".join(f"{x:.0e}" for x in err.amax(dim=(0, 1)).tolist()))
    print("   plain err by feature", " ".join(f"{x:.0e}" for x in errp.amax(dim=(0, 1)).tolist()))
    print("   ref   max by feature", " ".join(f"{x:.0e}" for x in b.abs().amax(dim=(0, 1)).tolist()))
    print("   err by key (first 12)", [f"{x:.1e}" for x in err.amax(dim=(0, 2))[0:12].tolist()] if err.dim() == 3 else "")
