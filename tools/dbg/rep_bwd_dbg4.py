"""debug: decompose the worst dV element of the rep backward into per-query terms"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
import torch
import test_gpu_rep_sf16 as T
from test_gpu_sf16 import _decode_bits
E, H = T.E, T.H
Bd, R, L, p = 1, 1, 37, 0.1
qkv, kb, do = T._inputs(Bd, R, L, 0.0, 3)
o, lse, bits, st = T._rep_fwd(qkv, kb, Bd, R, L, p, 5)
rc, dx = T._rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)
torch.cuda.synchronize()
keep = _decode_bits(bits, 1, L, L, True)[0].double()
ro, rdx = T._dense64_rep(qkv, kb, do, keep[None], Bd, R, L, p)
a = dx.double().cpu()[0, :, 2 * E:]; b = rdx[0, :, 2 * E:]
err = (a - b).abs()
i = int(err.argmax()); k, f = i // E, i % E
h, ff = f // 8, f % 8
print("worst", k, f, "got", a[k, f].item(), "ref", b[k, f].item(), "diff", (a[k, f] - b[k, f]).item())
x = qkv.double().cpu()[0]
q_, k_ = (x[:, j * E:(j + 1) * E].view(L, H, 8).transpose(0, 1) for j in range(2))
P = torch.softmax(q_ @ k_.transpose(-1, -2) / math.sqrt(8), -1)[h]    # [L, L]
dO = do.double().cpu()[0].view(L, H, 8)[:, h, ff]
sd = 1 / (1 - p)
terms = P[:, k] * keep[h, :, k] * sd * dO
print("sum terms", terms.sum().item())
for qq in range(L):
    print(qq, f"P {P[qq, k].item():.3e} keep {int(keep[h, qq, k])} dO {dO[qq].item():+.3f} term {terms[qq].item():+.3e} flip {(P[qq, k] * sd * dO[qq]).item():+.3e}")
