"""debug: dump dS'', acc, CD of the rep backward (VAESNE_REPBWD_DBG build) vs fp64"""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
import torch
import test_gpu_rep_sf16 as T
from test_gpu_sf16 import _decode_bits
Bd, R, L, p = 1, 1, 37, 0.1
E, H = T.E, T.H
qkv, kb, do = T._inputs(Bd, R, L, 0.0, 3)
o, lse, bits, st = T._rep_fwd(qkv, kb, Bd, R, L, p, 5)
rc, dx = T._rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)
torch.cuda.synchronize()
keep = _decode_bits(bits, 1, L, L, True)[0].double()   # [H, L, L]
x = qkv.double().cpu()[0]
q, k, v = (x[:, i * E:(i + 1) * E].view(L, H, 8).transpose(0, 1) for i in range(3))
S = q @ k.transpose(-1, -2) / math.sqrt(8)
P = torch.softmax(S, -1)
dO = do.double().cpu()[0].view(L, H, 8).transpose(0, 1)
O = o.double().cpu()[0].view(L, H, 8).transpose(0, 1)
dP = dO @ v.transpose(-1, -2)
D = (dO * O).sum(-1)
sd = 1 / (1 - p)
dS = P * (keep * sd * dP - D[..., None])
dx = dx.cpu().double()[0]
for h in range(1):
    s = dx[0, 2 * E + h * 8 + 1].item()
    print("s", s)
    kd = dx[:, h * 8:h * 8 + 8]                 # dS'' [q, key 0..7]
    ka = dx[:, E + h * 8:E + h * 8 + 8]         # acc
    kc = dx[:, 2 * E + h * 8]                   # CD
    f = 2.0 ** (14 + s)
    for qq in range(8):
        print(qq, "dS ratio", [round((kd[qq, j] / (f * dS[h, qq, j])).item(), 4) for j in range(4)],
              "acc ratio", [round((ka[qq, j] / (2 ** s * keep[h, qq, j] * sd * dP[h, qq, j])).item(), 4) if keep[h, qq, j] else float(ka[qq, j]) for j in range(4)],
              "CD ratio", round((kc[qq] / (-(2 ** s) * D[h, qq])).item(), 4))
