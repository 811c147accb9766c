"""Run the operand-map probe (tools/probe/mfma_probe.hip) on the GPU; prints PASS/FAIL lines."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libmfma_probe.so"))
for f in ("probe_mfma", "probe_tr16"):
    getattr(lib, f).argtypes = [C.c_void_p] * 4 if f == "probe_mfma" else [C.c_void_p] * 3
lib.probe_split.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
dev = torch.device("cuda")
st = torch.cuda.current_stream().cuda_stream
ok = True
# 1. MFMA map, asymmetric integer data
A = torch.randint(-3, 4, (16, 32)).float()
B = torch.randint(-3, 4, (32, 16)).float()
D = torch.zeros(16, 16, device=dev)
lib.probe_mfma(A.half().to(dev).data_ptr(), B.half().to(dev).data_ptr(), D.data_ptr(), st)
torch.cuda.synchronize()
good = torch.equal(D.cpu(), A @ B)
print("mfma_f32_16x16x32_f16 map:", "PASS" if good else "FAIL")
ok &= good
# 2. transposed read
M = torch.arange(256, dtype=torch.int16).view(16, 16)
out = torch.zeros(64, 4, dtype=torch.int16, device=dev)
lib.probe_tr16(M.to(dev).data_ptr(), out.data_ptr(), st)
torch.cuda.synchronize()
o = out.cpu()
exp = torch.zeros(64, 4, dtype=torch.int16)
for l in range(64):
    g, i = l >> 4, l & 15
    for q in range(4):
        exp[l, q] = M[4 * g + q, i]
good = torch.equal(o, exp)
print("ds_read_b64_tr_b16 map:", "PASS" if good else "FAIL")
if not good:
    print(o[:20].tolist())
ok &= good
# 3. split: x = hi + lo to 2^-22 relative over the normal range
x = torch.cat([torch.randn(1 << 20) * s for s in (1e-3, 1.0, 1e3)]).to(dev)
n = x.numel()
hi = torch.zeros(n // 2, dtype=torch.int32, device=dev)
lo = torch.zeros_like(hi)
lib.probe_split(x.data_ptr(), hi.data_ptr(), lo.data_ptr(), n, st)
torch.cuda.synchronize()
h = hi.view(torch.float16).float()
lw = lo.view(torch.float16).float()
rec = (h.double() + lw.double())
err = ((rec - x.double()).abs() / x.double().abs().clamp_min(1e-30))
big = x.abs() > 2.0 ** -3
print("split rel err (|x| > 1/8): max %.3g (2^%.1f); hi == RNE f16: %s" % (
    err[big].max().item(), np.log2(err[big].max().item()), torch.equal(h, x.half().float())))
ok &= bool(err[big].max().item() <= 2.0 ** -21) and torch.equal(h, x.half().float())
# 4. raw fragments: which k does element j of lane group g carry (A and B alike)?
lib.probe_raw.argtypes = [C.c_void_p] * 4
Af = torch.randint(-3, 4, (64, 8)).float()
Bf = torch.randint(-3, 4, (64, 8)).float()
Df = torch.zeros(64, 4, device=dev)
lib.probe_raw(Af.half().to(dev).data_ptr(), Bf.half().to(dev).data_ptr(), Df.data_ptr(), st)
torch.cuda.synchronize()
Df = Df.cpu()
cands = {"8g+j": lambda g, j: 8 * g + j,
         "4g+j | 16+4g+j-4": lambda g, j: 4 * g + j if j < 4 else 16 + 4 * g + (j - 4),
         "2-interleave": lambda g, j: 4 * g + (j % 4) + 16 * (j // 4)}
for name, km in cands.items():
    A = torch.zeros(16, 32); B = torch.zeros(32, 16)
    for l in range(64):
        for j in range(8):
            A[l % 16, km(l // 16, j)] = Af[l, j]
            B[km(l // 16, j), l % 16] = Bf[l, j]
    D = A @ B
    got = torch.zeros(16, 16)
    for l in range(64):
        for r in range(4):
            got[4 * (l // 16) + r, l % 16] = Df[l, r]
    print("candidate k map", name, ":", "MATCH" if torch.equal(got, D) else "no")
# 5. slot pairing: A ones in every lane of group g at element j, B slot codes 1 + 8 lane + jj
res = {}
for g in range(4):
    for j in range(8):
        Af = torch.zeros(64, 8)
        Af[16 * g:16 * g + 16, j] = 1.0
        Bf = (1 + torch.arange(512)).float().view(64, 8)
        Df = torch.zeros(64, 4, device=dev)
        lib.probe_raw(Af.half().to(dev).data_ptr(), Bf.half().to(dev).data_ptr(), Df.data_ptr(), st)
        torch.cuda.synchronize()
        res[f"{g},{j}"] = Df.cpu().int().tolist()
import json
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/mfma_slots.json", "w"))
for key in ("0,0", "0,4", "1,0", "3,7"):
    v = res[key]
    print("A ones at group,elem", key, "-> D lane0..3 regs:", v[0], v[1], "lane16:", v[16], "lane32:", v[32])
print("ALL", "PASS" if ok else "FAIL")
sys.exit(0 if ok else 1)
