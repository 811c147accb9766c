"""Diagnostic (not product): is the split-f16 attention bitwise stable when other kernels
share the GPU?  Runs forward + backward of the decoder-shaped attention alone (reference),
then repeatedly with a concurrent workload on a second stream (MODE=valu: the packed-VALU
attention on other data; sf16: the split-f16 attention on other data; gemm: torch.mm),
eagerly and as a captured two-stream graph, and compares every output bitwise."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd"), os.path.join(ROOT, "tests")]
from VAESNe import _lib, rng  # noqa: E402

lib = _lib.lib
DEV = "cuda"
H, DH = 4, 8
E = H * DH
B, L = int(os.environ.get("B", "24")), int(os.environ.get("L", "982"))
P = float(os.environ.get("P", "0.1"))
MODE = os.environ.get("MODE", "sf16")


def bufs(B, L, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    q, k, v, do = (torch.randn(B, L, E, device=DEV, generator=g) for _ in range(4))
    kb = torch.where(torch.rand(B, L, device=DEV, generator=g) < 0.05, float("-inf"), 0.0)
    kb[:, 0] = 0.0
    n = lib.attn_keep_bits_size(B, H, L, L) // 4
    ws = max(lib.attn_workspace(B, H, L, L, DH, 0), lib.attn_workspace(B, H, L, L, DH, 1)) // 4
    return dict(q=q, k=k, v=v, do=do, kb=kb, st=rng.state(DEV).clone(),
                bits=torch.zeros(n, dtype=torch.int32, device=DEV),
                ws=torch.empty(max(1, ws), device=DEV),
                o=torch.empty(B, L, E, device=DEV), lse=torch.empty(B, H, L, device=DEV),
                dq=torch.empty(B, L, E, device=DEV), dk=torch.empty(B, L, E, device=DEV),
                dv=torch.empty(B, L, E, device=DEV))


def attn(d, cid, stream):
    Bq = d["q"].shape[0]
    Lq = d["q"].shape[1]
    s = stream.cuda_stream
    a = (d["q"].data_ptr(), Lq * E, E, d["k"].data_ptr(), Lq * E, E, d["v"].data_ptr(), Lq * E, E,
         d["kb"].data_ptr(), Lq)
    assert lib.attn_fwd(*a, d["o"].data_ptr(), Lq * E, E, d["lse"].data_ptr(), Bq, H, Lq, Lq, DH, P,
                        d["st"].data_ptr(), cid, d["bits"].data_ptr(), d["ws"].data_ptr(), s) == 0
    assert lib.attn_bwd(*a, d["o"].data_ptr(), Lq * E, E, d["lse"].data_ptr(), d["do"].data_ptr(),
                        Lq * E, E, d["dq"].data_ptr(), Lq * E, E, d["dk"].data_ptr(), Lq * E, E,
                        d["dv"].data_ptr(), Lq * E, E, Bq, H, Lq, Lq, DH, P, d["st"].data_ptr(), cid,
                        d["bits"].data_ptr(), d["ws"].data_ptr(), s) == 0


def snap(d):
    return [d[n].clone() for n in ("o", "lse", "dq", "dk", "dv", "bits")]


main = torch.cuda.current_stream()
side = torch.cuda.Stream()
d = bufs(B, L, 1)
other = bufs(int(os.environ.get("OB", "24")), int(os.environ.get("OL", "982")), 2)
A = torch.randn(4096, 4096, device=DEV)


def concurrent():
    if MODE == "gemm":
        with torch.cuda.stream(side):
            for _ in range(4):
                torch.mm(A, A)
    else:
        if MODE == "valu":
            assert lib.attn_force_geometry(256, 2) == 0
        attn(other, 7, side)
        lib.attn_force_geometry(0, 0)


attn(d, 5, main)
torch.cuda.synchronize()
ref = snap(d)
bad = 0
for it in range(int(os.environ.get("ITERS", "30"))):
    for n in ("o", "lse", "dq", "dk", "dv", "bits"):
        d[n].fill_(7.0 if n != "bits" else 0)
    torch.cuda.synchronize()
    side.wait_stream(main)
    concurrent()
    attn(d, 5, main)
    torch.cuda.synchronize()
    diff = [n for n, a, b in zip(("o", "lse", "dq", "dk", "dv", "bits"), ref, snap(d)) if not torch.equal(a, b)]
    if diff:
        bad += 1
        print("eager iter", it, "differs:", diff)
print(f"eager MODE={MODE}: {bad} differing iterations")

# captured: the concurrent workload on a forked stream inside the graph
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    concurrent()
    attn(d, 5, cur)
    cur.wait_stream(side)
bad = 0
for it in range(int(os.environ.get("ITERS", "30"))):
    for n in ("o", "lse", "dq", "dk", "dv", "bits"):
        d[n].fill_(7.0 if n != "bits" else 0)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    diff = [(n, float((a.float() - b.float()).abs().max())) for n, a, b in
            zip(("o", "lse", "dq", "dk", "dv", "bits"), ref, snap(d)) if not torch.equal(a, b)]
    if diff:
        bad += 1
        print("graph replay", it, "differs:", diff)
print(f"graph MODE={MODE}: {bad} differing replays")
