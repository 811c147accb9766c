"""Diagnostic (not product): split-f16 forward of the spectra-decoder shape on the capture
stream beside photometry-decoder-shaped forwards on a side stream, captured as one graph;
the inputs change before every replay and the output is compared with an isolated eager
launch on the same inputs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
from VAESNe import _lib, rng  # noqa: E402

lib = _lib.lib
DEV = "cuda"
H, DH, E = 4, 8, 32
P = float(os.environ.get("P", "0.0"))


def bufs(B, L, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(B, L, 3 * E, device=DEV, generator=g)
    kb = torch.where(torch.rand(B, L, device=DEV, generator=g) < 0.05, float("-inf"), 0.0)
    kb[:, 0] = 0.0
    n = lib.attn_keep_bits_size(B, H, L, L) // 4
    return dict(qkv=qkv, kb=kb, B=B, L=L, st=rng.state(DEV).clone(),
                bits=torch.zeros(max(1, n), dtype=torch.int32, device=DEV),
                o=torch.empty(B, L, E, device=DEV), lse=torch.empty(B, H, L, device=DEV))


def fwd(d, cid, s):
    B, L = d["B"], d["L"]
    b = d["qkv"].data_ptr()
    assert lib.attn_fwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        d["kb"].data_ptr(), L, d["o"].data_ptr(), L * E, E, d["lse"].data_ptr(),
                        B, H, L, L, DH, P, d["st"].data_ptr(), cid, d["bits"].data_ptr(), None,
                        s.cuda_stream) == 0


side = torch.cuda.Stream()
spec = bufs(24, 982, 1)
phot = [bufs(24, 60, 2 + i) for i in range(3)]
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cap = torch.cuda.current_stream()
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        for i, d in enumerate(phot):
            fwd(d, 10 + i, side)
    fwd(spec, 5, cap)
    cap.wait_stream(side)
gen = torch.Generator(device=DEV).manual_seed(9)
bad = 0
for r in range(int(os.environ.get("R", "50"))):
    spec["qkv"].add_(1e-3 * torch.randn(spec["qkv"].shape, device=DEV, generator=gen))
    torch.cuda.synchronize()
    fwd(spec, 5, torch.cuda.current_stream())
    torch.cuda.synchronize()
    ref = (spec["o"].clone(), spec["lse"].clone())
    spec["o"].fill_(float("nan"))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    if not (torch.equal(ref[0], spec["o"]) and torch.equal(ref[1], spec["lse"])):
        bad += 1
        print("replay", r, float((ref[0] - spec["o"]).abs().max()), float((ref[1] - spec["lse"]).abs().max()))
print(f"{bad} differing replays")
