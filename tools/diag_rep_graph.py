"""Diagnostic (not product): the packed-VALU repeated-sequence attention forward
(vaesne_attn_rep_fwd, the decoders' block 1) captured on one stream beside split-f16
launches on another; inputs change before every replay, output compared with an isolated
eager launch on the same inputs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
from VAESNe import _lib, rng  # noqa: E402

lib = _lib.lib
DEV = "cuda"
H, E = 4, 32
P = float(os.environ.get("P", "0.0"))
Bd, R, L = int(os.environ.get("BD", "4")), int(os.environ.get("R", "6")), int(os.environ.get("L", "982"))
g = torch.Generator(device=DEV).manual_seed(1)
qkv = torch.randn(Bd, L, 3 * E, device=DEV, generator=g)
kb = torch.where(torch.rand(Bd, L, device=DEV, generator=g) < 0.05, float("-inf"), 0.0)
kb[:, 0] = 0.0
o = torch.empty(R * Bd, L, E, device=DEV)
lse = torch.empty(Bd, H, L, device=DEV)
st = rng.state(DEV).clone()
bits = torch.zeros(max(1, lib.attn_keep_bits_size(R * Bd, H, L, L) // 4), dtype=torch.int32, device=DEV)
# side load: split-f16 forwards of the context-path shape
SB, SL = int(os.environ.get("SB", "16")), int(os.environ.get("SL", "983"))
sq = torch.randn(SB, SL, 3 * E, device=DEV, generator=g)
so = torch.empty(SB, SL, E, device=DEV)
sl = torch.empty(SB, H, SL, device=DEV)
side = torch.cuda.Stream()


def rep(s):
    assert lib.attn_rep_fwd(qkv.data_ptr(), L * 3 * E, 3 * E, kb.data_ptr(), L, o.data_ptr(), L * E, E,
                            lse.data_ptr(), Bd, R, H, L, 8, P, st.data_ptr(), 7, bits.data_ptr(),
                            s.cuda_stream) == 0


A_ = torch.randn(2048, 2048, device=DEV, generator=g)
C_ = torch.empty(2048, 2048, device=DEV)


AGG = None
if os.environ.get("LOAD", "").startswith("agg"):
    import ctypes
    AGG = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libaggressors.so"))
    AGG_OUT = torch.empty(1 << 16, device=DEV)


def load(s):
    if AGG is not None:
        which = {"agg_mfma": 0, "agg_cvt": 1, "agg_perm": 2, "agg_exp": 3, "agg_mfma_all": 4}[os.environ["LOAD"]]
        for _ in range(int(os.environ.get("NS", "3"))):
            assert AGG.agg_launch(which, ctypes.c_void_p(AGG_OUT.data_ptr()), 1024,
                                  int(os.environ.get("ITERS", "20000")), ctypes.c_void_p(s.cuda_stream)) == 0
        return
    if os.environ.get("LOAD") == "gemm":
        for _ in range(int(os.environ.get("NS", "3"))):
            torch.mm(A_, A_, out=C_)
        return
    b = sq.data_ptr()
    for _ in range(int(os.environ.get("NS", "3"))):
        assert lib.attn_fwd(b, SL * 3 * E, 3 * E, b + 4 * E, SL * 3 * E, 3 * E, b + 8 * E, SL * 3 * E,
                            3 * E, None, SL, so.data_ptr(), SL * E, E, sl.data_ptr(), SB, H, SL, SL,
                            8, 0.0, None, 0, None, None, s.cuda_stream) == 0


load(torch.cuda.current_stream())     # warm (hipBLASLt's first call is not capturable)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    cap = torch.cuda.current_stream()
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        rep(side)
    load(cap)
    cap.wait_stream(side)
gen = torch.Generator(device=DEV).manual_seed(9)
if os.environ.get("EAGER"):
    class _G:
        def replay(self):
            cap = torch.cuda.current_stream()
            side.wait_stream(cap)
            with torch.cuda.stream(side):
                rep(side)
            load(cap)
            cap.wait_stream(side)
    gr = _G()
bad = 0
for r in range(int(os.environ.get("REPS", "40"))):
    qkv.add_(1e-3 * torch.randn(qkv.shape, device=DEV, generator=gen))
    torch.cuda.synchronize()
    rep(torch.cuda.current_stream())
    torch.cuda.synchronize()
    ref = (o.clone(), lse.clone())
    o.fill_(float("nan"))
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    if not (torch.equal(ref[0], o) and torch.equal(ref[1], lse)):
        bad += 1
        if bad <= 3:
            print("replay", r, float((ref[0] - o).abs().max()), float((ref[1] - lse).abs().max()))
            d = (ref[0] - o).abs().view(R, Bd, L, H, 8).amax(-1)     # [copy, seq, query, head]
            bad_idx = (d > 0).nonzero()
            print("   differing (copy, seq, query, head) entries:", bad_idx.shape[0], "of", d.numel(),
                  "copies", sorted(set(bad_idx[:, 0].tolist()))[:8], "seqs", sorted(set(bad_idx[:, 1].tolist())),
                  "heads", sorted(set(bad_idx[:, 3].tolist())), "queries", bad_idx[:, 2].min().item(), "-", bad_idx[:, 2].max().item())
            # which is right: fp64 reference of copy 0
            q = qkv[..., :E].double().cpu().view(Bd, L, H, 8).transpose(1, 2)
            k = qkv[..., E:2 * E].double().cpu().view(Bd, L, H, 8).transpose(1, 2)
            v = qkv[..., 2 * E:].double().cpu().view(Bd, L, H, 8).transpose(1, 2)
            S = q @ k.transpose(-1, -2) / 8 ** 0.5 + kb.double().cpu()[:, None, None, :]
            o64 = (torch.softmax(S, -1) @ v).transpose(1, 2).reshape(Bd, L, E)
            print("   err vs fp64: eager", float((ref[0][:Bd].double().cpu() - o64).abs().max()),
                  "graph", float((o[:Bd].double().cpu() - o64).abs().max()))
print(f"{bad} differing replays")
