"""The decoders' first-block self-attention over R copies of each distinct sequence on the
split-f16 matrix cores (csrc/attention_sf16.hip: attn_fwd_sf16_kernel with copies,
attn_rep_bwd_sf16_kernel), the default for 16 < L <= 1024 (SpectraLayers.py:54-62,
PhotometricLayers.py:59-67; the reference runs every copy through nn.MultiheadAttention,
util_layers.py:289 -> torch/nn/functional.py:6559-6594).

* forward: o, lse and the keep bitmap BIT FOR BIT equal to the plain split-f16 forward on the
  expanded input (the same per-tile arithmetic: one shared score / exponential / split per
  distinct query tile, the plain kernel's keep decisions per copy), for every copies-per-
  workgroup configuration and ragged copy counts;
* backward: d(qkv) against an fp64 attention of every copy with its decoded keep mask, summed
  over the copies, at the split-f16 tolerances of test_gpu_sf16.py, and no worse than 4x the
  plain split-f16 backward of the expanded input; copy groups (R > 16), several query chunks,
  L at the 1024 limit; L = 1025 takes the packed-VALU kernels and still matches;
* the bitmap guard: a backward asked to read a bitmap the other kernel family wrote (the
  geometry override flipped between forward and backward) fails instead of reading it.
"""
import math

import pytest
import torch

from test_gpu_sf16 import _decode_bits

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, DH = 4, 8
E = H * DH


def _inputs(Bd, R, L, pm, seed):
    from VAESNe import _ops
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(Bd, L, 3 * E, device=DEV, generator=g)
    mask = None
    if pm > 0:
        mask = torch.rand(Bd, L, device=DEV, generator=g) < pm
        mask[:, 0] = False
    kb = _ops.key_bias(mask)
    do = torch.randn(R * Bd, L, E, device=DEV, generator=g)
    return qkv, kb, do


def _rep_fwd(qkv, kb, Bd, R, L, p, cid):
    from VAESNe import _lib, rng
    lib = _lib.lib
    N = R * Bd
    o = torch.full((N, L, E), float("nan"), device=DEV)
    lse = torch.empty(Bd, H, L, device=DEV)
    bits = torch.full((lib.attn_keep_bits_size(N, H, L, L) // 4,), -1, dtype=torch.int32, device=DEV)
    st = rng.state(DEV)
    assert lib.attn_rep_fwd(qkv.data_ptr(), L * 3 * E, 3 * E, None if kb is None else kb.data_ptr(), L,
                            o.data_ptr(), L * E, E, lse.data_ptr(), Bd, R, H, L, 8, p, st.data_ptr(),
                            cid, bits.data_ptr(), _lib.stream()) == 0
    return o, lse, bits, st


def _rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, cid):
    from VAESNe import _lib
    lib = _lib.lib
    dqkv = torch.full_like(qkv, 7.0)
    wsn = lib.attn_rep_workspace(Bd, R, H, L, 8, p) // 4
    ws = torch.empty(max(1, wsn), device=DEV)
    rc = lib.attn_rep_bwd(qkv.data_ptr(), L * 3 * E, 3 * E, None if kb is None else kb.data_ptr(), L,
                          o.data_ptr(), L * E, E, lse.data_ptr(), do.data_ptr(), dqkv.data_ptr(),
                          Bd, R, H, L, 8, p, st.data_ptr(), cid, bits.data_ptr(), ws.data_ptr(),
                          _lib.stream())
    return rc, dqkv


def _plain(qkv_full, kb_full, do, N, L, p, cid, st):
    """plain forward + backward of the expanded input through the C ABI"""
    from VAESNe import _lib
    lib = _lib.lib
    b = qkv_full.data_ptr()
    o = torch.empty(N, L, E, device=DEV)
    lse = torch.empty(N, H, L, device=DEV)
    bits = torch.full((lib.attn_keep_bits_size(N, H, L, L) // 4,), -1, dtype=torch.int32, device=DEV)
    wsn = max(lib.attn_workspace(N, H, L, L, 8, 0), lib.attn_workspace(N, H, L, L, 8, 1)) // 4
    ws = torch.empty(max(1, wsn), device=DEV)
    kbp = None if kb_full is None else kb_full.data_ptr()
    assert lib.attn_fwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        kbp, L, o.data_ptr(), L * E, E, lse.data_ptr(), N, H, L, L, 8, p,
                        st.data_ptr(), cid, bits.data_ptr(), ws.data_ptr(), _lib.stream()) == 0
    d = torch.full_like(qkv_full, 7.0)
    dp = d.data_ptr()
    assert lib.attn_bwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        kbp, L, o.data_ptr(), L * E, E, lse.data_ptr(), do.data_ptr(), L * E, E,
                        dp, L * 3 * E, 3 * E, dp + 4 * E, L * 3 * E, 3 * E, dp + 8 * E, L * 3 * E, 3 * E,
                        N, H, L, L, 8, p, st.data_ptr(), cid, bits.data_ptr(), ws.data_ptr(),
                        _lib.stream()) == 0
    return o, lse, bits, d


def _dense64_rep(qkv, kb, do, keep, Bd, R, L, p):
    """fp64 attention of every copy with its keep mask [R*Bd, H, L, L]: o, and d(qkv) summed
    over the copies"""
    x = qkv.double().cpu().requires_grad_(True)
    xf = x.repeat(R, 1, 1)
    N = R * Bd
    q, k, v = (xf[..., i * E:(i + 1) * E].reshape(N, L, H, DH).transpose(1, 2) for i in range(3))
    S = q @ k.transpose(-1, -2) / math.sqrt(DH)
    if kb is not None:
        S = S + kb.double().cpu().repeat(R, 1)[:, None, None, :]
    P = torch.softmax(S, dim=-1)
    A = P * keep.double() / (1 - p) if p > 0 else P
    o = (A @ v).transpose(1, 2).reshape(N, L, E)
    (o * do.double().cpu()).sum().backward()
    return o.detach(), x.grad


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    fin = torch.isfinite(b)
    return float((a[fin] - b[fin]).abs().max() / b[fin].abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("frc", [0, 4, 8, 16])
@pytest.mark.parametrize("Bd,R,L,pm,p", [(2, 16, 982, 0.05, 0.1), (3, 6, 60, 0.1, 0.1),
                                         (2, 5, 37, 0.0, 0.1), (1, 16, 300, 0.3, 0.0),
                                         (2, 1, 129, 0.05, 0.1), (1, 19, 200, 0.05, 0.1),
                                         (1, 3, 1024, 0.05, 0.1)])
def test_rep_sf16_forward_bitwise_equals_plain(frc, Bd, R, L, pm, p):
    from VAESNe import _lib
    lib = _lib.lib
    qkv, kb, do = _inputs(Bd, R, L, pm, 11 * L + R)
    N = R * Bd
    assert lib.attn_rep_sf16_config(frc, 256) == 0
    try:
        o1, l1, b1, st = _rep_fwd(qkv, kb, Bd, R, L, p, 4242)
        kb_full = None if kb is None else kb.repeat(R, 1).contiguous()
        o0, l0, b0, _ = _plain(qkv.repeat(R, 1, 1).contiguous(), kb_full, do, N, L, p, 4242, st)
        torch.cuda.synchronize()
    finally:
        lib.attn_rep_sf16_config(-1, 0)
    assert torch.equal(o0, o1)
    assert torch.equal(l0.view(R, Bd, H, L), l1.unsqueeze(0).expand(R, Bd, H, L))
    if p > 0:
        assert torch.equal(b0, b1)


@pytest.mark.parametrize("bwgs", [256, 1000])
@pytest.mark.parametrize("Bd,R,L,pm,p", [(2, 16, 982, 0.05, 0.1), (3, 6, 60, 0.1, 0.1),
                                         (2, 19, 37, 0.0, 0.1), (2, 16, 300, 0.3, 0.0),
                                         (1, 3, 983, 0.05, 0.1), (1, 33, 130, 0.1, 0.2),
                                         (1, 4, 1024, 0.0, 0.1), (1, 4, 1025, 0.05, 0.1)])
def test_rep_sf16_backward_matches_fp64(bwgs, Bd, R, L, pm, p):
    from VAESNe import _lib
    lib = _lib.lib
    qkv, kb, do = _inputs(Bd, R, L, pm, 7 * L + R)
    N = R * Bd
    cid = 700 + L
    assert lib.attn_rep_sf16_config(0, bwgs) == 0
    try:
        o, lse, bits, st = _rep_fwd(qkv, kb, Bd, R, L, p, cid)
        rc, dx = _rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, cid)
        assert rc == 0
        kb_full = None if kb is None else kb.repeat(R, 1).contiguous()
        _, _, _, dplain = _plain(qkv.repeat(R, 1, 1).contiguous(), kb_full, do, N, L, p, cid, st)
        torch.cuda.synchronize()
    finally:
        lib.attn_rep_sf16_config(-1, 0)
    sf16 = L <= 1024
    keep = _decode_bits(bits, N, L, L, sf16) if p > 0 else torch.ones(N, H, L, L, dtype=torch.bool)
    if p > 0:
        rate = 1 - keep.float().mean().item()
        assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / keep.numel()), rate
    ro, rdx = _dense64_rep(qkv, kb, do, keep, Bd, R, L, p)
    assert _rel(o, ro) < 2e-5
    dsum = dplain.view(R, Bd, L, 3 * E).double().sum(0)
    for name, sl in (("dq", slice(0, E)), ("dk", slice(E, 2 * E)), ("dv", slice(2 * E, 3 * E))):
        e, ep = _rel(dx[..., sl], rdx[..., sl]), _rel(dsum[..., sl], rdx[..., sl])
        assert e < 1e-4, (name, e, ep)
        assert e <= max(4 * ep, 2e-6), (name, e, ep)


def test_rep_sf16_backward_bitwise_reproducible():
    qkv, kb, do = _inputs(2, 16, 982, 0.05, 5)
    outs = []
    for _ in range(2):
        o, lse, bits, st = _rep_fwd(qkv, kb, 2, 16, 982, 0.1, 99)
        rc, dx = _rep_bwd(qkv, kb, o, lse, do, bits, st, 2, 16, 982, 0.1, 99)
        assert rc == 0
        outs.append((o, lse, bits, dx))
    torch.cuda.synchronize()
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_bitmap_family_guard():
    """A forward under one kernel family and the backward under the other (the geometry
    override flipped in between) would read the wrong keep bits: the backward refuses."""
    from VAESNe import _lib
    lib = _lib.lib
    Bd, R, L, p = 2, 4, 300, 0.1
    qkv, kb, do = _inputs(Bd, R, L, 0.05, 3)
    o, lse, bits, st = _rep_fwd(qkv, kb, Bd, R, L, p, 5)          # split-f16
    assert lib.attn_force_geometry(256, 1) == 0
    try:
        with pytest.raises(RuntimeError, match="hipError 1"):        # hipErrorInvalidValue
            _rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)   # packed-VALU reader
    finally:
        lib.attn_force_geometry(0, 0)
    rc, _ = _rep_bwd(qkv, kb, o, lse, do, bits, st, Bd, R, L, p, 5)
    assert rc == 0
    # the plain entry points: forward under the forced geometry, backward by default
    N = R * Bd
    qf = qkv.repeat(R, 1, 1).contiguous()
    kbf = kb.repeat(R, 1).contiguous()
    assert lib.attn_force_geometry(256, 1) == 0
    try:
        with pytest.raises(RuntimeError, match="hipError 1"):
            _plain_split(qf, kbf, do, N, L, p, st)
    finally:
        lib.attn_force_geometry(0, 0)
    torch.cuda.synchronize()


def _plain_split(qf, kbf, do, N, L, p, st):
    """forward now (whatever the geometry), backward after restoring the default"""
    from VAESNe import _lib
    lib = _lib.lib
    b = qf.data_ptr()
    o = torch.empty(N, L, E, device=DEV)
    lse = torch.empty(N, H, L, device=DEV)
    bits = torch.zeros(lib.attn_keep_bits_size(N, H, L, L) // 4, dtype=torch.int32, device=DEV)
    wsn = max(lib.attn_workspace(N, H, L, L, 8, 0), lib.attn_workspace(N, H, L, L, 8, 1)) // 4
    ws = torch.empty(max(1, wsn), device=DEV)
    assert lib.attn_fwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        kbf.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(), N, H, L, L, 8, p,
                        st.data_ptr(), 9, bits.data_ptr(), ws.data_ptr(), _lib.stream()) == 0
    lib.attn_force_geometry(0, 0)
    wsn = max(lib.attn_workspace(N, H, L, L, 8, 0), lib.attn_workspace(N, H, L, L, 8, 1)) // 4
    ws = torch.empty(max(1, wsn), device=DEV)
    d = torch.empty_like(qf)
    dp = d.data_ptr()
    lib.attn_bwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                      kbf.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(), do.data_ptr(), L * E, E,
                      dp, L * 3 * E, 3 * E, dp + 4 * E, L * 3 * E, 3 * E, dp + 8 * E, L * 3 * E, 3 * E,
                      N, H, L, L, 8, p, st.data_ptr(), 9, bits.data_ptr(), ws.data_ptr(), _lib.stream())
