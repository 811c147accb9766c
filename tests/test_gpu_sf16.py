"""The split-f16 matrix-core attention (csrc/attention_sf16.hip), the default path for
head_dim 8 (util_layers.py:289 -> torch/nn/functional.py:6559-6594), against a dense fp64
attention and against the packed-fp32 VALU kernels (a forced geometry) on the same inputs
and the same dropout draws.

* the keep decisions are the VALU forward's, bit for bit (both hash each (query, key pair)
  with attn_pair_bits_mixed); only the bitmap layout differs;
* o / lse / dq / dk / dv against fp64 at the fp32 tolerances of test_gpu_kernels.py, and no
  worse than 4x the fp32 VALU kernel's own error (fp32-grade);
* the split product: lse (a log-sum of exp2 scores) within 2^-19 of max |S| of fp64 for
  inputs from 1e-5 to 1e4 (and q / k out of balance by 1e4 either way), o = v to 2^-20 |v|
  for a single key (P V alone), and o relative to fp64 at 2e-5 for v from 1e-5 to 1e4;
* bitwise reproducibility; several key blocks per sequence (Lk > 1024: dQ partials summed
  after the launch); ragged and fully masked sequences.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, DH = 4, 8
E = H * DH


def _lib():
    from VAESNe import _lib
    return _lib


def _decode_bits(bits, B, Lq, Lk, sf16, H=H):
    """dense keep [B, H, Lq, Lk] (bool) from a keep bitmap of either layout"""
    w = bits.cpu().numpy().view(np.uint32)
    if not sf16:
        nw = (Lk + 31) // 32
        w = w[:B * H * nw * Lq].reshape(B * H, nw, Lq)
        b = np.unpackbits(w.view(np.uint8), bitorder="little").reshape(B * H, nw, Lq, 32)
        keep = b.transpose(0, 2, 1, 3).reshape(B * H, Lq, nw * 32)[:, :, :Lk]
    else:
        nt8, lqp = (Lk + 127) // 128, (Lq + 15) // 16 * 16
        w = w[:B * H * nt8 * 4 * lqp].reshape(B * H, nt8, 4, lqp)[..., :Lq]
        b = np.unpackbits(w.view(np.uint8), bitorder="little").reshape(B * H, nt8, 4, Lq, 8, 4)
        # key = 128 T8 + 16 tt + 4 gq + r  <->  [T8][gq][q][tt][r]
        keep = b.transpose(0, 3, 1, 4, 2, 5).reshape(B * H, Lq, nt8 * 128)[:, :, :Lk]
    return torch.from_numpy(keep.astype(bool)).view(B, H, Lq, Lk)


def _run(q, k, v, kbias, do, p, cid, geo=(0, 0)):
    """forward + backward through the C ABI; returns (o, lse, bits, dq, dk, dv)"""
    _l = _lib()
    lib = _l.lib
    from VAESNe import rng
    B, Lq, Lk = q.shape[0], q.shape[1], k.shape[1]
    assert lib.attn_force_geometry(*geo) == 0
    try:
        st = rng.state(DEV)
        nbits = lib.attn_keep_bits_size(B, H, Lq, Lk) // 4
        bits = torch.zeros(nbits, dtype=torch.int32, device=DEV)
        wsn = max(lib.attn_workspace(B, H, Lq, Lk, DH, 0), lib.attn_workspace(B, H, Lq, Lk, DH, 1)) // 4
        ws = torch.empty(max(1, wsn), device=DEV)
        o = torch.empty(B, Lq, E, device=DEV)
        lse = torch.empty(B, H, Lq, device=DEV)
        kb = None if kbias is None else kbias.data_ptr()
        assert lib.attn_fwd(q.data_ptr(), Lq * E, E, k.data_ptr(), Lk * E, E, v.data_ptr(), Lk * E, E,
                            kb, Lk, o.data_ptr(), Lq * E, E, lse.data_ptr(), B, H, Lq, Lk, DH, p,
                            st.data_ptr(), cid, bits.data_ptr(), ws.data_ptr(), _l.stream()) == 0
        dq = torch.full((B, Lq, E), 7.0, device=DEV)
        dk = torch.full((B, Lk, E), 7.0, device=DEV)
        dv = torch.full((B, Lk, E), 7.0, device=DEV)
        assert lib.attn_bwd(q.data_ptr(), Lq * E, E, k.data_ptr(), Lk * E, E, v.data_ptr(), Lk * E, E,
                            kb, Lk, o.data_ptr(), Lq * E, E, lse.data_ptr(), do.data_ptr(), Lq * E, E,
                            dq.data_ptr(), Lq * E, E, dk.data_ptr(), Lk * E, E, dv.data_ptr(), Lk * E, E,
                            B, H, Lq, Lk, DH, p, st.data_ptr(), cid, bits.data_ptr(), ws.data_ptr(),
                            _l.stream()) == 0
        torch.cuda.synchronize()
    finally:
        lib.attn_force_geometry(0, 0)
    return o, lse, bits, dq, dk, dv


def _dense64(q, k, v, kbias, do, keep, p):
    """fp64 attention with the kernel's keep mask: o, lse (log2), dq, dk, dv"""
    B, Lq, Lk = q.shape[0], q.shape[1], k.shape[1]
    qr, kr, vr = (x.double().cpu().requires_grad_(True) for x in (q, k, v))
    qh = qr.view(B, Lq, H, DH).transpose(1, 2)
    kh = kr.view(B, Lk, H, DH).transpose(1, 2)
    vh = vr.view(B, Lk, H, DH).transpose(1, 2)
    S = qh @ kh.transpose(-1, -2) / math.sqrt(DH)
    if kbias is not None:
        S = S + kbias.double().cpu()[:, None, None, :]
    lse = torch.logsumexp(S, dim=-1) / math.log(2.0)
    P = torch.softmax(S, dim=-1)
    A = P * keep.double() / (1 - p) if p > 0 else P
    o = (A @ vh).transpose(1, 2).reshape(B, Lq, E)
    (o * do.double().cpu()).sum().backward()
    return o.detach(), lse.detach(), qr.grad, kr.grad, vr.grad


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    fin = torch.isfinite(b)
    return float((a[fin] - b[fin]).abs().max() / b[fin].abs().max().clamp_min(1e-30))


def _inputs(B, Lq, Lk, pm, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    q, k, v = (torch.randn(B, n, E, device=DEV, generator=g) * scale for n in (Lq, Lk, Lk))
    do = torch.randn(B, Lq, E, device=DEV, generator=g)
    kbias = None
    if pm > 0:
        kbias = torch.where(torch.rand(B, Lk, device=DEV, generator=g) < pm, float("-inf"), 0.0)
        kbias[:, 0] = 0.0
    return q, k, v, kbias, do


@pytest.mark.parametrize("B,Lq,Lk,pm,p", [(3, 982, 982, 0.05, 0.1), (2, 983, 983, 0.05, 0.1),
                                         (4, 60, 60, 0.1, 0.1), (2, 300, 257, 0.5, 0.1),
                                         (2, 37, 70, 0.0, 0.0), (2, 17, 1, 0.0, 0.1),
                                         (1, 130, 1100, 0.1, 0.1), (2, 200, 40, 0.0, 0.2)])
def test_sf16_matches_fp64_and_valu(B, Lq, Lk, pm, p):
    q, k, v, kbias, do = _inputs(B, Lq, Lk, pm, B * 1000 + Lq + Lk)
    cid = 4000 + Lq
    o, lse, bits, dq, dk, dv = _run(q, k, v, kbias, do, p, cid)
    ov, lsev, bitsv, dqv, dkv, dvv = _run(q, k, v, kbias, do, p, cid, geo=(256, 2))
    keep = _decode_bits(bits, B, Lq, Lk, True) if p > 0 else torch.ones(B, H, Lq, Lk, dtype=torch.bool)
    if p > 0:   # the same keep decisions as the packed-VALU forward
        assert torch.equal(keep, _decode_bits(bitsv, B, Lq, Lk, False))
        rate = 1 - keep.float().mean().item()
        assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / keep.numel()), rate
    ro, rl, rdq, rdk, rdv = _dense64(q, k, v, kbias, do, keep, p)
    tol = {"o": 2e-5, "lse": 1e-6, "dq": 1e-4, "dk": 1e-4, "dv": 1e-4}
    for name, got, val, ref in (("o", o, ov, ro), ("lse", lse, lsev, rl), ("dq", dq, dqv, rdq),
                                ("dk", dk, dkv, rdk), ("dv", dv, dvv, rdv)):
        if name in ("dq", "dk") and Lk == 1:   # softmax over one key is constant: both are 0
            assert got.abs().max().item() < 1e-5
            continue
        e, ev = _rel(got, ref), _rel(val, ref)
        assert e < tol[name], (name, e, ev)
        assert e <= max(4 * ev, 2e-6), (name, e, ev)


@pytest.mark.parametrize("scale,qk", [(1e-5, 1.0), (1e-3, 1.0), (0.1, 1.0), (1.0, 1.0), (10.0, 1.0),
                                      (100.0, 1.0), (1e4, 1.0), (1.0, 1e-4), (1.0, 3e4)])
def test_sf16_split_product_error_bound(scale, qk):
    """The split product hi hi + hi lo + lo hi: per row, |lse - lse_64| <= 2^-19 max|S2|
    (S2 = log2(e) q.k / sqrt(8)) + 2^-20 |lse| (fp32 exp2 / log2), across input magnitudes
    (q, k, v scaled by `scale`; then q by `qk` and k by 1 / qk: the power-of-two balance of
    q' and k' keeps both f16 splits normal); with one key o = v to 2^-20 |v| + 2^-38 max |v|
    of the (sequence, head) (the v' = v 2^ev range scale: relative precision at any
    magnitude, an absolute floor only for elements 2^-17 below the head's maximum)."""
    B, L = 2, 300
    q, k, v, _, do = _inputs(B, L, L, 0.0, 77, scale)
    q, k = q * qk, k / qk
    o, lse, _, _, _, _ = _run(q, k, v, None, do, 0.0, 1)
    qh = q.double().cpu().view(B, L, H, DH).transpose(1, 2)
    kh = k.double().cpu().view(B, L, H, DH).transpose(1, 2)
    S2 = qh @ kh.transpose(-1, -2) / math.sqrt(DH) / math.log(2.0)
    ref = torch.logsumexp(S2 * math.log(2.0), dim=-1) / math.log(2.0)
    bound = 2.0 ** -19 * S2.abs().amax(-1) + 2.0 ** -20 * ref.abs()   # + fp32 exp2 / log2
    assert ((lse.double().cpu() - ref).abs() <= bound).all(), ((lse.double().cpu() - ref).abs() / bound).max()
    o1, _, _, _, _, _ = _run(q, k[:, :1].contiguous(), v[:, :1].contiguous(), None, do, 0.0, 1)
    vv = v[:, :1].double().cpu().expand(B, L, E)
    err = (o1.double().cpu() - vv).abs()
    vmax = vv.view(B, L, H, DH).abs().amax(-1, keepdim=True).expand(B, L, H, DH).reshape(B, L, E)
    assert (err <= 2.0 ** -20 * vv.abs() + 2.0 ** -38 * vmax).all(), (err / vv.abs()).max()


@pytest.mark.parametrize("vscale", [1e-5, 1e-3, 1e4])
def test_sf16_o_relative_at_any_v_magnitude(vscale):
    """o over a full softmax (982 keys, dropout, padding) relative to fp64 at 2e-5 (the
    tolerance of test_sf16_matches_fp64_and_valu) when v is far from unit magnitude: the
    per-(sequence, head) v' = v 2^ev scale keeps the f16 hi / lo parts of v normal."""
    B, L = 2, 982
    q, k, v, kbias, do = _inputs(B, L, L, 0.05, 91)
    v = v * vscale
    o, _, bits, _, _, _ = _run(q, k, v, kbias, do, 0.1, 5)
    keep = _decode_bits(bits, B, L, L, True)
    ro = _dense64(q, k, v, kbias, do, keep, 0.1)[0]
    assert _rel(o, ro) < 2e-5, _rel(o, ro)


def test_sf16_bitwise_reproducible():
    q, k, v, kbias, do = _inputs(3, 982, 982, 0.05, 5)
    a = _run(q, k, v, kbias, do, 0.1, 99)
    b = _run(q, k, v, kbias, do, 0.1, 99)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_sf16_fully_masked_sequence_is_nan_like_reference():
    q, k, v, kbias, do = _inputs(2, 100, 100, 0.3, 6)
    kbias[1] = float("-inf")
    o, lse, _, dq, dk, dv = _run(q, k, v, kbias, do, 0.1, 3)
    assert torch.isfinite(o[0]).all() and torch.isnan(o[1]).all()
    assert torch.isneginf(lse[1]).all() and torch.isfinite(lse[0]).all()
    assert torch.isfinite(dq[0]).all() and torch.isfinite(dk[0]).all() and torch.isfinite(dv[0]).all()
