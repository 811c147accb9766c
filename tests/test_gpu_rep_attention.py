"""The decoders' first-block self-attention over R copies of each distinct sequence
(vaesne_attn_rep_fwd / _bwd, _ops.self_attention_rep) against the plain attention
kernels on the expanded input (the reference computes every copy separately:
SpectraVAE.py:189-192 expands z and the decoder embeds the expanded grid).

* forward, same geometry: o, lse and the dropout keep bitmap bit for bit (here the
  packed-VALU kernels under a forced geometry; the default split-f16 kernels in
  tests/test_gpu_rep_sf16.py);
* backward: d(qkv) equals the plain backward's gradients summed over the copies
  (summation order differs: max-abs-relative 1e-5), with and without dropout, for
  every kernel configuration, ragged copy batches (R % RC != 0), masked keys and
  short / odd sequence lengths;
* the whole decoder (decoder_stack with rep) and a training step of the MMVAE equal
  the expanded path for the same dropout call ids."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, E = 4, 32


def _rel(a, b):
    a = a.detach().double()
    b = b.detach().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _inputs(Bd, R, L, pm, seed):
    from VAESNe import _ops
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkv = torch.randn(Bd, L, 3 * E, device=DEV, generator=g)
    mask = None
    if pm > 0:
        mask = torch.rand(Bd, L, device=DEV, generator=g) < pm
        mask[:, 0] = False
    kb = _ops.key_bias(mask)
    kb_full = None if kb is None else kb.repeat(R, 1).contiguous()
    return qkv, kb, kb_full, qkv.repeat(R, 1, 1).contiguous()


def _plain_fwd(lib, qkv, kb, N, L, p, st, cid):
    from VAESNe import _lib
    o = torch.empty(N, L, E, device=DEV)
    lse = torch.empty(N, H, L, device=DEV)
    bits = torch.full((lib.attn_keep_bits_size(N, H, L, L) // 4,), -1, dtype=torch.int32, device=DEV)
    b = qkv.data_ptr()   # no workspace: one unsplit launch (a split one sums key chunks)
    rc = lib.attn_fwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                      None if kb is None else kb.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(),
                      N, H, L, L, 8, p, st.data_ptr(), cid, bits.data_ptr(), None,
                      _lib.stream())
    assert rc == 0
    return o, lse, bits


def _rep_fwd(lib, qkv, kb, Bd, R, L, p, st, cid):
    from VAESNe import _lib
    N = R * Bd
    o = torch.full((N, L, E), float("nan"), device=DEV)
    lse = torch.empty(Bd, H, L, device=DEV)
    bits = torch.full((lib.attn_keep_bits_size(N, H, L, L) // 4,), -1, dtype=torch.int32, device=DEV)
    rc = lib.attn_rep_fwd(qkv.data_ptr(), L * 3 * E, 3 * E, None if kb is None else kb.data_ptr(), L,
                          o.data_ptr(), L * E, E, lse.data_ptr(), Bd, R, H, L, 8, p, st.data_ptr(),
                          cid, bits.data_ptr(), _lib.stream())
    assert rc == 0
    return o, lse, bits


@pytest.mark.parametrize("fnp,frc", [(1, 2), (1, 4), (1, 8), (2, 2), (2, 4)])
@pytest.mark.parametrize("Bd,R,L,pm,p", [(2, 16, 982, 0.05, 0.1), (3, 6, 60, 0.1, 0.1),
                                         (2, 5, 37, 0.0, 0.1), (1, 16, 300, 0.3, 0.0),
                                         (2, 1, 129, 0.05, 0.1)])
def test_rep_forward_bitwise_equals_plain_forward(fnp, frc, Bd, R, L, pm, p):
    """Same query-to-wave mapping (plain geometry 256 x fnp = rep forward at 256
    threads x fnp): identical arithmetic per copy, so o, lse and the bitmap are equal."""
    from VAESNe import _lib, rng
    lib = _lib.lib
    qkv, kb, kb_full, qkv_full = _inputs(Bd, R, L, pm, 11 * L + R)
    st = rng.state(DEV)
    N = R * Bd
    assert lib.attn_force_geometry(256, fnp) == 0
    assert lib.attn_rep_config(256, frc, 256, 1, 16, 768, fnp) == 0
    try:
        o0, l0, b0 = _plain_fwd(lib, qkv_full, kb_full, N, L, p, st, 4242)
        o1, l1, b1 = _rep_fwd(lib, qkv, kb, Bd, R, L, p, st, 4242)
        torch.cuda.synchronize()
    finally:
        lib.attn_force_geometry(0, 0)
        lib.attn_rep_config(-1, 0, 0, 0, 0, 0, 0)
    assert torch.equal(o0, o1)
    assert torch.equal(l0.view(R, Bd, H, L), l1.unsqueeze(0).expand(R, Bd, H, L))
    if p > 0:
        assert torch.equal(b0, b1)


@pytest.mark.parametrize("cfg", [(0, 4, 256, 1, 16, 768, 1), (64, 8, 128, 2, 8, 64, 1),
                                 (128, 2, 256, 2, 16, 4000, 2), (0, 4, 128, 1, 8, 300, 2)])
@pytest.mark.parametrize("Bd,R,L,pm,p", [(2, 16, 982, 0.05, 0.1), (3, 6, 60, 0.1, 0.1),
                                         (2, 19, 37, 0.0, 0.1), (2, 16, 300, 0.3, 0.0),
                                         (1, 3, 983, 0.05, 0.1)])
def test_rep_backward_equals_summed_plain_backward(cfg, Bd, R, L, pm, p):
    """the packed-VALU kernels (a forced geometry selects them on both paths; the default
    split-f16 ones: tests/test_gpu_rep_sf16.py)"""
    from VAESNe import _lib, _ops, rng
    lib = _lib.lib
    assert lib.attn_rep_config(*cfg) == 0
    assert lib.attn_force_geometry(256, 1) == 0
    try:
        qkv, kb, kb_full, qkv_full = _inputs(Bd, R, L, pm, 7 * L + R + cfg[1])
        g = torch.Generator(device=DEV).manual_seed(L + 3)
        do = torch.randn(R * Bd, L, E, device=DEV, generator=g)
        res = []
        for rep in (False, True):
            rng._call = 700
            x = (qkv if rep else qkv_full).clone().requires_grad_(True)
            if rep:
                o = _ops.self_attention_rep(x, kb, H, p, R)
            else:
                o = _ops.self_attention(x, None, H, p, kbias=kb_full)
            o.backward(do)
            dx = x.grad if rep else x.grad.view(R, Bd, L, 3 * E).double().sum(0)
            res.append((o.detach(), dx))
        torch.cuda.synchronize()
    finally:
        lib.attn_rep_config(-1, 0, 0, 0, 0, 0, 0)
        lib.attn_force_geometry(0, 0)
    (o0, d0), (o1, d1) = res
    assert _rel(o1, o0) < 1e-5     # plain launch may split the key axis (chunk combine)
    for sl in (slice(0, E), slice(E, 2 * E), slice(2 * E, 3 * E)):     # dQ, dK, dV
        assert _rel(d1[..., sl], d0[..., sl]) < 1e-5, (sl, _rel(d1[..., sl], d0[..., sl]))


def test_rep_decoder_stack_and_model_step_equal_expanded_path(monkeypatch):
    """A cfg-5-shaped MMVAE training step (dropout on) with the repeated first-block
    attention against _config.rep_attn off (expanded input, plain kernels): the same
    dropout call ids, so the loss agrees to fp32 summation order (1e-5) and so do
    the gradients, up to the importance weights: lw sums ~10^3 log-probabilities, so
    a 1e-7 relative change in a decoder location moves lw by ~1e-4 and the softmax
    weights over the K samples by as much (gradients max-abs-relative 2e-3).  The
    repeated path itself is bitwise reproducible (a stream race would not be)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from VAESNe import _config, rng
    from VAESNe.losses import m_iwae
    torch.manual_seed(3)
    model = bench.make_model(DEV, 0.1)
    model.train()
    x = bench.synthetic_batch(2, 5, DEV)
    outs = []
    for flag in ("0", "1", "1"):
        monkeypatch.setattr(_config, "rep_attn", flag == "1")
        model.zero_grad(set_to_none=True)
        rng.manual_seed(77)
        loss = -m_iwae(model, x, K=3)
        loss.backward()
        outs.append((loss.item(), {n: p.grad.detach().clone() for n, p in model.named_parameters()
                                   if p.grad is not None}))
    (l0, g0), (l1, g1), (l2, g2) = outs
    assert abs(l1 - l0) <= 1e-5 * abs(l0)
    assert g0.keys() == g1.keys() == g2.keys()
    assert l1 == l2
    for n in g0:
        assert torch.equal(g1[n], g2[n]), n
        assert _rel(g1[n], g0[n]) < 2e-3, (n, _rel(g1[n], g0[n]))


@pytest.mark.parametrize("parts", [(1, 2), (2, 3), (1, 3), (3, 4)])
@pytest.mark.parametrize("Bd,R,L,p", [(2, 16, 982, 0.1), (3, 6, 60, 0.1), (2, 4, 300, 0.0)])
def test_rep_forward_in_parts_equals_one_launch(parts, Bd, R, L, p):
    """vaesne_attn_rep_fwd_part: query parts [0, k) and [k, n) launched separately (the
    first beside the encoders, the rest later) give the one-launch o, lse and bitmap."""
    from VAESNe import _lib, rng
    lib = _lib.lib
    k, n = parts
    qkv, kb, _, _ = _inputs(Bd, R, L, 0.05, 3 * L + R)
    st = rng.state(DEV)
    o0, l0, b0 = _rep_fwd(lib, qkv, kb, Bd, R, L, p, st, 77)
    N = R * Bd
    o1 = torch.full((N, L, E), float("nan"), device=DEV)
    l1 = torch.empty(Bd, H, L, device=DEV)
    b1 = torch.full((lib.attn_keep_bits_size(N, H, L, L) // 4,), -1, dtype=torch.int32, device=DEV)
    for p0, p1 in ((0, k), (k, n)):
        assert lib.attn_rep_fwd_part(qkv.data_ptr(), L * 3 * E, 3 * E, kb.data_ptr(), L,
                                     o1.data_ptr(), L * E, E, l1.data_ptr(), Bd, R, H, L, 8, p,
                                     st.data_ptr(), 77, b1.data_ptr(), p0, p1, n,
                                     _lib.stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
    if p > 0:
        assert torch.equal(b0, b1)
