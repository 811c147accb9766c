"""Per-kernel parity of libvaesne_hip.so against the CPU oracle (fp64 torch
restatement of the reference arithmetic), on random shapes and the edge cases
the reference's data produce: ragged key padding masks, a single unmasked key,
L not a multiple of any tile, the 983-token encoder context, Lk = 4/5 context
tokens, and dropout (mask statistics and forward/backward mask agreement)."""
import math

import numpy as np
import pytest
import torch

from oracle import vaesne_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _mha_params(E, seed):
    g = torch.Generator().manual_seed(seed)
    return {"a.in_proj_weight": torch.randn(3 * E, E, generator=g) / math.sqrt(E),
            "a.in_proj_bias": 0.1 * torch.randn(3 * E, generator=g),
            "a.out_proj.weight": torch.randn(E, E, generator=g) / math.sqrt(E),
            "a.out_proj.bias": 0.1 * torch.randn(E, generator=g)}


def _rand_mask(B, L, p, g, keep_first=True):
    m = torch.rand(B, L, generator=g) < p
    if keep_first:
        m[:, 0] = False
    return m


@pytest.mark.parametrize("B,Lq,Lk,self_attn,pm", [
    (3, 982, 982, True, 0.05),     # spectra decoder self-attention
    (2, 983, 983, True, 0.05),     # spectra encoder context self-attention (cfg 5)
    (4, 60, 60, True, 0.1),        # photometry decoder self-attention
    (3, 8, 983, False, 0.05),      # encoder cross-attention (queries = latent tokens)
    (3, 13, 983, False, 0.05),     # few-query path, two ragged query groups
    (4, 16, 60, False, 0.1),       # latent_len 8 (16 latent tokens) over a light curve
    (5, 8, 8, True, 0.0),          # encoder latent self-attention
    (5, 982, 5, False, 0.0),       # spectra decoder cross-attention (4 latent + phase)
    (2, 37, 1, False, 0.0),        # a single key
    (2, 300, 257, False, 0.9),     # heavy ragged masking
])
def test_mha_forward_backward_vs_oracle(B, Lq, Lk, self_attn, pm):
    from VAESNe.util_layers import MultiheadAttention
    E, H = 32, 4
    g = torch.Generator().manual_seed(B * 1000 + Lq + Lk)
    p64 = {k: v.double() for k, v in _mha_params(E, Lq + Lk).items()}
    xq = torch.randn(B, Lq, E, generator=g, dtype=torch.float64)
    xk = xq if self_attn else torch.randn(B, Lk, E, generator=g, dtype=torch.float64)
    mask = _rand_mask(B, Lk, pm, g) if pm > 0 else None
    # oracle (fp64, CPU)
    pr = {k: v.clone().requires_grad_(True) for k, v in p64.items()}
    xq_r = xq.clone().requires_grad_(True)
    xk_r = xq_r if self_attn else xk.clone().requires_grad_(True)
    ref = O.multihead_attention(pr, "a", xq_r, xk_r, mask, H)
    go = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (ref * go).sum().backward()
    # HIP
    mha = MultiheadAttention(E, H, dropout=0.0, batch_first=True).to(DEV)
    with torch.no_grad():
        mha.in_proj_weight.copy_(p64["a.in_proj_weight"].float())
        mha.in_proj_bias.copy_(p64["a.in_proj_bias"].float())
        mha.out_proj.weight.copy_(p64["a.out_proj.weight"].float())
        mha.out_proj.bias.copy_(p64["a.out_proj.bias"].float())
    xq_d = xq.float().to(DEV).requires_grad_(True)
    xk_d = xq_d if self_attn else xk.float().to(DEV).requires_grad_(True)
    out, _ = mha(xq_d, xk_d, xk_d, key_padding_mask=None if mask is None else mask.to(DEV))
    (out * go.float().to(DEV)).sum().backward()
    assert _rel(out, ref) < 2e-5
    if Lk == 1:   # softmax over one key is constant: dQ is analytically 0 (rounding only)
        assert xq_d.grad.abs().max().item() < 1e-5
    else:
        assert _rel(xq_d.grad, xq_r.grad) < 1e-4
    if not self_attn:
        assert _rel(xk_d.grad, xk_r.grad) < 1e-4
    assert _rel(mha.in_proj_weight.grad, pr["a.in_proj_weight"].grad) < 1e-4
    assert _rel(mha.out_proj.weight.grad, pr["a.out_proj.weight"].grad) < 1e-4
    # q/v bias grads (the k-bias grad is analytically 0)
    E_ = E
    bref = pr["a.in_proj_bias"].grad
    bgot = mha.in_proj_bias.grad
    if Lk == 1:
        assert bgot[:E_].abs().max().item() < 1e-5
    else:
        assert _rel(bgot[:E_], bref[:E_]) < 1e-4
    assert _rel(bgot[2 * E_:], bref[2 * E_:]) < 1e-4
    assert bgot[E_:2 * E_].abs().max().item() < 1e-4 * bref.abs().max().item() + 1e-6


def test_fully_masked_row_gives_nan_like_reference():
    """A key padding mask with no observed key makes softmax NaN in the
    reference (-inf everywhere); the kernel propagates the same NaN."""
    from VAESNe import _ops
    B, L, E = 2, 16, 32
    qkv = torch.randn(B, L, 3 * E, device=DEV)
    m = torch.zeros(B, L, dtype=torch.bool, device=DEV)
    m[1] = True
    o = _ops.self_attention(qkv, m, 4, 0.0)
    assert torch.isfinite(o[0]).all() and torch.isnan(o[1]).all()


def _probe_attention_mask(B, Lq, Lk, j0, p, seed_call):
    """Read the attention-dropout keep mask of keys j0..j0+7 for every query:
    q = 0 (uniform softmax over the 8 unmasked probe keys), v_j = e_(j-j0)."""
    from VAESNe import _ops, rng
    E, H, dh = 32, 4, 8
    q = torch.zeros(B, Lq, E, device=DEV)
    kv = torch.zeros(B, Lk, 2 * E, device=DEV)
    for h in range(H):
        for t in range(8):
            kv[:, j0 + t, E + h * dh + t] = 1.0
    mask = torch.ones(B, Lk, dtype=torch.bool, device=DEV)
    mask[:, j0:j0 + 8] = False
    rng._call = seed_call - 1
    o = _ops.cross_attention(q, kv, mask, H, p)
    keep = (o.view(B, Lq, H, dh) * 8 * (1 - p)).round()   # 1 kept / 0 dropped
    return keep, q, kv, mask


@pytest.mark.parametrize("B,Lq,Lk", [(4, 512, 130), (128, 8, 130), (96, 13, 983)])
def test_attention_dropout_statistics_and_backward_mask(B, Lq, Lk):
    """Query-tiled (Lq=512) and key-parallel few-query (Lq<=16) kernels."""
    from VAESNe import _ops, rng
    p = 0.1
    keep, q, kv, mask = _probe_attention_mask(B, Lq, Lk, 100, p, 777)
    assert set(torch.unique(keep).tolist()) <= {0.0, 1.0}
    rate = 1 - keep.mean().item()
    n = keep.numel()
    assert abs(rate - p) < 4 * math.sqrt(p * (1 - p) / n), rate
    # neighbouring keys / heads / queries are not correlated
    k = keep.float() - keep.float().mean()
    for a, b in [(k[..., :-1], k[..., 1:]), (k[:, :-1], k[:, 1:])]:
        corr = (a * b).mean() / (k * k).mean()
        assert abs(corr.item()) < 0.02
    # backward regenerates the same mask: dV of probe key j for head h equals
    # sum_q keep[q, h, j] / (8 (1 - p)) * dO[q, h, :]
    qd = q.clone().requires_grad_(True)
    kvd = kv.clone().requires_grad_(True)
    rng._call = 777 - 1
    o = _ops.cross_attention(qd, kvd, mask, 4, p)
    go = torch.randn_like(o)
    (o * go).sum().backward()
    dv = kvd.grad[:, 100:108, 32:].view(B, 8, 4, 8)          # [B, j, h, d]
    expect = torch.einsum("bqhj,bqhd->bjhd", keep, go.view(B, Lq, 4, 8)) / (8 * (1 - p))
    assert _rel(dv, expect) < 1e-5


@pytest.mark.parametrize("nt,np_", [(256, 2), (128, 2), (64, 2), (256, 1)])
@pytest.mark.parametrize("B,Lq,Lk", [(2, 200, 40), (2, 300, 300)])
def test_attention_forced_geometries_vs_dense(nt, np_, B, Lq, Lk):
    """Every query-tiled geometry (the decoders' 982-token launches run 256 x 2,
    which small shapes never pick by themselves), dropout on, against the dense
    reference: forward, dQ (fused into the dK / dV kernel), dK, dV."""
    from VAESNe._lib import lib
    assert lib.attn_force_geometry(nt, np_) == 0
    try:
        test_attention_dropout_outputs_and_all_gradients_vs_dense(B, Lq, Lk)
    finally:
        lib.attn_force_geometry(0, 0)


@pytest.mark.parametrize("B,Lq,Lk", [(2, 200, 40), (3, 37, 70), (2, 300, 300)])
def test_attention_dropout_outputs_and_all_gradients_vs_dense(B, Lq, Lk):
    """With dropout on, out / dQ / dK / dV of the query-tiled kernels equal a
    dense fp64 attention that applies the kernel's own keep mask (probed 8
    keys at a time: the decisions depend only on (seed, counter, call id,
    b, h, q, key), never on the values or the key padding mask)."""
    from VAESNe import _ops, rng
    p, E, H, dh, cid = 0.1, 32, 4, 8, 4242
    keep = torch.zeros(B, Lq, H, Lk, device=DEV)
    for j0 in range(0, Lk, 8):
        kk, _, _, _ = _probe_attention_mask(B, Lq, Lk, j0, p, cid) if j0 + 8 <= Lk else \
            _probe_attention_mask(B, Lq, Lk + (j0 + 8 - Lk), j0, p, cid)
        n = min(8, Lk - j0)
        keep[..., j0:j0 + n] = kk[..., :n]
    g = torch.Generator().manual_seed(B * Lq + Lk)
    q = torch.randn(B, Lq, E, generator=g, dtype=torch.float64)
    kv = torch.randn(B, Lk, 2 * E, generator=g, dtype=torch.float64)
    go = torch.randn(B, Lq, E, generator=g, dtype=torch.float64)
    qd = q.float().to(DEV).requires_grad_(True)
    kvd = kv.float().to(DEV).requires_grad_(True)
    rng._call = cid - 1
    o = _ops.cross_attention(qd, kvd, None, H, p)
    (o * go.float().to(DEV)).sum().backward()
    qr, kvr = q.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    qh = qr.view(B, Lq, H, dh).transpose(1, 2)
    kh = kvr[..., :E].reshape(B, Lk, H, dh).transpose(1, 2)
    vh = kvr[..., E:].reshape(B, Lk, H, dh).transpose(1, 2)
    P = torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(dh), dim=-1)
    A = P * keep.double().cpu().permute(0, 2, 1, 3) / (1 - p)
    ref = (A @ vh).transpose(1, 2).reshape(B, Lq, E)
    (ref * go).sum().backward()
    assert _rel(o, ref) < 2e-5
    assert _rel(qd.grad, qr.grad) < 1e-4
    assert _rel(kvd.grad, kvr.grad) < 1e-4


def test_add_layernorm_vs_oracle_and_dropout():
    from VAESNe import _ops, rng
    M, E = 5000, 32
    ln = torch.nn.LayerNorm(E).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(1 + 0.1 * torch.randn(E))
        ln.bias.copy_(0.1 * torch.randn(E))
    x = torch.randn(M, E, device=DEV, requires_grad=True)
    r = torch.randn(M, E, device=DEV, requires_grad=True)
    y = _ops.add_layernorm(x, r, ln, 0.0)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    p = {"n.weight": ln.weight.detach().double().cpu().requires_grad_(True),
         "n.bias": ln.bias.detach().double().cpu().requires_grad_(True)}
    xr = x.detach().double().cpu().requires_grad_(True)
    rr = r.detach().double().cpu().requires_grad_(True)
    yr = O.layer_norm(p, "n", xr + rr)
    (yr * gy.double().cpu()).sum().backward()
    assert _rel(y, yr) < 1e-5
    assert _rel(x.grad, xr.grad) < 1e-4 and _rel(r.grad, rr.grad) < 1e-4
    assert _rel(ln.weight.grad, p["n.weight"].grad) < 1e-4
    assert _rel(ln.bias.grad, p["n.bias"].grad) < 1e-4
    # dropout: x = 0, res = 1 -> kept entries sit above the row mean
    ln2 = torch.nn.LayerNorm(E).to(DEV)
    xz = torch.zeros(M, E, device=DEV)
    ones = torch.ones(M, E, device=DEV, requires_grad=True)
    rng._call = 41
    y2 = _ops.add_layernorm(xz, ones, ln2, 0.1)
    kept = (y2 > 0) | (y2.abs() < 1e-6)
    rate = 1 - kept.float().mean().item()
    assert abs(rate - 0.1) < 4 * math.sqrt(0.09 / kept.numel())
    # backward uses the same mask: d res = dLN * keep / (1-p)
    gy2 = torch.randn_like(y2)
    (y2 * gy2).sum().backward()
    assert (ones.grad[~kept] == 0).all()


@pytest.mark.parametrize("K,N,act", [(32, 96, None), (32, 32, "gelu"), (64, 32, "relu"),
                                     (96, 32, "relu"), (1, 32, None), (4, 32, "relu"),
                                     (3, 32, "relu"), (32, 1, None), (32, 2, None)])
def test_linear_vs_oracle(K, N, act):
    from VAESNe import _ops
    g = torch.Generator().manual_seed(K * 100 + N)
    M = 3001
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).double()
    b = (0.1 * torch.randn(N, generator=g)).double()
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    x2 = torch.randn(M, K, generator=g, dtype=torch.float64)
    Wd, bd = W.float().to(DEV).requires_grad_(True), b.float().to(DEV).requires_grad_(True)
    xd, x2d = x.float().to(DEV).requires_grad_(True), x2.float().to(DEV).requires_grad_(True)
    y = _ops.linear(xd, Wd, bd, act=act, x2=x2d)
    Wr, br = W.clone().requires_grad_(True), b.clone().requires_grad_(True)
    xr, x2r = x.clone().requires_grad_(True), x2.clone().requires_grad_(True)
    yr = torch.nn.functional.linear(xr + x2r, Wr, br)
    yr = {None: yr, "relu": torch.relu(yr), "gelu": torch.nn.functional.gelu(yr)}[act]
    gy = torch.randn(M, N, generator=g, dtype=torch.float64)
    (y * gy.float().to(DEV)).sum().backward()
    (yr * gy).sum().backward()
    assert _rel(y, yr) < 1e-5
    assert _rel(xd.grad, xr.grad) < 1e-4 and _rel(x2d.grad, x2r.grad) < 1e-4
    assert _rel(Wd.grad, Wr.grad) < 1e-4 and _rel(bd.grad, br.grad) < 1e-4


def test_embedding_sincos_rsample_latent_head():
    from VAESNe import _ops
    g = torch.Generator().manual_seed(5)
    # embedding gather + deterministic scatter-add, with fused base add
    idx = torch.randint(0, 6, (37, 60), generator=g)
    table = torch.randn(6, 32, generator=g)
    base = torch.randn(37, 60, 32, generator=g)
    td = table.to(DEV).requires_grad_(True)
    bd = base.to(DEV).requires_grad_(True)
    out = _ops.embedding(idx.to(DEV), td, base=bd)
    go = torch.randn(37, 60, 32, generator=g)
    (out * go.to(DEV)).sum().backward()
    assert _rel(out, table[idx] + base) < 1e-6
    ref = torch.zeros(6, 32, dtype=torch.float64).index_add_(0, idx.reshape(-1), go.reshape(-1, 32).double())
    assert _rel(td.grad, ref) < 1e-5 and _rel(bd.grad, go) == 0.0
    # sinusoidal features vs the reference recipe
    x = torch.randn(7, 982, generator=g)
    div = torch.exp(torch.arange(0, 32).float() * (-torch.log(torch.tensor(10000.0)) / 32))
    f = _ops.sincos(x.to(DEV), div.to(DEV))
    assert _rel(f, O.sinus_features(x.double(), div.double())) < 1e-5
    # latent head + rsample (+ grads)
    bott = torch.randn(5, 8, 4, generator=g, dtype=torch.float64)
    bott[0, 4, 0] = 25.0   # softplus threshold branch
    u = O.draw_u((3, 5, 4, 4), generator=g).double()
    b_d = bott.float().to(DEV).requires_grad_(True)
    mu, sc = _ops.latent_head(b_d, 4)
    z = _ops.RsampleFn.apply(mu, sc, u.float().to(DEV), False)
    gz = torch.randn(z.shape, generator=g, dtype=torch.float64)
    (z * gz.float().to(DEV)).sum().backward()
    b_r = bott.clone().requires_grad_(True)
    mu_r, sc_r = b_r[:, :4], torch.nn.functional.softplus(b_r[:, 4:])
    z_r = O.laplace_rsample(mu_r, sc_r, u)
    (z_r * gz).sum().backward()
    assert _rel(z, z_r) < 1e-5 and _rel(b_d.grad, b_r.grad) < 1e-5


def test_posterior_rsample_and_latent_cat_sums_match_autograd():
    """The loss's gradients of loc / scale added inside the sampler's backward
    (vaesne_rsample_bwd_acc) and the latent concat's readers + loss gradients summed in one
    launch (vaesne_cat_grad): bit-identical to autograd's own adds (two-term sums)."""
    from VAESNe import _ops, rng
    g = torch.Generator().manual_seed(11)
    K, B, Lz, Dz = 8, 16, 4, 4
    locs = [torch.randn(B, Lz, Dz, generator=g).to(DEV).requires_grad_(True) for _ in range(2)]
    scs = [torch.rand(B, Lz, Dz, generator=g).add(0.1).to(DEV).requires_grad_(True)
           for _ in range(2)]
    us = [O.draw_u((K, B, Lz, Dz), generator=g).float().to(DEV) for _ in range(2)]
    w = [torch.randn(K, 2 * B, Lz, Dz, generator=g).to(DEV) for _ in range(2)]
    wl = [torch.randn(B, Lz, Dz, generator=g).to(DEV) for _ in range(4)]
    wz = [torch.randn(K, B, Lz, Dz, generator=g).to(DEV) for _ in range(2)]

    def run(fused):
        for t in locs + scs:
            t.grad = None
        zs, ps = [], []
        for m in range(2):
            with rng.inject_uniform([us[m]]):
                if fused:
                    z, l, s = _ops.posterior_rsample(locs[m], scs[m], K)
                else:
                    z, l, s = _ops.laplace_rsample(locs[m], scs[m], K), locs[m], scs[m]
            zs.append(z)
            ps += [l, s]
        if fused:
            zcats, zl = _ops.latent_cat(zs, 2)
        else:
            zc = torch.cat(zs, dim=1)
            zcats, zl = (zc, zc), zs
        f = sum((zcats[d] * w[d]).sum() for d in range(2))
        f = f + sum((zl[m] * wz[m]).sum() for m in range(2))
        f = f + sum((ps[i] * wl[i]).sum() for i in range(4))
        f.backward()
        return [t.grad.clone() for t in locs + scs], torch.cat(zcats, 0).detach()

    g_ref, z_ref = run(False)
    g_new, z_new = run(True)
    assert torch.equal(z_ref, z_new)
    for a, b in zip(g_ref, g_new):
        assert torch.equal(a, b)


def test_device_uniform_range_and_moments():
    from VAESNe import rng
    u = rng.draw_uniform((4096, 256), DEV)
    eps = torch.finfo(torch.float32).eps
    assert u.min().item() >= eps - 1 and u.max().item() < 1
    assert abs(u.mean().item()) < 5e-3 and abs(u.var().item() - 1 / 3) < 5e-3
    u2 = rng.draw_uniform((4096, 256), DEV)
    assert not torch.equal(u, u2)


def _decoder_blocks(n, seed):
    from VAESNe.util_layers import TransformerBlock
    torch.manual_seed(seed)
    blocks = torch.nn.ModuleList([TransformerBlock(32, 4, 32, 0.0) for _ in range(n)])
    with torch.no_grad():
        for prm in blocks.parameters():   # non-trivial biases / LN affine
            prm.add_(0.1 * torch.randn_like(prm))
    return blocks


@pytest.mark.parametrize("N,L,Lc,nblk", [(6, 982, 5, 2), (5, 60, 4, 2), (3, 37, 1, 1), (2, 130, 8, 3),
                                         (3, 300, 2, 2), (2, 400, 3, 2)])
def test_fused_decoder_stack_vs_oracle(N, L, Lc, nblk):
    """util_layers.decoder_stack (self-attention kernel + fused tail kernel per
    block) against the oracle's TransformerBlock chain in fp64."""
    from VAESNe.util_layers import decoder_stack
    blocks = _decoder_blocks(nblk, N + L).to(DEV)
    blocks.train()
    g = torch.Generator().manual_seed(L)
    x = torch.randn(N, L, 32, generator=g, dtype=torch.float64)
    ctx = torch.randn(N, Lc, 32, generator=g, dtype=torch.float64)
    mask = _rand_mask(N, L, 0.1, g)
    go = torch.randn(N, L, 32, generator=g, dtype=torch.float64)
    # oracle
    p = {k: v.detach().double().cpu().clone().requires_grad_(True) for k, v in blocks.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    cr = ctx.clone().requires_grad_(True)
    h = xr
    for i in range(nblk):
        h = O.transformer_block(p, f"{i}", h, cr, mask, None, 4)
    (h * go).sum().backward()
    # HIP
    xd = x.float().to(DEV).requires_grad_(True)
    cd = ctx.float().to(DEV).requires_grad_(True)
    out = decoder_stack(blocks, xd, cd, mask.to(DEV))
    (out * go.float().to(DEV)).sum().backward()
    assert _rel(out, h) < 2e-5
    assert _rel(xd.grad, xr.grad) < 2e-4
    assert _rel(cd.grad, cr.grad) < 2e-4
    for k, prm in blocks.named_parameters():
        ref = p[k].grad
        if k.endswith("in_proj_bias"):
            # key-bias slice: analytically zero gradient (softmax shift invariance)
            assert _rel(prm.grad[:32], ref[:32]) < 2e-4 and _rel(prm.grad[64:], ref[64:]) < 2e-4, k
            continue
        assert _rel(prm.grad, ref) < 2e-4, k


def test_fused_decoder_tail_dropout_fwd_bwd_consistent():
    """With dropout on, the fused tail's backward regenerates the forward's
    masks: a directional finite difference matches <grad, v>."""
    from VAESNe import rng
    from VAESNe.util_layers import decoder_stack
    blocks = _decoder_blocks(2, 3).to(DEV)
    for b in blocks:
        b.dropout.p = 0.1
        b.self_attn.dropout = 0.1
        b.cross_attn.dropout = 0.1
    blocks.train()
    g = torch.Generator().manual_seed(11)
    N, L, Lc = 3, 200, 5
    x = torch.randn(N, L, 32, generator=g).to(DEV)
    ctx = torch.randn(N, Lc, 32, generator=g).to(DEV)
    go = torch.randn(N, L, 32, generator=g).to(DEV)
    v = torch.randn(N, L, 32, generator=g).to(DEV)

    def f(xx, grad=False):
        rng._call = 500
        xx = xx.clone().requires_grad_(grad)
        out = decoder_stack(blocks, xx, ctx, None)
        return xx, (out * go).sum()

    xx, val = f(x, True)
    val.backward()
    dirn = (xx.grad * v).sum().item()
    eps = 1e-2
    with torch.no_grad():
        fd = (f(x + eps * v)[1].item() - f(x - eps * v)[1].item()) / (2 * eps)
    assert abs(fd - dirn) < 2e-2 * abs(dirn) + 1e-3, (fd, dirn)
    # and the mask is really on: a different call id changes the output
    with torch.no_grad():
        rng._call = 900
        o2 = decoder_stack(blocks, x, ctx, None)
        rng._call = 500
        o1 = decoder_stack(blocks, x, ctx, None)
    assert (o1 - o2).abs().max().item() > 1e-3


@pytest.mark.parametrize("L,Lc,store", [(982, 5, True), (300, 4, False), (57, 8, True),
                                        (300, 2, True), (400, 3, False)])
def test_decoder_tail_fused_backward_matches_two_kernel_path(L, Lc, store):
    """The fused per-sequence tail backward (no per-token scratch) against the
    data-kernel + scratch + weight-gradient-kernel path on the same draws: every
    gradient, with dropout (stored masks and re-hashed), a fused next in_proj
    (blocks 0..n-2) and a last block."""
    from VAESNe import _lib, _ops, rng
    from VAESNe.util_layers import decoder_stack
    blocks = _decoder_blocks(3, L + Lc).to(DEV)
    for b in blocks:
        b.dropout.p = 0.1
        b.self_attn.dropout = 0.1
        b.cross_attn.dropout = 0.1
    blocks.train()
    g = torch.Generator().manual_seed(L + Lc)
    N = 4
    x = torch.randn(N, L, 32, generator=g).to(DEV)
    ctx = torch.randn(N, Lc, 32, generator=g).to(DEV)
    mask = _rand_mask(N, L, 0.1, g).to(DEV)
    go = torch.randn(N, L, 32, generator=g).to(DEV)
    res = []
    old = _ops.STORE_TAIL_MASKS
    try:
        _ops.STORE_TAIL_MASKS = store
        for path in (1, 2):
            _lib.lib.dec_tail_force_path(path)
            blocks.zero_grad(set_to_none=True)
            rng._call = 700
            xx = x.clone().requires_grad_(True)
            cc = ctx.clone().requires_grad_(True)
            out = decoder_stack(blocks, xx, cc, mask)
            (out * go).sum().backward()
            torch.cuda.synchronize()
            res.append([out.detach(), xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()])
    finally:
        _lib.lib.dec_tail_force_path(0)
        _ops.STORE_TAIL_MASKS = old
    names = ["out", "dx", "dcontext"] + [n for n, _ in blocks.named_parameters()]
    assert torch.equal(res[0][0], res[1][0])
    for n, a, b in zip(names, *res):
        if n.endswith("in_proj_bias"):   # the key slice is analytically zero (shift invariance)
            a, b = torch.cat([a[:32], a[64:]]), torch.cat([b[:32], b[64:]])
        assert _rel(a, b) < 1e-5, n


def test_fused_decoder_tail_stored_masks_match_rehash():
    """The tail backward reading the forward's stored dropout masks gives the
    same gradients as re-hashing them from the counter RNG.  The two paths are
    separate kernel instantiations (the compiler may contract mul/add pairs
    differently), so the bar is 1e-5 relative: one mismatched keep decision
    moves a gradient by O(1)."""
    from VAESNe import _ops, rng
    from VAESNe.util_layers import decoder_stack
    blocks = _decoder_blocks(2, 5).to(DEV)
    for b in blocks:
        b.dropout.p = 0.2
        b.self_attn.dropout = 0.2
        b.cross_attn.dropout = 0.2
    blocks.train()
    g = torch.Generator().manual_seed(12)
    N, L, Lc = 3, 333, 7                      # ragged chunk tail, Lc < LCMAX
    x = torch.randn(N, L, 32, generator=g).to(DEV)
    ctx = torch.randn(N, Lc, 32, generator=g).to(DEV)
    go = torch.randn(N, L, 32, generator=g).to(DEV)
    res = []
    for store in (True, False):
        _ops.STORE_TAIL_MASKS = store
        try:
            rng._call = 700
            blocks.zero_grad(set_to_none=True)
            xx = x.clone().requires_grad_(True)
            cc = ctx.clone().requires_grad_(True)
            out = decoder_stack(blocks, xx, cc, None)
            (out * go).sum().backward()
            res.append([out, xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()])
        finally:
            _ops.STORE_TAIL_MASKS = True
    assert torch.equal(res[0][0], res[1][0])   # forward: same kernel both times
    for a, b in zip(res[0][1:], res[1][1:]):
        assert (a - b).abs().max().item() <= 1e-5 * max(a.abs().max().item(), 1e-3)


def _encoder_blocks(n, seed, selfattn):
    from VAESNe.util_layers import TransformerBlock
    torch.manual_seed(seed)
    blocks = torch.nn.ModuleList([TransformerBlock(32, 4, 32, 0.0, selfattn) for _ in range(n)])
    with torch.no_grad():
        for prm in blocks.parameters():
            prm.add_(0.1 * torch.randn_like(prm))
    return blocks


@pytest.mark.parametrize("selfattn,B,T,Lc", [(False, 16, 8, 60), (True, 5, 8, 129), (False, 3, 5, 37)])
def test_fused_encoder_stack_matches_per_op(selfattn, B, T, Lc):
    """util_layers.encoder_stack (PRE / cross-attention / POST kernels) against the
    per-op TransformerBlock chain on the same blocks: outputs and every gradient."""
    from VAESNe.util_layers import encoder_stack
    blocks = _encoder_blocks(3, B + Lc, selfattn).to(DEV)
    blocks.train()
    g = torch.Generator().manual_seed(Lc)
    x = torch.randn(B, T, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    mask = _rand_mask(B, Lc, 0.1, g).to(DEV)
    go = torch.randn(B, T, 32, generator=g).to(DEV)
    res = []
    for fused in (True, False):
        blocks.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        cc = ctx.clone().requires_grad_(True)
        if fused:
            out = encoder_stack(blocks, xx, cc, context_mask=mask)
        else:
            out = xx
            for blk in blocks:
                out = blk(out, cc, context_mask=mask)
        (out * go).sum().backward()
        # detached: the fused pass's graph (AccumulateGrad nodes bound to the context
        # side streams) must not outlive it into the one-stream per-op pass
        res.append([out.detach(), xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()])
        del out
    names = ["out", "dx", "dcontext"] + [n for n, _ in blocks.named_parameters()]
    for n, a, b in zip(names, *res):
        assert _rel(a, b) < 2e-5, n


@pytest.mark.parametrize("B,Lc,defer", [(16, 983, False), (3, 70, True)])
def test_merged_context_paths_match_per_block(B, Lc, defer, monkeypatch):
    """The blocks' context self-attention paths batch-stacked into one attention
    launch (util_layers._merged_context_paths, _config.ctx_merge) against one path
    per block: outputs and every gradient (cfg-5 shape: 4 blocks, 983 tokens)."""
    from VAESNe import _config, _defer
    from VAESNe.util_layers import encoder_stack
    blocks = _encoder_blocks(4, B + Lc + 1, True).to(DEV)
    blocks.train()
    g = torch.Generator().manual_seed(Lc + 1)
    x = torch.randn(B, 8, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    mask = _rand_mask(B, Lc, 0.05, g).to(DEV)
    go = torch.randn(B, 8, 32, generator=g).to(DEV)
    res = []
    for merge in ("1", "0"):
        monkeypatch.setattr(_config, "ctx_merge", merge == "1")
        blocks.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        cc = ctx.clone().requires_grad_(True)
        with _defer.deferred(defer):
            out = encoder_stack(blocks, xx, cc, context_mask=mask)
            (out * go).sum().backward()
        torch.cuda.synchronize()
        res.append([out.detach(), xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()])
        del out
    names = ["out", "dx", "dcontext"] + [n for n, _ in blocks.named_parameters()]
    assert len(names) == len(res[0]) and any("context_self_attn" in n for n in names)
    for n, a, b in zip(names, *res):
        assert _rel(a, b) < 1e-5, n


def test_fused_encoder_stack_dropout_fwd_bwd_consistent():
    """With dropout on, the encoder halves' backward replays the forward's masks:
    a directional finite difference matches <grad, v>."""
    from VAESNe import rng
    from VAESNe.util_layers import encoder_stack
    blocks = _encoder_blocks(2, 9, True).to(DEV)
    for b in blocks:
        b.dropout.p = 0.1
        b.self_attn.dropout = 0.1
        b.cross_attn.dropout = 0.1
        b.context_self_attn.dropout = 0.1
    blocks.train()
    g = torch.Generator().manual_seed(21)
    B, T, Lc = 4, 8, 70
    x = torch.randn(B, T, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    go = torch.randn(B, T, 32, generator=g).to(DEV)
    v = torch.randn(B, T, 32, generator=g).to(DEV)

    def f(xx, grad=False):
        rng._call = 300
        xx = xx.clone().requires_grad_(grad)
        out = encoder_stack(blocks, xx, ctx)
        return xx, (out * go).sum()

    xx, val = f(x, True)
    val.backward()
    dirn = (xx.grad * v).sum().item()
    eps = 1e-2
    with torch.no_grad():
        fd = (f(x + eps * v)[1].item() - f(x - eps * v)[1].item()) / (2 * eps)
    assert abs(fd - dirn) < 2e-2 * abs(dirn) + 1e-3, (fd, dirn)


def _fwd_raw(q, k, v, kbias, B, H, L_q, L_k, p, st, cid, bits, ws=None):
    """vaesne_attn_fwd on [B, L, E] q / k / v (separate tensors); returns (o, lse)."""
    from VAESNe import _lib
    E = q.shape[-1]
    o = torch.empty(B, L_q, E, device=DEV)
    lse = torch.empty(B, H, L_q, device=DEV)
    rc = _lib.lib.attn_fwd(q.data_ptr(), L_q * E, E, k.data_ptr(), L_k * E, E, v.data_ptr(),
                           L_k * E, E, None if kbias is None else kbias.data_ptr(), L_k,
                           o.data_ptr(), L_q * E, E, lse.data_ptr(), B, H, L_q, L_k, E // H, p,
                           st.data_ptr(), cid, bits.data_ptr(),
                           None if ws is None else ws.data_ptr(), _lib.stream())
    assert rc == 0
    return o, lse


@pytest.mark.parametrize("geo", [(0, 0), (256, 2), (128, 1), (64, 2)])
@pytest.mark.parametrize("B,H,Lq,Lk,dh", [(3, 4, 982, 982, 8), (2, 4, 983, 983, 8),
                                         (2, 4, 300, 77, 8), (5, 2, 17, 17, 8),
                                         (2, 2, 260, 130, 16)])
def test_forward_is_bitwise_reproducible_and_keep_rate(geo, B, H, Lq, Lk, dh):
    """Two launches of the query-tiled forward on the same inputs and draws give o, lse and
    the keep bitmap bit for bit (no atomics, fixed summation orders); the bitmap's valid
    (query, key) bits keep 1 - p of the scores."""
    from VAESNe import _lib, rng
    lib = _lib.lib
    assert lib.attn_force_geometry(*geo) == 0
    try:
        E, p, cid = H * dh, 0.1, 9001
        g = torch.Generator(device=DEV).manual_seed(Lq * 7 + Lk)
        q, k, v = (torch.randn(B, n, E, device=DEV, generator=g) for n in (Lq, Lk, Lk))
        st = rng.state(DEV)
        n = lib.attn_keep_bits_size(B, H, Lq, Lk) // 4
        runs = []
        for _ in range(2):
            bits = torch.full((n,), -1, dtype=torch.int32, device=DEV)
            o, lse = _fwd_raw(q, k, v, None, B, H, Lq, Lk, p, st, cid, bits)
            torch.cuda.synchronize()
            runs.append((o, lse, bits))
        (o0, l0, b0), (o1, l1, b1) = runs
        assert torch.equal(o0, o1) and torch.equal(l0, l1) and torch.equal(b0, b1)
        from test_gpu_sf16 import _decode_bits   # the split-f16 path (default, dh 8) or the VALU one
        keep = _decode_bits(b0, B, Lq, Lk, geo == (0, 0) and dh == 8, H=H).numpy()
        rate = 1 - keep.mean()
        assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / keep.size), rate
    finally:
        lib.attn_force_geometry(0, 0)


@pytest.mark.parametrize("M,with_h,defer", [(982 * 3, True, False), (251392, True, True),
                                            (77, False, False), (1, True, False)])
def test_fused_mlp_head_matches_two_linears(M, with_h, defer, monkeypatch):
    """singlelayerMLP(32 -> 1) on x (+ h) (util_layers.py:9-18, the decoders'
    get_flux / get_photo heads): the fused kernel pair (vaesne_mlp_head_fwd/bwd)
    against the two-linear path (fc1 + ReLU, fc2), forward and every gradient.
    Tokens with a pre-activation within 1e-3 of the ReLU kink get dy = 0: the two
    paths sum in different orders, so there a ReLU decision may legitimately flip."""
    from VAESNe import _config, _defer
    from VAESNe.util_layers import singlelayerMLP
    g = torch.Generator().manual_seed(M)
    head = singlelayerMLP(32, 1)
    x0 = torch.randn(M, 32, generator=g)
    h0 = torch.randn(M, 32, generator=g) if with_h else None
    dy = torch.randn(M, 1, generator=g)
    s64 = (x0 if h0 is None else x0 + h0).double()
    z64 = s64 @ head.fc1.weight.detach().double().T + head.fc1.bias.detach().double()
    dy[(z64.abs() < 1e-3).any(dim=1)] = 0.0
    head = head.to(DEV)
    x0, dy = x0.to(DEV), dy.to(DEV)
    h0 = None if h0 is None else h0.to(DEV)
    res = []
    for fused in ("0", "1"):
        monkeypatch.setattr(_config, "fused_head", fused == "1")
        head.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        h = None if h0 is None else h0.clone().requires_grad_(True)
        with _defer.deferred(defer):
            y = head(x, h)
            y.backward(dy)
        res.append((y.detach(), x.grad, None if h is None else h.grad,
                    [p.grad.clone() for p in head.parameters()]))
    (y0, dx0, dh0, g0), (y1, dx1, dh1, g1) = res
    assert y1.shape == y0.shape
    assert _rel(y1, y0) < 1e-5
    assert _rel(dx1, dx0) < 1e-5
    if with_h:
        assert torch.equal(dh1, dx1) and _rel(dh1, dh0) < 1e-5
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-5
