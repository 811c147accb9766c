"""Fused encoder latent chain (VAESNe/_chain.py, csrc/enc_chain.hip) against the
per-op encoder path (few-query attention kernels + PRE / POST halves, itself pinned
to the per-op TransformerBlock chain and the golden vectors): outputs, input and
context gradients and every block-parameter gradient, with dropout on (same call
ids -> identical keep masks), masks, the cfg-5 983-token context and ragged T."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _blocks(n, seed, selfattn, p):
    from VAESNe.util_layers import TransformerBlock
    torch.manual_seed(seed)
    blocks = torch.nn.ModuleList([TransformerBlock(32, 4, 32, p, selfattn) for _ in range(n)])
    with torch.no_grad():
        for prm in blocks.parameters():
            prm.add_(0.1 * torch.randn_like(prm))
    return blocks.to(DEV)


def _mask(B, L, p, g):
    m = torch.rand(B, L, generator=g) < p
    m[:, 0] = False
    return m


def _run(blocks, x, ctx, mask, go, chain, monkeypatch, defer=False):
    from VAESNe import _config, _defer, rng
    from VAESNe.util_layers import encoder_stack
    monkeypatch.setattr(_config, "enc_chain", bool(chain))
    rng.manual_seed(1234)
    blocks.zero_grad(set_to_none=True)
    xx = x.clone().requires_grad_(True)
    cc = ctx.clone().requires_grad_(True)
    with _defer.deferred(defer):
        out = encoder_stack(blocks, xx, cc, context_mask=mask)
        (out * go).sum().backward()
    torch.cuda.synchronize()
    return [out.detach(), xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()]


@pytest.mark.parametrize("selfattn,B,T,Lc,p,nb", [
    (False, 16, 8, 60, 0.1, 4),     # photometry encoder (cfg 5)
    (True, 16, 8, 983, 0.1, 4),     # spectra encoder with context self-attention (cfg 5)
    (False, 3, 5, 37, 0.1, 2),      # ragged T, short context
    (True, 5, 8, 129, 0.0, 3),      # no dropout
    (False, 2, 8, 300, 0.3, 1),     # one block, key tiles cross a 256 boundary
])
def test_chain_matches_per_op(selfattn, B, T, Lc, p, nb, monkeypatch):
    blocks = _blocks(nb, B + Lc + nb, selfattn, p)
    blocks.train()
    g = torch.Generator().manual_seed(Lc + B)
    x = torch.randn(B, T, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    mask = _mask(B, Lc, 0.1, g).to(DEV)
    go = torch.randn(B, T, 32, generator=g).to(DEV)
    fused = _run(blocks, x, ctx, mask, go, True, monkeypatch)
    ref = _run(blocks, x, ctx, mask, go, False, monkeypatch)
    names = ["out", "dx", "dcontext"] + [n for n, _ in blocks.named_parameters()]
    assert len(names) == len(fused)
    for n, a, b in zip(names, fused, ref):
        assert torch.isfinite(a).all(), n
        assert _rel(a, b) < 3e-5, (n, _rel(a, b))


def test_chain_deferred_and_repeat_bitwise(monkeypatch):
    """Deferred gradient sums equal immediate ones, and two runs agree, bit for bit."""
    B, T, Lc = 16, 8, 983
    blocks = _blocks(4, 7, True, 0.1)
    blocks.train()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, T, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    mask = _mask(B, Lc, 0.05, g).to(DEV)
    go = torch.randn(B, T, 32, generator=g).to(DEV)
    a = _run(blocks, x, ctx, mask, go, True, monkeypatch, defer=True)
    b = _run(blocks, x, ctx, mask, go, True, monkeypatch, defer=False)
    c = _run(blocks, x, ctx, mask, go, True, monkeypatch, defer=True)
    for u, v, w in zip(a, b, c):
        assert torch.equal(u, v) and torch.equal(u, w)


def test_chain_two_groups_one_launch_equals_separate():
    """Two encoders (different context lengths, masks, dropout ids) in ONE launch
    give exactly what two single-group launches give."""
    from VAESNe import _chain, rng
    specs_in = [(False, 16, 8, 60, 11), (True, 16, 8, 983, 12)]
    items, inputs = [], []
    for selfattn, B, T, Lc, seed in specs_in:
        blocks = _blocks(4, seed, False, 0.1)
        blocks.train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(B, T, 32, generator=g).to(DEV)
        ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
        mask = _mask(B, Lc, 0.1, g).to(DEV)
        go = torch.randn(B, T, 32, generator=g).to(DEV)
        inputs.append((blocks, x, ctx, mask, go))
    rng.manual_seed(99)
    ids = [_chain.reserve_call_ids(list(inp[0])) for inp in inputs]

    def run(grouped):
        outs = []
        for blocks, *_ in inputs:
            blocks.zero_grad(set_to_none=True)
        leaves = []
        items = []
        for (blocks, x, ctx, mask, go), cid in zip(inputs, ids):
            xx = x.clone().requires_grad_(True)
            cc = ctx.clone().requires_grad_(True)
            leaves.append((xx, cc))
            spec = _chain.make_spec(list(blocks), mask, shared=True, call_ids=cid)
            items.append((spec, xx, [cc], list(blocks)))
        if grouped:
            hs = _chain.enc_chain(items)
        else:
            hs = [_chain.enc_chain([it])[0] for it in items]
        loss = sum((h * inp[4]).sum() for h, inp in zip(hs, inputs))
        loss.backward()
        torch.cuda.synchronize()
        for h, (xx, cc), (blocks, *_) in zip(hs, leaves, inputs):
            outs += [h.detach(), xx.grad, cc.grad] + [p.grad.clone() for p in blocks.parameters()]
        return outs

    a, b = run(True), run(False)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_chain_fully_masked_row_gives_nan_like_reference(monkeypatch):
    """A sequence whose context keys are all masked: the reference's softmax over
    -inf gives NaN; the chain does the same (and only for that sequence)."""
    B, T, Lc = 3, 8, 20
    blocks = _blocks(2, 5, False, 0.0)
    blocks.train()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, T, 32, generator=g).to(DEV)
    ctx = torch.randn(B, Lc, 32, generator=g).to(DEV)
    mask = torch.zeros(B, Lc, dtype=torch.bool)
    mask[1] = True
    mask = mask.to(DEV)
    from VAESNe import _config
    from VAESNe.util_layers import encoder_stack
    monkeypatch.setattr(_config, "enc_chain", True)
    with torch.no_grad():
        out = encoder_stack(blocks, x, ctx, context_mask=mask)
    assert torch.isnan(out[1]).all()
    assert torch.isfinite(out[0]).all() and torch.isfinite(out[2]).all()
