"""Grouped linear launches (vaesne_linear_*_group) against one launch per group:
bit-identical outputs, input gradients and weight / bias gradients (the grouped
kernels run the same per-workgroup arithmetic, the same fixed-order sums), for the
shapes the encoders use (context in / out / k|v projections) and ragged M."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("G,M,K,N,shared", [(4, 16 * 984, 32, 96, True), (4, 16 * 984, 32, 32, False),
                                            (3, 37, 32, 64, False), (8, 1000, 64, 32, True)])
def test_group_linear_matches_per_group(G, M, K, N, shared):
    from VAESNe import _ops
    from VAESNe._lib import lib, stream
    g = torch.Generator().manual_seed(G * M + K)
    Ws = [torch.randn(N, K, generator=g).to(DEV).requires_grad_(True) for _ in range(G)]
    bs = [torch.randn(N, generator=g).to(DEV).requires_grad_(True) for _ in range(G)]
    x = torch.randn(*(() if shared else (G,)), M, K, generator=g).to(DEV).requires_grad_(True)
    ys = _ops.group_linear(x, Ws, bs, shared=shared)
    ys = list(ys) if not shared else [ys[i] for i in range(G)]
    gos = [torch.randn(M, N, generator=g).to(DEV) for _ in range(G)]
    sum((y * go).sum() for y, go in zip(ys, gos)).backward()
    ref_y, ref_dW, ref_db, ref_dx = [], [], [], []
    for i in range(G):
        xi = (x if shared else x[i]).detach().clone().requires_grad_(True)
        Wi = Ws[i].detach().clone().requires_grad_(True)
        bi = bs[i].detach().clone().requires_grad_(True)
        y = _ops.linear(xi, Wi, bi)
        (y * gos[i]).sum().backward()
        ref_y.append(y.detach())
        ref_dW.append(Wi.grad)
        ref_db.append(bi.grad)
        ref_dx.append(xi.grad)
    for i in range(G):
        assert torch.equal(ys[i].detach(), ref_y[i])
        assert torch.equal(Ws[i].grad, ref_dW[i])
        assert torch.equal(bs[i].grad, ref_db[i])
    if shared:
        tot = ref_dx[0]
        for d in ref_dx[1:]:
            tot = tot + d
        assert float((x.grad - tot).abs().max() / tot.abs().max()) < 1e-6
    else:
        for i in range(G):
            assert torch.equal(x.grad[i], ref_dx[i])
