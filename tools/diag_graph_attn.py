"""Diagnostic (not product): the head_dim-8 attention forward + backward eager vs replayed
from a captured graph, bitwise, at the decoder shapes (N x 982, N x 60) with dropout."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
from VAESNe import _lib, rng  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.lib
H, dh = 4, 8
E = H * dh
for N, L in ((8, 982), (16, 60), (4, 983)):
    g = torch.Generator(device=dev).manual_seed(L)
    qkv = torch.randn(N, L, 3 * E, device=dev, generator=g)
    do = torch.randn(N, L, E, device=dev, generator=g)
    kb = torch.where(torch.rand(N, L, device=dev, generator=g) < 0.05, float("-inf"), 0.0)
    kb[:, 0] = 0.0
    st = rng.state(dev)
    bits = torch.zeros(lib.attn_keep_bits_size(N, H, L, L) // 4, dtype=torch.int32, device=dev)
    o = torch.zeros(N, L, E, device=dev)
    lse = torch.zeros(N, H, L, device=dev)
    dqkv = torch.zeros_like(qkv)
    b, d, s3 = qkv.data_ptr(), dqkv.data_ptr(), L * 3 * E

    def run():
        s = torch.cuda.current_stream().cuda_stream
        lib.attn_fwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E, kb.data_ptr(), L,
                     o.data_ptr(), L * E, E, lse.data_ptr(), N, H, L, L, dh, 0.1, st.data_ptr(), 7,
                     bits.data_ptr(), None, s)
        lib.attn_bwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E, kb.data_ptr(), L,
                     o.data_ptr(), L * E, E, lse.data_ptr(), do.data_ptr(), L * E, E, d, s3, 3 * E,
                     d + 4 * E, s3, 3 * E, d + 8 * E, s3, 3 * E, N, H, L, L, dh, 0.1, st.data_ptr(),
                     7, bits.data_ptr(), None, s)

    run()
    torch.cuda.synchronize()
    ref = [t.clone() for t in (o, lse, bits, dqkv)]
    for t in (o, lse, bits, dqkv):
        t.zero_()
    run()
    torch.cuda.synchronize()
    eq2 = [torch.equal(a, t) for a, t in zip(ref, (o, lse, bits, dqkv))]
    sg = torch.cuda.Stream()
    sg.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(sg):
        with torch.cuda.graph(graph, stream=sg):
            run()
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        for t in (o, lse, bits, dqkv):
            t.zero_()
        graph.replay()
        torch.cuda.synchronize()
        outs.append([torch.equal(a, t) for a, t in zip(ref, (o, lse, bits, dqkv))])
        if not all(outs[-1]):
            bad = (dqkv - ref[3]).abs()
            print("  max |d dqkv|", bad.max().item(), "rows", torch.nonzero(bad.amax(-1) > 0)[:5].tolist())
    print(f"N={N} L={L}: eager twice {eq2}; graph replays {outs}")
    # garbage in every buffer the kernels write: results must not change
    for fill in (-1, 12345, float("nan")):
        bits.fill_(-1 if fill != 12345 else 0x5A5A5A5A)
        o.fill_(float("nan") if fill != 12345 else 3.0)
        lse.fill_(float("nan") if fill != 12345 else -3.0)
        dqkv.fill_(float("nan") if fill != 12345 else 5.0)
        run()
        torch.cuda.synchronize()
        eqg = [torch.equal(a[:N], t[:N]) if i != 2 else True for i, (a, t) in
               enumerate(zip(ref, (o, lse, bits, dqkv)))]
        print(f"   garbage fill {fill}: equal {eqg}")
