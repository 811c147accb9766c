"""Probe (not product): do the split-f16 attention launches write outside their outputs?
o / lse / dq / dk / dv / bits are carved out of one buffer with canary words on both
sides; after forward + backward every canary must be intact."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
from VAESNe import _lib, rng  # noqa: E402

lib = _lib.lib
H, E = 4, 32
PAD = 4096
CAN = -12345.5


def carve(big, off, n):
    return big[off:off + n], off + n + PAD


for B, L, p in [(16, 983, 0.0), (96, 60, 0.0), (24, 982, 0.1), (3, 130, 0.1), (2, 1100, 0.1)]:
    g = torch.Generator(device="cuda").manual_seed(B + L)
    qkv = torch.randn(B, L, 3 * E, device="cuda", generator=g)
    do = torch.randn(B, L, E, device="cuda", generator=g)
    nbits = lib.attn_keep_bits_size(B, H, L, L) // 4
    nws = max(lib.attn_workspace(B, H, L, L, 8, 0), lib.attn_workspace(B, H, L, L, 8, 1)) // 4
    sizes = [B * L * E, B * H * L, B * L * 3 * E, nbits, max(1, nws)]
    big = torch.full((sum(sizes) + PAD * (len(sizes) + 1),), CAN, device="cuda")
    off = PAD
    o, off = carve(big, off, sizes[0])
    lse, off = carve(big, off, sizes[1])
    dqkv, off = carve(big, off, sizes[2])
    bitsf, off = carve(big, off, sizes[3])
    ws, off = carve(big, off, sizes[4])
    bits = bitsf.view(torch.int32)
    st = rng.state("cuda")
    b, d = qkv.data_ptr(), dqkv.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    assert lib.attn_fwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        None, L, o.data_ptr(), L * E, E, lse.data_ptr(), B, H, L, L, 8, p,
                        st.data_ptr(), 3, bits.data_ptr(), ws.data_ptr(), s) == 0
    assert lib.attn_bwd(b, L * 3 * E, 3 * E, b + 4 * E, L * 3 * E, 3 * E, b + 8 * E, L * 3 * E, 3 * E,
                        None, L, o.data_ptr(), L * E, E, lse.data_ptr(), do.data_ptr(), L * E, E,
                        d, L * 3 * E, 3 * E, d + 4 * E, L * 3 * E, 3 * E, d + 8 * E, L * 3 * E, 3 * E,
                        B, H, L, L, 8, p, st.data_ptr(), 3, bits.data_ptr(), ws.data_ptr(), s) == 0
    torch.cuda.synchronize()
    mask = torch.ones_like(big, dtype=torch.bool)
    off = PAD
    for n in sizes:
        mask[off:off + n] = False
        off += n + PAD
    broken = (big[mask] != CAN).nonzero()
    print(B, L, p, "canary words overwritten:", broken.numel())
