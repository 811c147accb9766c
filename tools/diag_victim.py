"""Diagnostic (not product): does the spectra decoder's forward (eager, main stream) give
bitwise the same output while split-f16 attention launches (photometry-decoder shape) run
on a side stream?  SF16_DBG_ONLY_L=60 keeps the decoder itself on the packed-VALU kernels,
so a change names a co-scheduling-sensitive kernel in the decoder path."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vaesne-dev_amd")]
import bench  # noqa: E402
from VAESNe import _lib, rng  # noqa: E402

lib = _lib.lib
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = bench.make_model(dev, 0.0)
x = bench.synthetic_batch(4, 7, dev)
H, E = 4, 32
BS, LS = int(os.environ.get("SB", "96")), int(os.environ.get("SL", "60"))
g = torch.Generator(device=dev).manual_seed(3)
qkv = torch.randn(BS, LS, 3 * E, device=dev, generator=g)
o = torch.empty(BS, LS, E, device=dev)
lse = torch.empty(BS, H, LS, device=dev)
side = torch.cuda.Stream()
K = 3
spec = model.vaes[1]
zs = torch.randn(K, 2 * 4, spec.latent_len, spec.latent_dim, device=dev, generator=g)


def side_load(n):
    b = qkv.data_ptr()
    for _ in range(n):
        assert lib.attn_fwd(b, LS * 3 * E, 3 * E, b + 4 * E, LS * 3 * E, 3 * E, b + 8 * E, LS * 3 * E,
                            3 * E, None, LS, o.data_ptr(), LS * E, E, lse.data_ptr(), BS, H, LS, LS,
                            8, 0.0, None, 0, None, None, side.cuda_stream) == 0


def dec():
    with torch.no_grad():
        loc, scale = spec.decode_params(zs, x[1], groups=2)
    return loc


ref = dec().clone()
torch.cuda.synchronize()
bad = 0
for it in range(int(os.environ.get("ITERS", "40"))):
    side.wait_stream(torch.cuda.current_stream())
    side_load(int(os.environ.get("NS", "30")))
    out = dec()
    torch.cuda.synchronize()
    if not torch.equal(out, ref):
        bad += 1
        if bad <= 5:
            print("iter", it, "max diff", float((out - ref).abs().max()))
print(f"{bad} differing iterations (side: {os.environ.get('SF16_DBG_ONLY_L', 'all sf16')})")
