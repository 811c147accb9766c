"""Per-phase timing of the fused encoder-chain kernels (csrc/enc_chain.hip built with
VAESNE_CHAIN_PROFILE: thread 0 of each workgroup stamps wall_clock64() (100 MHz) at
the phase boundaries of every block).  Prints the mean phase durations (us) over the
sequences and blocks of cfg-5-shaped encoders (B 16, T 8, 4 blocks, dropout 0.1):
the photometry chain (60 context tokens) and the spectra chain (984).

    python -c "import sys; sys.path.insert(0,'vaesne-dev_amd'); import build_lib; \
        build_lib.build_profile_lib('vaesne-dev_amd/lib/libvaesne_hip_prof.so')"   # CPU box
    python tools/chain_phases.py                                                    # GPU box
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VAESNE_HIP_LIB"] = os.path.join(ROOT, "vaesne-dev_amd", "lib", "libvaesne_hip_prof.so")
sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from VAESNe import _lib  # noqa: E402
from VAESNe.util_layers import TransformerBlock, encoder_stack  # noqa: E402

FWD = ["stage", "in_proj", "self-attn", "PRE", "cross-attn", "POST"]
BWD = ["stage", "POST bwd", "cross bwd", "PRE bwd", "self-attn bwd", "partials"]


def run(Lk, selfattn, reps=5):
    torch.manual_seed(0)
    blocks = torch.nn.ModuleList([TransformerBlock(32, 4, 32, 0.1, selfattn) for _ in range(4)]).cuda()
    blocks.train()
    B, T = 16, 8
    x = torch.randn(B, T, 32, device="cuda", requires_grad=True)
    ctx = torch.randn(B, Lk, 32, device="cuda", requires_grad=True)
    mask = torch.zeros(B, Lk, dtype=torch.bool, device="cuda")
    mask[:, -5:] = True
    lib = _lib.load()
    fn = lib.vaesne_enc_chain_profile_read
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p]
    buf = np.zeros((2, 2, 64, 6, 8), dtype=np.uint64)
    acc = {0: [], 1: []}
    for _ in range(reps):
        out = encoder_stack(blocks, x, ctx, context_mask=mask)
        out.sum().backward()
        torch.cuda.synchronize()
        fn(buf.ctypes.data)
        for d in (0, 1):
            t = buf[d, 0, :B, :4, :7].astype(np.int64)
            acc[d].append(np.diff(t, axis=-1) * 10e-3)        # 100 MHz ticks -> us
            blk_total = (t[:, :, 6] - t[:, :, 0]) * 10e-3
            acc[d][-1] = np.concatenate([acc[d][-1], blk_total[..., None]], axis=-1)
    for d, names in ((0, FWD), (1, BWD)):
        a = np.mean(np.stack(acc[d][1:]), axis=(0, 1))      # [block, phase]
        print(f"  {'fwd' if d == 0 else 'bwd'}: " + "  ".join(
            f"{n} {a[:, i].mean():6.2f}" for i, n in enumerate(names + ['block'])))


if __name__ == "__main__":
    print("photometry chain (Lk 60):")
    run(60, False)
    print("spectra chain (Lk 984, context self-attention):")
    run(984, True)
