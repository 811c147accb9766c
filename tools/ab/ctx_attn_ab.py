"""Isolated timing of the attention launches at the encoders' context self-attention shape
(B*H = 64 sequences x 983 tokens: split launches) and the decoder shape, packed-VALU vs
matrix-core kernels (vaesne_attn_mfma_config).
    python tools/ab/ctx_attn_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    from VAESNe import _lib, rng
    lib = _lib.lib
    dev = torch.device("cuda", 0)
    H, dh, E, pd = 4, 8, 32, 0.1
    for B, L in ((16, 983), (256, 982)):
        qkv = torch.randn(B, L, 3 * E, device=dev)
        mask = torch.rand(B, L, device=dev) < 0.05
        mask[:, 0] = False
        kbias = torch.where(mask, float("-inf"), 0.0).float().contiguous()
        o = torch.empty(B, L, E, device=dev)
        lse = torch.empty(B, H, L, device=dev)
        do = torch.randn(B, L, E, device=dev)
        dqkv = torch.empty_like(qkv)
        st = rng.state(dev)
        bits = torch.empty(lib.attn_keep_bits_size(B, H, L, L), dtype=torch.uint8, device=dev)
        b, d, s3 = qkv.data_ptr(), dqkv.data_ptr(), L * 3 * E
        for cfg in ((0, 0, 0), (4, 0, 0), (0, 4, 0), (0, 4, 1), (0, 8, 0)):
            assert lib.attn_mfma_config(*cfg) == 0
            wf = torch.empty(max(1, lib.attn_workspace(B, H, L, L, dh, 0) // 4), device=dev)
            wb = torch.empty(max(1, lib.attn_workspace(B, H, L, L, dh, 1) // 4), device=dev)

            def fwd():
                lib.attn_fwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E,
                             kbias.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(),
                             B, H, L, L, dh, pd, st.data_ptr(), 7, bits.data_ptr(), 0,
                             wf.data_ptr(), _lib.stream())

            def bwd():
                lib.attn_bwd(b, s3, 3 * E, b + 4 * E, s3, 3 * E, b + 8 * E, s3, 3 * E,
                             kbias.data_ptr(), L, o.data_ptr(), L * E, E, lse.data_ptr(),
                             do.data_ptr(), L * E, E, d, s3, 3 * E, d + 4 * E, s3, 3 * E,
                             d + 8 * E, s3, 3 * E, B, H, L, L, dh, pd, st.data_ptr(), 7,
                             bits.data_ptr(), wb.data_ptr(), _lib.stream())
            fwd()
            tf = bench.time_kernel(fwd, 20, dev)
            tb = bench.time_kernel(bwd, 20, dev)
            print(f"B*H={B * H:5d} L={L} cfg(fwd,bwd,ahead)={cfg}: fwd {tf * 1e3:.4f} ms  "
                  f"bwd {tb * 1e3:.4f} ms", flush=True)
        lib.attn_mfma_config(-2, -1, -1)


if __name__ == "__main__":
    main()
