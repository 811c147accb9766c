"""Probe (not product): run the fp32 FMA victim kernels (scalar, packed, asm packed) on one
stream while an aggressor kernel (f16 MFMA 16x16x32, conversions, permlane, exp) runs on
another; count wrong results (each victim lane checks its exact answer)."""
import ctypes
import os
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "probe", "libaggressors.so"))
a, v = torch.cuda.Stream(), torch.cuda.Stream()
out = torch.empty(1 << 16, device="cuda")
bad = torch.zeros(1, dtype=torch.int32, device="cuda")
for agg in [int(a) for a in os.environ.get('AGGS', '-1,0,4').split(',')]:
    for mode in [int(m) for m in os.environ.get('MODES', '0,1,2,3,4,5').split(',')]:
        bad.zero_()
        torch.cuda.synchronize()
        for rep in range(int(os.environ.get("REPS", "20"))):
            if agg >= 0:
                assert L.agg_launch(agg, ctypes.c_void_p(out.data_ptr()), 2048, 20000, ctypes.c_void_p(a.cuda_stream)) == 0
            assert L.victim_launch(mode, 1024, 4000, ctypes.c_void_p(bad.data_ptr()), ctypes.c_void_p(v.cuda_stream)) == 0
        torch.cuda.synchronize()
        print(f"aggressor {['none', 'mfma_f16_16x16x32', 'cvt', 'permlane', 'exp', 'mfma_all', 'bf16_16x16x32', 'f16_16x16x16', 'f32_16x16x4', 'f32_32x32x2'][agg + 1]:>18} victim "
              f"{['scalar fma', 'packed fma', 'asm pk_fma op_sel', 'asm 2 chains 1 apart', 'lds reads + add', 'lds reads + asm pk', 'asm pk op_sel hi', 'pk mul/add neg', 'mov_b64 max3', 'op_sel hi padded', 'op_sel hi indep', 'pk_add op_sel hi', 'pk_mul op_sel hi', 'pk_mul sgpr op_sel hi', 'pk_mov_b32 op_sel hi'][mode]:>18}: {int(bad.item())} wrong lanes", flush=True)
