"""ctypes binding of libvaesne_hip.so (C ABI: include/vaesne_hip.h).

The product path has exactly one implementation: these gfx950 kernels.  There
is no CPU fallback.  If the library is missing, or a tensor handed to an op is
not on a ROCm device, the op raises.  `import torch` happens before the
library is opened, so the library's libamdhip64.so.7 dependency binds to the
HIP runtime torch already loaded (one runtime per process).
"""
from __future__ import annotations

import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAESNE_HIP_LIB",
                          os.path.join(os.path.dirname(_HERE), "lib", "libvaesne_hip.so"))

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
U32 = C.c_uint32
F32 = C.c_float
PP = C.POINTER(C.c_void_p)

# name -> (restype, argtypes).  Mirrors include/vaesne_hip.h one to one.
_ATTN_BWD = (I32, [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, P, I64, I64, P, P, I64, I64, P,
                   I64, I64, P, I64, I64, P, I64, I64, I32, I32, I32, I32, I32, F32, P, U32, P,
                   P, P])

SIGNATURES = {
    "vaesne_linear_fwd": (I32, [P, I64, P, I64, I64, I32, P, P, I32, P, I64, P, I64, I32, I32, P]),
    "vaesne_linear_bwd_data": (I32, [P, I64, P, I64, I32, I64, I32, P, I32, P, I64, I32, P]),
    "vaesne_linear_bwd_weight_workspace": (I64, [I64, I32, I32]),
    "vaesne_linear_bwd_weight": (I32, [P, I64, P, I64, I32, P, I64, P, I64, I64, I32, I32, P, P,
                                       I32, P, P, P]),
    "vaesne_colsum_flush": (I32, [P, P]),
    "vaesne_mlp_head_fwd": (I32, [P, I64, P, I64, I64, I32, P, P, P, P, P, P]),
    "vaesne_mlp_head_bwd_workspace": (I64, [I64, I32]),
    "vaesne_mlp_head_bwd": (I32, [P, I64, P, I64, P, I64, I32, P, P, P, P, P, P, P, P, P, P]),
    "vaesne_add_ln_fwd": (I32, [P, I64, P, I64, I64, I32, P, P, F32, P, U32, P, I64, P, P, P]),
    "vaesne_add_ln_bwd_workspace": (I64, [I64, I32]),
    "vaesne_add_ln_bwd": (I32, [P, I64, P, I64, P, I64, I64, I32, P, P, P, F32, P, U32, P, I64,
                                I32, P, I64, I32, P, P, I32, P, P, P]),
    "vaesne_reduce_partials": (I32, [P, I32, I32, P, P, I32, I32, P]),
    "vaesne_mask_bias": (I32, [P, I64, P, P]),
    "vaesne_attn_keep_bits_size": (I64, [I32, I32, I32, I32]),
    "vaesne_attn_workspace": (I64, [I32, I32, I32, I32, I32, I32]),
    "vaesne_attn_fwd": (I32, [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, P, I64, I64, P, I32,
                              I32, I32, I32, I32, F32, P, U32, P, P, P]),
    "vaesne_attn_bwd": _ATTN_BWD,
    "vaesne_attn_bwd_kv": _ATTN_BWD,
    "vaesne_attn_bwd_q": _ATTN_BWD,
    "vaesne_dec_tail_workspace": (I64, [I32, I32, I32]),
    "vaesne_dec_tail_fwd": (I32, [P, P, P, I32, I32, I32, PP, F32, P, U32, P, P, P, P]),
    "vaesne_dec_tail_bwd": (I32, [P, P, P, I32, I32, I32, PP, F32, P, U32, P, P, P, P, P, P, P,
                                  P, P, P, P]),
    "vaesne_dec_tail_grad_layout": (I32, [C.POINTER(I32)]),
    "vaesne_dec_tail_force_path": (I32, [I32]),
    "vaesne_enc_block_workspace": (I64, [I32]),
    "vaesne_attn_force_geometry": (I32, [I32, I32]),
    "vaesne_attn_rep_workspace": (I64, [I32, I32, I32, I32, I32, F32]),
    "vaesne_attn_rep_fwd": (I32, [P, I64, I64, P, I64, P, I64, I64, P, I32, I32, I32, I32, I32, F32,
                                  P, U32, P, P]),
    "vaesne_attn_rep_fwd_part": (I32, [P, I64, I64, P, I64, P, I64, I64, P, I32, I32, I32, I32, I32,
                                       F32, P, U32, P, I32, I32, I32, P]),
    "vaesne_attn_rep_bwd": (I32, [P, I64, I64, P, I64, P, I64, I64, P, P, P, I32, I32, I32, I32, I32,
                                  F32, P, U32, P, P, P]),
    "vaesne_attn_rep_config": (I32, [I32, I32, I32, I32, I32, I32, I32]),
    "vaesne_attn_rep_sf16_config": (I32, [I32, I32]),
    "vaesne_enc_block_fwd": (I32, [I32, P, P, I32, PP, F32, P, U32, P, P, P, P]),
    "vaesne_enc_block_bwd": (I32, [I32, P, P, I32, PP, F32, P, U32, P, P, P, P, P, P, P, P, P,
                                   P]),
    "vaesne_linear_fwd_group": (I32, [I32, P, I32, I32, P]),
    "vaesne_linear_bwd_data_group": (I32, [I32, P, I32, I32, P]),
    "vaesne_linear_bwd_weight_group_workspace": (I64, [I32, I64, I32, I32]),
    "vaesne_linear_bwd_weight_group": (I32, [I32, P, I64, I32, I32, P, P, P]),
    "vaesne_enc_chain_layout": (I32, [P, P, P]),
    "vaesne_enc_chain_fwd": (I32, [I32, P, P]),
    "vaesne_enc_chain_bwd": (I32, [I32, P, P, P]),
    "vaesne_sincos": (I32, [P, I64, I64, P, I32, P, I64, P]),
    "vaesne_embed_fwd": (I32, [P, I64, I64, P, I32, P, I64, P, I64, P]),
    "vaesne_embed_bwd_workspace": (I64, [I64, I32, I32]),
    "vaesne_embed_bwd": (I32, [P, I64, I64, P, I64, I32, I32, P, I32, P, P, P]),
    "vaesne_sum_leading": (I32, [P, I32, I32, P, I32, P]),
    "vaesne_sum_n": (I32, [PP, I32, I64, P, P]),
    "vaesne_latent_head_fwd": (I32, [P, I32, I32, P, P, P, P]),
    "vaesne_latent_head_bwd": (I32, [P, I32, I32, P, P, P, P]),
    "vaesne_uniform": (I32, [P, I64, P, U32, P]),
    "vaesne_rsample_fwd": (I32, [P, P, P, I32, I64, P, P]),
    "vaesne_rsample_bwd": (I32, [P, P, I32, I64, P, P, P]),
    "vaesne_rsample_bwd_acc": (I32, [P, P, I32, I64, P, P, P, P, P]),
    "vaesne_cat_grad": (I32, [PP, I32, PP, I32, I32, I64, PP, P]),
    "vaesne_mask_scale": (I32, [P, I64, I32, F32, P, P]),
    "vaesne_bright_input_fwd": (I32, [P, I64, I32, P, I64, I64, P, P]),
    "vaesne_bright_input_bwd": (I32, [P, I32, I64, I32, I64, P, P]),
    "vaesne_bright_shift_fwd": (I32, [P, P, I64, I32, P, P]),
    "vaesne_bright_shift_bwd": (I32, [P, I64, I32, P, P, P]),
    "vaesne_iwae_lw_fwd": (I32, [PP, C.POINTER(F32), C.POINTER(I32), PP, PP, C.POINTER(I64), PP,
                                 PP, PP, P, P, I32, I32, I32, P, P]),
    "vaesne_iwae_lw_bwd": (I32, [PP, C.POINTER(F32), C.POINTER(I32), PP, PP, C.POINTER(I64), PP,
                                 PP, PP, P, P, I32, I32, I32, P, PP, PP, PP, PP, P]),
    "vaesne_lme_sum_fwd": (I32, [P, I32, I32, P, P, P]),
    "vaesne_lme_sum_bwd": (I32, [P, I32, I32, P, P, P]),
    "vaesne_elbo_fwd": (I32, [P, I32, F32, P, P, P, P, P, P, I32, I32, I32, P, P, P, P]),
    "vaesne_elbo_bwd": (I32, [P, I32, F32, P, P, P, P, P, P, I32, I32, I32, P, P, P, P, P]),
    "vaesne_infonce_fwd": (I32, [P, P, I32, I32, F32, P, P, P, P, P, P]),
    "vaesne_infonce_bwd": (I32, [P, P, P, I32, I32, F32, P, P, P, P]),
    "vaesne_adamw": (I32, [P, P, P, P, I64, P, P, F32, F32, F32, F32, F32, P, P]),
    "vaesne_adamw_steps_advance": (I32, [P, P, I32, P, P]),
    "vaesne_adamw_list": (I32, [PP, PP, PP, PP, C.POINTER(I64), C.POINTER(I32), C.POINTER(F32),
                                I32, P, I32, P]),
    "vaesne_step_advance": (I32, [P, P, P]),
    "vaesne_stamp": (I32, [P, I32, P]),
    "vaesne_loss_stat": (I32, [P, F32, P, P, P]),
    "vaesne_pack": (I32, [PP, C.POINTER(I64), C.POINTER(I64), I32, P, I32, P]),
    "vaesne_cat": (I32, [PP, C.POINTER(I64), I32, I64, P, P]),
}

# int-returning entry points whose result is a value, not a hipError_t
VALUE_RETURNING = {"vaesne_dec_tail_grad_layout"}

_lib = None


def load():
    """Open the library (once) and bind every symbol; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"VAESNe HIP library not found at {LIB_PATH}. Build it with "
            "`python vaesne-dev_amd/build_lib.py` (or __graft_entry__.build()); "
            "the VAESNe package has no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class _Fn:
    """Attribute access -> checked library call (raises RuntimeError on a HIP error)."""

    def __getattr__(self, name):
        fn = getattr(load(), "vaesne_" + name)

        def call(*args):
            rc = fn(*args)
            if fn.restype is I32 and rc != 0 and ("vaesne_" + name) not in VALUE_RETURNING:
                raise RuntimeError(f"vaesne_{name} failed: hipError {rc}")
            return rc
        return call


lib = _Fn()


def stream() -> int:
    """hipStream_t of torch's current stream (so launches are stream-ordered
    with torch and captured by torch.cuda.graph)."""
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def ptr_array(ts):
    arr = (C.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "VAESNe (MI355X build) runs on ROCm devices only: move the model and the batch "
                "to 'cuda' (HIP) first; there is no CPU path.")
