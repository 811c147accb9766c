// Definitions shared by the attention translation units (attention.hip: packed-VALU and
// few-query kernels, the launchers and the C ABI; attention_sf16.hip: the split-f16
// matrix-core kernels of head_dim 8).
#pragma once
#include "common.h"

namespace vaesne {

// running-max origin of the forward kernels before any key is seen: finite, so neither
// the exponent origin nor a rescale needs a -inf fix-up per group (a row's first finite
// score always moves it, through the lazy rescale, before any exponential reads it;
// fully masked rows keep it with l = 0 -> o = NaN, lse = -inf)
constexpr float M_INIT = -1e30f;

struct AttnArgs {
  const float* q; int64_t q_bs, q_ls;
  const float* k; int64_t k_bs, k_ls;
  const float* v; int64_t v_bs, v_ls;
  const float* kbias; int64_t kb_bs;        // [B, Lk] additive key bias (0 / -inf) or null
  const float* o; int64_t o_bs, o_ls;       // fwd output (bwd input)
  float* o_out;
  float* lse;                               // [B, H, Lq] log2 domain
  const float* dout; int64_t do_bs, do_ls;
  float* dq; int64_t dq_bs, dq_ls;
  float* dk; int64_t dk_bs, dk_ls;
  float* dv; int64_t dv_bs, dv_ls;
  uint32_t* bits;                           // keep bitmap (dropout only; layout per kernel family)
  int B, H, Lq, Lk, nw;
  float scale;        // 1/sqrt(dh)
  float scale_log2;   // log2(e)/sqrt(dh)
  uint32_t thr; float inv_keep;
  const int64_t* rng_state; uint32_t call_id;
  // split launches (gridDim.y chunks, small grids only): chunk y covers keys
  // [y*kchunk, ..) (forward, dQ) or queries [y*qchunk, ..) (dK/dV) and writes
  // partial results at +y*(o_ss | dq_ss | dk_ss); the forward's partial o is
  // un-normalised, with (m, l) per query in ml.  Unsplit: chunk = whole axis.
  int kchunk, qchunk;
  int64_t o_ss, dq_ss, dk_ss;
  float* ml;                                // [split][B*H*Lq][2] or null
};

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// keep-bitmap assembly: w = 2 w + (this lane's bit of the lane mask m) -- one
// v_addc with the compare's lane mask as carry-in, instead of select-to-0/1, shift, or.
// Bits enter at the bottom, so after n pushes the first decision sits at bit n - 1:
// keep_word() shifts and bit-reverses a word of n pushes (the first push at bit 0).
__device__ __forceinline__ uint32_t push_bit(uint32_t w, uint64_t m) {
  uint32_t r;
  uint64_t co;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(w), "s"(m));
  return r;
}
__device__ __forceinline__ uint32_t keep_word(uint32_t w, int n) {
  return __builtin_bitreverse32(w << (32 - n));
}

// ---- the split-f16 matrix-core path (attention_sf16.hip) ----
// taken for head_dim 8 and query-tiled shapes (Lq > 16) unless a geometry is forced
bool sf16_path(int dh, int64_t bh, int Lq, int Lk);
// keep-bitmap bytes / backward workspace floats of that path
int64_t sf16_bits_bytes(int B, int H, int Lq, int Lk);
int64_t sf16_bwd_ws_floats(int B, int H, int Lq, int Lk);
int sf16_fwd(const AttnArgs& a, float p_drop, hipStream_t s);
int sf16_bwd(const AttnArgs& a, float p_drop, float* ws, hipStream_t s);
// the decoders' first block: R copies of each of a.B distinct sequences (vaesne_attn_rep_*),
// taken for L in (16, 1024] unless a geometry is forced
bool sf16_rep_path(int L, int R);
int64_t sf16_rep_bwd_ws_floats(int Bd, int H, int L);
int sf16_rep_fwd(const AttnArgs& a, int R, float p_drop, int p0, int p1, int np, hipStream_t s);
int sf16_rep_bwd(const AttnArgs& a, int R, float* ws, hipStream_t s);
int sf16_rep_config(int frc, int bwgs);

}  // namespace vaesne
