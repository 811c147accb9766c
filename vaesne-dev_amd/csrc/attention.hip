// Masked multi-head attention core for VAESNe (head_dim 8): the arithmetic of
// torch.nn.MultiheadAttention's slow path as the reference calls it
// (util_layers.py:289,297,301 -> torch/nn/functional.py:6559-6594):
//     S = (q / sqrt(dh)) k^T ;  S[:, j] += kbias[j]  (0, or -inf where key_padding_mask)
//     P = softmax(S) ;  A = Dropout_p(P) ;  O = A v
// Flash-style: scores never touch memory.  Scores live in the log2 domain
// (q pre-multiplied by log2(e)/sqrt(dh)) so each exponential is one v_exp_f32.
//
// gfx950 design (head_dim 8 is too thin for MFMA tiles to pay, so the dot
// products run on the packed-FP32 VALU, 2 FMAs per lane per instruction):
//   * one 64-lane wave per workgroup; each lane owns TWO queries (fwd, dQ) or
//     TWO adjacent keys (dK/dV) held as packed float2 pairs -> v_pk_fma_f32;
//   * the streamed operand (keys in fwd/dQ, queries in dK/dV) is wave-uniform:
//     it is read with scalar loads (s_load_dwordx8) into SGPRs and fed to the
//     VALU as a broadcast operand — no LDS, no barriers, no bank conflicts;
//   * D = rowsum(dO * O) is computed where needed (no separate pre-pass);
//   * dropout: one 32-bit counter hash per (row, key pair) -> two 16-bit keep
//     draws; fwd, dK/dV and dQ regenerate identical masks.
#include "common.h"

using namespace vaesne;

namespace {

constexpr int NT = 64;   // one wave per workgroup

typedef float f2 __attribute__((ext_vector_type(2)));

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
  int B, H, Lq, Lk;
  float scale;        // 1/sqrt(dh)
  float scale_log2;   // log2(e)/sqrt(dh)
  uint32_t thr; float inv_keep;
  const int64_t* rng_state; uint32_t call_id;
};

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f2 ex2(f2 x) { return (f2){ex2(x.x), ex2(x.y)}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(float s) { return (f2){s, s}; }

template <int DH>
__device__ __forceinline__ void ld8(const float* __restrict__ p, float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 a = *reinterpret_cast<const float4*>(p + d);
    r[d] = a.x; r[d + 1] = a.y; r[d + 2] = a.z; r[d + 3] = a.w;
  }
}
template <int DH>
__device__ __forceinline__ void st8(float* __restrict__ p, const float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4)
    *reinterpret_cast<float4*>(p + d) = make_float4(r[d], r[d + 1], r[d + 2], r[d + 3]);
}

// keep decisions for keys (2kp, 2kp+1) of a row: bit0 / bit1
__device__ __forceinline__ uint32_t keep2(uint32_t row_key, uint32_t kp, uint32_t thr) {
  const uint32_t bits = attn_pair_bits(row_key, kp);
  return ((bits & 0xffffu) >= thr ? 1u : 0u) | ((bits >> 16) >= thr ? 2u : 0u);
}

// ============================== forward ====================================
// lane owns queries i0 = qb*128 + lane and i1 = i0 + 64 (packed .x / .y)
template <int DH, bool DROP>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(AttnArgs a) {
  const int nqb = (a.Lq + 2 * NT - 1) / (2 * NT);
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int lane = threadIdx.x;
  const int i0 = qb * 2 * NT + lane, i1 = i0 + NT;
  const int c0 = min(i0, a.Lq - 1), c1 = min(i1, a.Lq - 1);
  float qa[DH], qc[DH];
  ld8(a.q + (int64_t)b * a.q_bs + (int64_t)c0 * a.q_ls + h * DH, qa);
  ld8(a.q + (int64_t)b * a.q_bs + (int64_t)c1 * a.q_ls + h * DH, qc);
  f2 q[DH], o[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    q[d] = (f2){qa[d], qc[d]} * a.scale_log2;
    o[d] = bc(0.f);
  }
  f2 m = bc(-INFINITY), l = bc(0.f);
  uint32_t rk0 = 0, rk1 = 0;
  if (DROP) {
    const uint32_t skey = key_of(a.rng_state, a.call_id);
    rk0 = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + c0));
    rk1 = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + c1));
  }
  const float* __restrict__ kp = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* __restrict__ vp = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* __restrict__ kb = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;

  constexpr int G = 8;   // keys per online-softmax update
  for (int j0 = 0; j0 < a.Lk; j0 += G) {
    f2 s[G];
    f2 mx = m;
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int j = j0 + u;
      if (j < a.Lk) {
        const float* kr = kp + (int64_t)j * a.k_ls;
        f2 acc = bc(kb ? kb[j] : 0.f);
#pragma unroll
        for (int d = 0; d < DH; ++d) acc = fma2(q[d], bc(kr[d]), acc);
        s[u] = acc;
      } else {
        s[u] = bc(-INFINITY);
      }
      mx = __builtin_elementwise_max(mx, s[u]);
    }
    // all-masked-so-far rows keep m = -inf; use 0 as the exponent origin then
    const f2 mu = (f2){mx.x == -INFINITY ? 0.f : mx.x, mx.y == -INFINITY ? 0.f : mx.y};
    const f2 corr = ex2(m - mu);
    m = mx;
    l *= corr;
#pragma unroll
    for (int d = 0; d < DH; ++d) o[d] *= corr;
#pragma unroll
    for (int u = 0; u < G; u += 2) {
      const int j = j0 + u;
      if (j >= a.Lk) break;
      f2 p0 = ex2(s[u] - mu), p1 = ex2(s[u + 1] - mu);
      l += p0 + p1;
      if (DROP) {
        const uint32_t kpair = (uint32_t)(j >> 1);
        const uint32_t k0 = keep2(rk0, kpair, a.thr), k1 = keep2(rk1, kpair, a.thr);
        p0 = (f2){(k0 & 1u) ? p0.x : 0.f, (k1 & 1u) ? p0.y : 0.f};
        p1 = (f2){(k0 & 2u) ? p1.x : 0.f, (k1 & 2u) ? p1.y : 0.f};
      }
      const float* vr0 = vp + (int64_t)j * a.v_ls;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = fma2(p0, bc(vr0[d]), o[d]);
      if (j + 1 < a.Lk) {
        const float* vr1 = vp + (int64_t)(j + 1) * a.v_ls;
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] = fma2(p1, bc(vr1[d]), o[d]);
      }
    }
  }
  // l == 0 (every key masked) -> 0/0 = NaN, as the reference's -inf softmax
  const f2 inv = bc(DROP ? a.inv_keep : 1.f) / l;
  float r0[DH], r1[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) { r0[d] = o[d].x * inv.x; r1[d] = o[d].y * inv.y; }
  if (i0 < a.Lq) {
    st8(a.o_out + (int64_t)b * a.o_bs + (int64_t)i0 * a.o_ls + h * DH, r0);
    a.lse[(int64_t)bh * a.Lq + i0] = m.x + __log2f(l.x);
  }
  if (i1 < a.Lq) {
    st8(a.o_out + (int64_t)b * a.o_bs + (int64_t)i1 * a.o_ls + h * DH, r1);
    a.lse[(int64_t)bh * a.Lq + i1] = m.y + __log2f(l.y);
  }
}

// ============================== dK, dV =====================================
// lane owns keys k0 = kb*128 + 2*lane, k0 + 1 (packed .x / .y); queries stream
template <int DH, bool DROP>
__global__ __launch_bounds__(NT) void attn_bwd_kv_kernel(AttnArgs a) {
  const int nkb = (a.Lk + 2 * NT - 1) / (2 * NT);
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int lane = threadIdx.x;
  const int key0 = kb * 2 * NT + 2 * lane;
  const int ka = min(key0, a.Lk - 1), kc = min(key0 + 1, a.Lk - 1);
  float ta[DH], tc[DH];
  f2 k[DH], v[DH], dk[DH], dv[DH];
  ld8(a.k + (int64_t)b * a.k_bs + (int64_t)ka * a.k_ls + h * DH, ta);
  ld8(a.k + (int64_t)b * a.k_bs + (int64_t)kc * a.k_ls + h * DH, tc);
#pragma unroll
  for (int d = 0; d < DH; ++d) { k[d] = (f2){ta[d], tc[d]} * a.scale_log2; dk[d] = bc(0.f); dv[d] = bc(0.f); }
  ld8(a.v + (int64_t)b * a.v_bs + (int64_t)ka * a.v_ls + h * DH, ta);
  ld8(a.v + (int64_t)b * a.v_bs + (int64_t)kc * a.v_ls + h * DH, tc);
#pragma unroll
  for (int d = 0; d < DH; ++d) v[d] = (f2){ta[d], tc[d]};
  // masked / out-of-range keys: bias -inf -> p = 0 -> no contribution
  f2 kbias = bc(0.f);
  {
    const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
    kbias.x = key0 < a.Lk ? (kbp ? kbp[key0] : 0.f) : -INFINITY;
    kbias.y = key0 + 1 < a.Lk ? (kbp ? kbp[key0 + 1] : 0.f) : -INFINITY;
  }
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;
  const uint32_t kpair = (uint32_t)(key0 >> 1);
  const float* __restrict__ qp = a.q + (int64_t)b * a.q_bs + h * DH;
  const float* __restrict__ dop = a.dout + (int64_t)b * a.do_bs + h * DH;
  const float* __restrict__ op = a.o + (int64_t)b * a.o_bs + h * DH;
  const float* __restrict__ lp = a.lse + (int64_t)bh * a.Lq;
#pragma unroll 2
  for (int i = 0; i < a.Lq; ++i) {
    const float* qr = qp + (int64_t)i * a.q_ls;
    const float* dr = dop + (int64_t)i * a.do_ls;
    const float* orow = op + (int64_t)i * a.o_ls;
    float Di = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) Di = fmaf(dr[d], orow[d], Di);
    f2 s = kbias, dA = bc(0.f);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      s = fma2(k[d], bc(qr[d]), s);
      dA = fma2(v[d], bc(dr[d]), dA);
    }
    const f2 p = ex2(s - bc(lp[i]));
    f2 aP = p, dP = dA;
    if (DROP) {
      const uint32_t kk = keep2(attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + i)), kpair, a.thr);
      aP = (f2){(kk & 1u) ? p.x * a.inv_keep : 0.f, (kk & 2u) ? p.y * a.inv_keep : 0.f};
      dP = (f2){(kk & 1u) ? dA.x * a.inv_keep : 0.f, (kk & 2u) ? dA.y * a.inv_keep : 0.f};
    }
    const f2 dS = p * (dP - bc(Di));
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      dv[d] = fma2(aP, bc(dr[d]), dv[d]);
      dk[d] = fma2(dS, bc(qr[d]), dk[d]);
    }
  }
  float r0[DH], r1[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) { r0[d] = dk[d].x * a.scale; r1[d] = dk[d].y * a.scale; }
  if (key0 < a.Lk) st8(a.dk + (int64_t)b * a.dk_bs + (int64_t)key0 * a.dk_ls + h * DH, r0);
  if (key0 + 1 < a.Lk) st8(a.dk + (int64_t)b * a.dk_bs + (int64_t)(key0 + 1) * a.dk_ls + h * DH, r1);
#pragma unroll
  for (int d = 0; d < DH; ++d) { r0[d] = dv[d].x; r1[d] = dv[d].y; }
  if (key0 < a.Lk) st8(a.dv + (int64_t)b * a.dv_bs + (int64_t)key0 * a.dv_ls + h * DH, r0);
  if (key0 + 1 < a.Lk) st8(a.dv + (int64_t)b * a.dv_bs + (int64_t)(key0 + 1) * a.dv_ls + h * DH, r1);
}

// ================================ dQ =======================================
template <int DH, bool DROP>
__global__ __launch_bounds__(NT) void attn_bwd_q_kernel(AttnArgs a) {
  const int nqb = (a.Lq + 2 * NT - 1) / (2 * NT);
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int lane = threadIdx.x;
  const int i0 = qb * 2 * NT + lane, i1 = i0 + NT;
  const int c0 = min(i0, a.Lq - 1), c1 = min(i1, a.Lq - 1);
  float ta[DH], tc[DH], ua[DH], uc[DH];
  f2 q[DH], dov[DH], dq[DH];
  ld8(a.q + (int64_t)b * a.q_bs + (int64_t)c0 * a.q_ls + h * DH, ta);
  ld8(a.q + (int64_t)b * a.q_bs + (int64_t)c1 * a.q_ls + h * DH, tc);
#pragma unroll
  for (int d = 0; d < DH; ++d) { q[d] = (f2){ta[d], tc[d]} * a.scale_log2; dq[d] = bc(0.f); }
  ld8(a.dout + (int64_t)b * a.do_bs + (int64_t)c0 * a.do_ls + h * DH, ta);
  ld8(a.dout + (int64_t)b * a.do_bs + (int64_t)c1 * a.do_ls + h * DH, tc);
  ld8(a.o + (int64_t)b * a.o_bs + (int64_t)c0 * a.o_ls + h * DH, ua);
  ld8(a.o + (int64_t)b * a.o_bs + (int64_t)c1 * a.o_ls + h * DH, uc);
  f2 D = bc(0.f);
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    dov[d] = (f2){ta[d], tc[d]};
    D = fma2(dov[d], (f2){ua[d], uc[d]}, D);
  }
  const f2 lse = (f2){a.lse[(int64_t)bh * a.Lq + c0], a.lse[(int64_t)bh * a.Lq + c1]};
  uint32_t rk0 = 0, rk1 = 0;
  if (DROP) {
    const uint32_t skey = key_of(a.rng_state, a.call_id);
    rk0 = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + c0));
    rk1 = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + c1));
  }
  const float* __restrict__ kp = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* __restrict__ vp = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* __restrict__ kb = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  for (int j = 0; j < a.Lk; j += 2) {
    uint32_t k0 = 3u, k1 = 3u;
    if (DROP) {
      k0 = keep2(rk0, (uint32_t)(j >> 1), a.thr);
      k1 = keep2(rk1, (uint32_t)(j >> 1), a.thr);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int jj = j + u;
      if (jj >= a.Lk) break;
      const float* kr = kp + (int64_t)jj * a.k_ls;
      const float* vr = vp + (int64_t)jj * a.v_ls;
      f2 s = bc(kb ? kb[jj] : 0.f), dA = bc(0.f);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        s = fma2(q[d], bc(kr[d]), s);
        dA = fma2(dov[d], bc(vr[d]), dA);
      }
      const f2 p = ex2(s - lse);
      f2 dP = dA;
      if (DROP) {
        const uint32_t m = 1u << u;
        dP = (f2){(k0 & m) ? dA.x * a.inv_keep : 0.f, (k1 & m) ? dA.y * a.inv_keep : 0.f};
      }
      const f2 dS = p * (dP - D);
#pragma unroll
      for (int d = 0; d < DH; ++d) dq[d] = fma2(dS, bc(kr[d]), dq[d]);
    }
  }
  float r0[DH], r1[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) { r0[d] = dq[d].x * a.scale; r1[d] = dq[d].y * a.scale; }
  if (i0 < a.Lq) st8(a.dq + (int64_t)b * a.dq_bs + (int64_t)i0 * a.dq_ls + h * DH, r0);
  if (i1 < a.Lq) st8(a.dq + (int64_t)b * a.dq_bs + (int64_t)i1 * a.dq_ls + h * DH, r1);
}

__global__ void mask_bias_kernel(const uint8_t* __restrict__ m, int64_t n, float* __restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = m[t] ? -INFINITY : 0.f;
}

bool aligned16(const void* p, int64_t ls) {
  return ((uintptr_t)p % 16 == 0) && (ls % 4 == 0);
}

void fill_common(AttnArgs& a, int B, int H, int Lq, int Lk, int dh, float p_drop,
                 const int64_t* rng_state, uint32_t call_id) {
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.scale = 1.0f / sqrtf((float)dh);
  a.scale_log2 = a.scale * 1.4426950408889634f;
  a.thr = drop_thr16(p_drop);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.rng_state = rng_state; a.call_id = call_id;
}

template <int DHV>
int launch_fwd(const AttnArgs& a, float p_drop, hipStream_t s) {
  const int nqb = (a.Lq + 2 * NT - 1) / (2 * NT);
  dim3 grid((unsigned)((int64_t)a.B * a.H * nqb));
  if (p_drop > 0.f)
    hipLaunchKernelGGL((attn_fwd_kernel<DHV, true>), grid, dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<DHV, false>), grid, dim3(NT), 0, s, a);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

template <int DHV>
int launch_bwd(const AttnArgs& a, float p_drop, hipStream_t s) {
  const int nkb = (a.Lk + 2 * NT - 1) / (2 * NT);
  const int nqb = (a.Lq + 2 * NT - 1) / (2 * NT);
  dim3 gkv((unsigned)((int64_t)a.B * a.H * nkb)), gq((unsigned)((int64_t)a.B * a.H * nqb));
  if (p_drop > 0.f) {
    hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, true>), gkv, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, true>), gq, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, false>), gkv, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, false>), gq, dim3(NT), 0, s, a);
  }
  VAESNE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

VAESNE_API int vaesne_mask_bias(const uint8_t* mask, int64_t n, float* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mask_bias_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, mask, n, out);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_attn_fwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const float* kbias, int64_t kb_bs, float* o,
                               int64_t o_bs, int64_t o_ls, float* lse, int B, int H, int Lq,
                               int Lk, int dh, float p_drop, const int64_t* rng_state,
                               uint32_t call_id, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || (dh != 8 && dh != 16) || H * dh > 4096) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls))
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.q_bs = q_bs; a.q_ls = q_ls;
  a.k = k; a.k_bs = k_bs; a.k_ls = k_ls;
  a.v = v; a.v_bs = v_bs; a.v_ls = v_ls;
  a.kbias = kbias; a.kb_bs = kb_bs;
  a.o = o; a.o_out = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = lse;
  fill_common(a, B, H, Lq, Lk, dh, p_drop, rng_state, call_id);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return launch_fwd<8>(a, p_drop, s);
  return launch_fwd<16>(a, p_drop, s);
}

VAESNE_API int vaesne_attn_bwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const float* kbias, int64_t kb_bs, const float* o,
                               int64_t o_bs, int64_t o_ls, const float* lse, const float* dout,
                               int64_t do_bs, int64_t do_ls, float* dq, int64_t dq_bs,
                               int64_t dq_ls, float* dk, int64_t dk_bs, int64_t dk_ls, float* dv,
                               int64_t dv_bs, int64_t dv_ls, int B, int H, int Lq, int Lk, int dh,
                               float p_drop, const int64_t* rng_state, uint32_t call_id,
                               void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || (dh != 8 && dh != 16) || H * dh > 4096) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls) ||
      !aligned16(dout, do_ls) || !aligned16(dq, dq_ls) || !aligned16(dk, dk_ls) ||
      !aligned16(dv, dv_ls))
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.q_bs = q_bs; a.q_ls = q_ls;
  a.k = k; a.k_bs = k_bs; a.k_ls = k_ls;
  a.v = v; a.v_bs = v_bs; a.v_ls = v_ls;
  a.kbias = kbias; a.kb_bs = kb_bs;
  a.o = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = const_cast<float*>(lse);
  a.dout = dout; a.do_bs = do_bs; a.do_ls = do_ls;
  a.dq = dq; a.dq_bs = dq_bs; a.dq_ls = dq_ls;
  a.dk = dk; a.dk_bs = dk_bs; a.dk_ls = dk_ls;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_ls = dv_ls;
  fill_common(a, B, H, Lq, Lk, dh, p_drop, rng_state, call_id);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return launch_bwd<8>(a, p_drop, s);
  return launch_bwd<16>(a, p_drop, s);
}
