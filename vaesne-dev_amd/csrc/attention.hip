// Masked multi-head attention core for VAESNe: the arithmetic of
// torch.nn.MultiheadAttention's slow path as the reference calls it
// (util_layers.py:289,297,301 -> torch/nn/functional.py:6559-6594):
//     S = (q / sqrt(dh)) k^T ;  S[:, j] += kbias[j]  (0, or -inf where key_padding_mask)
//     P = softmax(S) ;  A = Dropout_p(P) ;  O = A v
// Flash-style: scores never touch memory.  Scores live in the log2 domain
// (q pre-multiplied by log2(e)/sqrt(dh)) so each exponential is one v_exp_f32.
//
// gfx950 design.  head_dim 8 (the reference's 32/4) is too thin for MFMA
// tiles to pay in fp32, so the dot products run on the packed-FP32 VALU
// (v_pk_fma_f32: 2 FMAs per lane per instruction):
//   * each lane owns FOUR queries (fwd, dQ) or FOUR adjacent keys (dK/dV) as
//     two packed float2 pairs; the streamed operand (K/V tiles, or Q/dO tiles)
//     is staged in LDS by the workgroup and read as wave-wide broadcast
//     ds_read_b128 (4 rows per lane amortise every LDS read);
//   * dropout: the forward draws one 32-bit counter hash per (query, key pair)
//     (two 16-bit keep decisions, p_eff = round(65536 p)/65536) and writes the
//     keep mask as a BITMAP (1 bit per score, [B*H][ceil(Lk/32)][Lq] words:
//     62 MB per 128x4x982^2 layer) so both backward kernels read bits instead
//     of re-hashing;
//   * D = rowsum(dO * O) is computed by the query-tile loaders (no pre-pass).
#include "common.h"

using namespace vaesne;

namespace {

constexpr int TK = 64;   // keys (or queries) per LDS tile

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
  uint32_t* bits;                           // [B*H][nw][Lq] keep bitmap (dropout only)
  int B, H, Lq, Lk, nw;
  float scale;        // 1/sqrt(dh)
  float scale_log2;   // log2(e)/sqrt(dh)
  uint32_t thr; float inv_keep;
  const int64_t* rng_state; uint32_t call_id;
};

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f2 ex2(f2 x) { return (f2){ex2(x.x), ex2(x.y)}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(float s) { return (f2){s, s}; }
__device__ __forceinline__ f2 sel2(uint32_t ma, uint32_t mb, f2 v) {
  return (f2){ma ? v.x : 0.f, mb ? v.y : 0.f};
}

template <int DH>
__device__ __forceinline__ void ldr(const float* __restrict__ p, float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 a = *reinterpret_cast<const float4*>(p + d);
    r[d] = a.x; r[d + 1] = a.y; r[d + 2] = a.z; r[d + 3] = a.w;
  }
}
template <int DH>
__device__ __forceinline__ void str(float* __restrict__ p, const float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4)
    *reinterpret_cast<float4*>(p + d) = make_float4(r[d], r[d + 1], r[d + 2], r[d + 3]);
}
// broadcast read of one LDS row (all lanes read the same address)
template <int DH>
__device__ __forceinline__ void lrow(const float* s, float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 a = *reinterpret_cast<const float4*>(s + d);
    r[d] = a.x; r[d + 1] = a.y; r[d + 2] = a.z; r[d + 3] = a.w;
  }
}

// stage rows [r0, r0 + TK) of a (row-major, stride ls) matrix's head slice
// into LDS [TK][DH] (zeros past `rows`)
template <int DH, int NTT>
__device__ __forceinline__ void stage(float* dst, const float* __restrict__ src, int64_t ls,
                                      int r0, int rows, float mul) {
  constexpr int V4 = DH / 4;
  for (int idx = threadIdx.x; idx < TK * V4; idx += NTT) {
    const int rr = idx / V4, c = (idx - rr * V4) * 4;
    float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + rr < rows) {
      val = *reinterpret_cast<const float4*>(src + (int64_t)(r0 + rr) * ls + c);
      val.x *= mul; val.y *= mul; val.z *= mul; val.w *= mul;
    }
    *reinterpret_cast<float4*>(dst + rr * DH + c) = val;
  }
}

// ============================== forward ====================================
// lane owns queries i + {0, 1, 2, 3} * NTT (pairs A = {0,1}, B = {2,3})
template <int DH, int NTT, bool DROP>
__global__ __launch_bounds__(NTT) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ float Kb[TK];
  constexpr int QB = 4 * NTT;
  const int nqb = (a.Lq + QB - 1) / QB;
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  int qi[4], qc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    qi[u] = qb * QB + u * NTT + threadIdx.x;
    qc[u] = min(qi[u], a.Lq - 1);
  }
  f2 qA[DH], qB[DH], oA[DH], oB[DH];
  {
    float t0[DH], t1[DH], t2[DH], t3[DH];
    const float* qbase = a.q + (int64_t)b * a.q_bs + h * DH;
    ldr<DH>(qbase + (int64_t)qc[0] * a.q_ls, t0);
    ldr<DH>(qbase + (int64_t)qc[1] * a.q_ls, t1);
    ldr<DH>(qbase + (int64_t)qc[2] * a.q_ls, t2);
    ldr<DH>(qbase + (int64_t)qc[3] * a.q_ls, t3);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      qA[d] = (f2){t0[d], t1[d]} * a.scale_log2;
      qB[d] = (f2){t2[d], t3[d]} * a.scale_log2;
      oA[d] = bc(0.f);
      oB[d] = bc(0.f);
    }
  }
  f2 mA = bc(-INFINITY), mB = bc(-INFINITY), lA = bc(0.f), lB = bc(0.f);
  uint32_t rk[4] = {0u, 0u, 0u, 0u};
  if (DROP) {
    const uint32_t skey = key_of(a.rng_state, a.call_id);
#pragma unroll
    for (int u = 0; u < 4; ++u) rk[u] = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + qc[u]));
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;

  for (int kt = 0; kt < a.Lk; kt += TK) {
    __syncthreads();
    stage<DH, NTT>(Ks, kg, a.k_ls, kt, a.Lk, 1.f);
    stage<DH, NTT>(Vs, vg, a.v_ls, kt, a.Lk, 1.f);
    for (int i = threadIdx.x; i < TK; i += NTT)
      Kb[i] = kt + i < a.Lk ? (kbg ? kbg[kt + i] : 0.f) : -INFINITY;
    __syncthreads();
    const int kend = min(TK, a.Lk - kt);
    uint32_t w[4] = {0u, 0u, 0u, 0u};   // keep bits of the current 32-key word
    for (int g0 = 0; g0 < kend; g0 += 8) {
      f2 sA[8], sB[8];
      f2 xA = mA, xB = mB;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float kr[DH];
        lrow<DH>(Ks + (g0 + u) * DH, kr);
        const float kb = Kb[g0 + u];
        f2 aA = bc(kb), aB = bc(kb);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          aA = fma2(qA[d], bc(kr[d]), aA);
          aB = fma2(qB[d], bc(kr[d]), aB);
        }
        sA[u] = aA;
        sB[u] = aB;
        xA = __builtin_elementwise_max(xA, aA);
        xB = __builtin_elementwise_max(xB, aB);
      }
      // rows whose keys are all masked so far keep m = -inf: exponent origin 0
      const f2 uA = (f2){xA.x == -INFINITY ? 0.f : xA.x, xA.y == -INFINITY ? 0.f : xA.y};
      const f2 uB = (f2){xB.x == -INFINITY ? 0.f : xB.x, xB.y == -INFINITY ? 0.f : xB.y};
      const f2 cA = ex2(mA - uA), cB = ex2(mB - uB);
      mA = xA; mB = xB;
      lA *= cA; lB *= cB;
#pragma unroll
      for (int d = 0; d < DH; ++d) { oA[d] *= cA; oB[d] *= cB; }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        f2 pA0 = ex2(sA[u] - uA), pA1 = ex2(sA[u + 1] - uA);
        f2 pB0 = ex2(sB[u] - uB), pB1 = ex2(sB[u + 1] - uB);
        lA += pA0 + pA1;
        lB += pB0 + pB1;
        if (DROP) {
          const uint32_t kp = (uint32_t)((kt + g0 + u) >> 1);
          const int sh = (g0 + u) & 31;
          uint32_t kk[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const uint32_t bits = attn_pair_bits(rk[t], kp);
            kk[t] = ((bits & 0xffffu) >= a.thr ? 1u : 0u) | ((bits >> 16) >= a.thr ? 2u : 0u);
            w[t] |= kk[t] << sh;
          }
          pA0 = sel2(kk[0] & 1u, kk[1] & 1u, pA0);
          pA1 = sel2(kk[0] & 2u, kk[1] & 2u, pA1);
          pB0 = sel2(kk[2] & 1u, kk[3] & 1u, pB0);
          pB1 = sel2(kk[2] & 2u, kk[3] & 2u, pB1);
        }
        float v0[DH], v1[DH];
        lrow<DH>(Vs + (g0 + u) * DH, v0);
        lrow<DH>(Vs + (g0 + u + 1) * DH, v1);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          oA[d] = fma2(pA0, bc(v0[d]), oA[d]);
          oB[d] = fma2(pB0, bc(v0[d]), oB[d]);
          oA[d] = fma2(pA1, bc(v1[d]), oA[d]);
          oB[d] = fma2(pB1, bc(v1[d]), oB[d]);
        }
      }
      if (DROP && (((g0 + 8) & 31) == 0 || g0 + 8 >= kend)) {
        const int word = (kt + g0) >> 5;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (qi[t] < a.Lq) bitp[(int64_t)word * a.Lq + qi[t]] = w[t];
          w[t] = 0u;
        }
      }
    }
  }
  // l == 0 (every key masked) -> 0/0 = NaN, as the reference's -inf softmax
  const float ik = DROP ? a.inv_keep : 1.f;
  const f2 iA = bc(ik) / lA, iB = bc(ik) / lB;
  float r[4][DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    r[0][d] = oA[d].x * iA.x; r[1][d] = oA[d].y * iA.y;
    r[2][d] = oB[d].x * iB.x; r[3][d] = oB[d].y * iB.y;
  }
  const float lse4[4] = {mA.x + __log2f(lA.x), mA.y + __log2f(lA.y), mB.x + __log2f(lB.x),
                         mB.y + __log2f(lB.y)};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (qi[u] < a.Lq) {
      str<DH>(a.o_out + (int64_t)b * a.o_bs + (int64_t)qi[u] * a.o_ls + h * DH, r[u]);
      a.lse[(int64_t)bh * a.Lq + qi[u]] = lse4[u];
    }
  }
}

// ============================== dK, dV =====================================
// lane owns keys k0 .. k0+3 (k0 = 4*lane + block offset): pairs A = {k0, k0+1},
// B = {k0+2, k0+3}; queries stream through LDS tiles
template <int DH, int NTT, bool DROP>
__global__ __launch_bounds__(NTT) void attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Qs[TK * DH];
  __shared__ __attribute__((aligned(16))) float Ds_[TK * DH];   // dO tile
  __shared__ float Ls[TK], Dd[TK];
  __shared__ uint32_t Ws[TK * (4 * NTT / 32)];
  constexpr int KB = 4 * NTT;
  constexpr int NWB = KB / 32;              // bitmap words of this key block
  const int nkb = (a.Lk + KB - 1) / KB;
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int key0 = kb * KB + 4 * threadIdx.x;
  f2 kA[DH], kB_[DH], vA[DH], vB[DH], dkA[DH], dkB[DH], dvA[DH], dvB[DH];
  {
    float t[4][DH];
    const float* kbase = a.k + (int64_t)b * a.k_bs + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) ldr<DH>(kbase + (int64_t)min(key0 + u, a.Lk - 1) * a.k_ls, t[u]);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      kA[d] = (f2){t[0][d], t[1][d]};     // the streamed Q tile carries the scale
      kB_[d] = (f2){t[2][d], t[3][d]};
    }
    const float* vbase = a.v + (int64_t)b * a.v_bs + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) ldr<DH>(vbase + (int64_t)min(key0 + u, a.Lk - 1) * a.v_ls, t[u]);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      vA[d] = (f2){t[0][d], t[1][d]};
      vB[d] = (f2){t[2][d], t[3][d]};
      dkA[d] = bc(0.f); dkB[d] = bc(0.f); dvA[d] = bc(0.f); dvB[d] = bc(0.f);
    }
  }
  f2 bA, bB;   // key bias (-inf for masked or out-of-range keys -> p = 0)
  {
    const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
    float t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = key0 + u < a.Lk ? (kbp ? kbp[key0 + u] : 0.f) : -INFINITY;
    bA = (f2){t[0], t[1]};
    bB = (f2){t[2], t[3]};
  }
  const int wl = threadIdx.x >> 3;               // my bitmap word within the block
  const int sh = (4 * threadIdx.x) & 31;         // my 4 bits within it
  const float* qg = a.q + (int64_t)b * a.q_bs + h * DH;
  const float* dg = a.dout + (int64_t)b * a.do_bs + h * DH;
  const float* og = a.o + (int64_t)b * a.o_bs + h * DH;
  const float* lg = a.lse + (int64_t)bh * a.Lq;
  const uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;
  const int wfirst = kb * NWB;
  for (int qt = 0; qt < a.Lq; qt += TK) {
    __syncthreads();
    stage<DH, NTT>(Qs, qg, a.q_ls, qt, a.Lq, a.scale_log2);
    stage<DH, NTT>(Ds_, dg, a.do_ls, qt, a.Lq, 1.f);
    for (int i = threadIdx.x; i < TK; i += NTT) {
      const int qi = qt + i;
      float Di = 0.f, li = INFINITY;
      if (qi < a.Lq) {
        float x[DH], y[DH];
        ldr<DH>(dg + (int64_t)qi * a.do_ls, x);
        ldr<DH>(og + (int64_t)qi * a.o_ls, y);
#pragma unroll
        for (int d = 0; d < DH; ++d) Di = fmaf(x[d], y[d], Di);
        li = lg[qi];
      }
      Dd[i] = Di;
      Ls[i] = li;     // +inf for padding rows -> p = 0
    }
    if (DROP) {
      for (int idx = threadIdx.x; idx < TK * NWB; idx += NTT) {
        const int i = idx / NWB, wv = idx - i * NWB;
        const int qi = qt + i, word = wfirst + wv;
        Ws[idx] = (qi < a.Lq && word < a.nw) ? bitp[(int64_t)word * a.Lq + qi] : 0u;
      }
    }
    __syncthreads();
    const int qend = min(TK, a.Lq - qt);
    for (int i = 0; i < qend; ++i) {
      float qr[DH], dr[DH];
      lrow<DH>(Qs + i * DH, qr);
      lrow<DH>(Ds_ + i * DH, dr);
      const f2 li = bc(Ls[i]), Di = bc(Dd[i]);
      f2 sA = bA, sB = bB, gA = bc(0.f), gB = bc(0.f);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        sA = fma2(kA[d], bc(qr[d]), sA);
        sB = fma2(kB_[d], bc(qr[d]), sB);
        gA = fma2(vA[d], bc(dr[d]), gA);
        gB = fma2(vB[d], bc(dr[d]), gB);
      }
      const f2 pA = ex2(sA - li), pB = ex2(sB - li);
      f2 aA = pA, aB = pB, dPA = gA, dPB = gB;
      if (DROP) {
        const uint32_t kw = Ws[i * NWB + wl] >> sh;
        const f2 ik = bc(a.inv_keep);
        aA = sel2(kw & 1u, kw & 2u, pA * ik);
        aB = sel2(kw & 4u, kw & 8u, pB * ik);
        dPA = sel2(kw & 1u, kw & 2u, gA * ik);
        dPB = sel2(kw & 4u, kw & 8u, gB * ik);
      }
      const f2 dSA = pA * (dPA - Di), dSB = pB * (dPB - Di);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        dvA[d] = fma2(aA, bc(dr[d]), dvA[d]);
        dvB[d] = fma2(aB, bc(dr[d]), dvB[d]);
        dkA[d] = fma2(dSA, bc(qr[d]), dkA[d]);
        dkB[d] = fma2(dSB, bc(qr[d]), dkB[d]);
      }
    }
  }
  // dK = sum_i dS_i q_i * scale = (scale / scale_log2) * sum_i dS_i Qs_i
  const float kf = a.scale / a.scale_log2;
  float r[4][DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    r[0][d] = dkA[d].x * kf; r[1][d] = dkA[d].y * kf; r[2][d] = dkB[d].x * kf; r[3][d] = dkB[d].y * kf;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (key0 + u < a.Lk) str<DH>(a.dk + (int64_t)b * a.dk_bs + (int64_t)(key0 + u) * a.dk_ls + h * DH, r[u]);
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    r[0][d] = dvA[d].x; r[1][d] = dvA[d].y; r[2][d] = dvB[d].x; r[3][d] = dvB[d].y;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (key0 + u < a.Lk) str<DH>(a.dv + (int64_t)b * a.dv_bs + (int64_t)(key0 + u) * a.dv_ls + h * DH, r[u]);
}

// ================================ dQ =======================================
template <int DH, int NTT, bool DROP>
__global__ __launch_bounds__(NTT) void attn_bwd_q_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ float Kb[TK];
  constexpr int QB = 4 * NTT;
  const int nqb = (a.Lq + QB - 1) / QB;
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  int qi[4], qc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    qi[u] = qb * QB + u * NTT + threadIdx.x;
    qc[u] = min(qi[u], a.Lq - 1);
  }
  f2 qA[DH], qB[DH], gA_[DH], gB_[DH], dqA[DH], dqB[DH];
  f2 DA, DB, lA, lB;
  {
    float t[4][DH], o4[4][DH];
    const float* qbase = a.q + (int64_t)b * a.q_bs + h * DH;
    const float* dbase = a.dout + (int64_t)b * a.do_bs + h * DH;
    const float* obase = a.o + (int64_t)b * a.o_bs + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) ldr<DH>(qbase + (int64_t)qc[u] * a.q_ls, t[u]);
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      qA[d] = (f2){t[0][d], t[1][d]} * a.scale_log2;
      qB[d] = (f2){t[2][d], t[3][d]} * a.scale_log2;
      dqA[d] = bc(0.f); dqB[d] = bc(0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ldr<DH>(dbase + (int64_t)qc[u] * a.do_ls, t[u]);
      ldr<DH>(obase + (int64_t)qc[u] * a.o_ls, o4[u]);
    }
    float Dv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      gA_[d] = (f2){t[0][d], t[1][d]};
      gB_[d] = (f2){t[2][d], t[3][d]};
#pragma unroll
      for (int u = 0; u < 4; ++u) Dv[u] = fmaf(t[u][d], o4[u][d], Dv[u]);
    }
    DA = (f2){Dv[0], Dv[1]};
    DB = (f2){Dv[2], Dv[3]};
    const float* lp = a.lse + (int64_t)bh * a.Lq;
    lA = (f2){lp[qc[0]], lp[qc[1]]};
    lB = (f2){lp[qc[2]], lp[qc[3]]};
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  const uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;
  const f2 ik = bc(DROP ? a.inv_keep : 1.f);
  for (int kt = 0; kt < a.Lk; kt += TK) {
    __syncthreads();
    stage<DH, NTT>(Ks, kg, a.k_ls, kt, a.Lk, 1.f);
    stage<DH, NTT>(Vs, vg, a.v_ls, kt, a.Lk, 1.f);
    for (int i = threadIdx.x; i < TK; i += NTT)
      Kb[i] = kt + i < a.Lk ? (kbg ? kbg[kt + i] : 0.f) : -INFINITY;
    __syncthreads();
    const int kend = min(TK, a.Lk - kt);
    uint32_t w[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    for (int j = 0; j < kend; ++j) {
      if (DROP && (j & 31) == 0) {
        const int word = (kt + j) >> 5;
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = bitp[(int64_t)word * a.Lq + qc[u]];
      }
      float kr[DH], vr[DH];
      lrow<DH>(Ks + j * DH, kr);
      lrow<DH>(Vs + j * DH, vr);
      const float kb = Kb[j];
      f2 sA = bc(kb), sB = bc(kb), tA = bc(0.f), tB = bc(0.f);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        sA = fma2(qA[d], bc(kr[d]), sA);
        sB = fma2(qB[d], bc(kr[d]), sB);
        tA = fma2(gA_[d], bc(vr[d]), tA);
        tB = fma2(gB_[d], bc(vr[d]), tB);
      }
      const f2 pA = ex2(sA - lA), pB = ex2(sB - lB);
      f2 dPA = tA * ik, dPB = tB * ik;
      if (DROP) {
        const int s = j & 31;
        dPA = sel2((w[0] >> s) & 1u, (w[1] >> s) & 1u, dPA);
        dPB = sel2((w[2] >> s) & 1u, (w[3] >> s) & 1u, dPB);
      }
      const f2 dSA = pA * (dPA - DA), dSB = pB * (dPB - DB);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        dqA[d] = fma2(dSA, bc(kr[d]), dqA[d]);
        dqB[d] = fma2(dSB, bc(kr[d]), dqB[d]);
      }
    }
  }
  float r[4][DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    r[0][d] = dqA[d].x * a.scale; r[1][d] = dqA[d].y * a.scale;
    r[2][d] = dqB[d].x * a.scale; r[3][d] = dqB[d].y * a.scale;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (qi[u] < a.Lq) str<DH>(a.dq + (int64_t)b * a.dq_bs + (int64_t)qi[u] * a.dq_ls + h * DH, r[u]);
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
  a.nw = (Lk + 31) / 32;
  a.scale = 1.0f / sqrtf((float)dh);
  a.scale_log2 = a.scale * 1.4426950408889634f;
  a.thr = drop_thr16(p_drop);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.rng_state = rng_state; a.call_id = call_id;
}

// threads per workgroup: the largest of {256, 128, 64} that still gives
// >= 1024 workgroups (fill 256 CUs x 4), else 64
int pick_nt(int64_t bh, int L) {
  for (int nt = 256; nt > 64; nt >>= 1)
    if (bh * ((L + 4 * nt - 1) / (4 * nt)) >= 1024) return nt;
  return 64;
}

#define VAESNE_NT_SWITCH(NTV, CALL) \
  switch (NTV) {                    \
    case 256: { constexpr int NTT = 256; CALL; break; } \
    case 128: { constexpr int NTT = 128; CALL; break; } \
    default: { constexpr int NTT = 64; CALL; break; }   \
  }

template <int DHV>
int launch_fwd(const AttnArgs& a, float p_drop, hipStream_t s) {
  const int nt = pick_nt((int64_t)a.B * a.H, a.Lq);
  VAESNE_NT_SWITCH(nt, {
    const int nqb = (a.Lq + 4 * NTT - 1) / (4 * NTT);
    dim3 grid((unsigned)((int64_t)a.B * a.H * nqb));
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_fwd_kernel<DHV, NTT, true>), grid, dim3(NTT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<DHV, NTT, false>), grid, dim3(NTT), 0, s, a);
  })
  VAESNE_CHECK_LAUNCH();
  return 0;
}

template <int DHV>
int launch_bwd(const AttnArgs& a, float p_drop, hipStream_t s) {
  const int ntk = pick_nt((int64_t)a.B * a.H, a.Lk);
  VAESNE_NT_SWITCH(ntk, {
    const int nkb = (a.Lk + 4 * NTT - 1) / (4 * NTT);
    dim3 g((unsigned)((int64_t)a.B * a.H * nkb));
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, true>), g, dim3(NTT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, false>), g, dim3(NTT), 0, s, a);
  })
  VAESNE_CHECK_LAUNCH();
  const int ntq = pick_nt((int64_t)a.B * a.H, a.Lq);
  VAESNE_NT_SWITCH(ntq, {
    const int nqb = (a.Lq + 4 * NTT - 1) / (4 * NTT);
    dim3 g((unsigned)((int64_t)a.B * a.H * nqb));
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, NTT, true>), g, dim3(NTT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, NTT, false>), g, dim3(NTT), 0, s, a);
  })
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

VAESNE_API int64_t vaesne_attn_keep_bits_size(int B, int H, int Lq, int Lk) {
  return (int64_t)B * H * ((Lk + 31) / 32) * Lq * (int64_t)sizeof(uint32_t);
}

VAESNE_API int vaesne_attn_fwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const float* kbias, int64_t kb_bs, float* o,
                               int64_t o_bs, int64_t o_ls, float* lse, int B, int H, int Lq,
                               int Lk, int dh, float p_drop, const int64_t* rng_state,
                               uint32_t call_id, uint32_t* keep_bits, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || (dh != 8 && dh != 16)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && (!keep_bits || !rng_state)) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls))
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.q_bs = q_bs; a.q_ls = q_ls;
  a.k = k; a.k_bs = k_bs; a.k_ls = k_ls;
  a.v = v; a.v_bs = v_bs; a.v_ls = v_ls;
  a.kbias = kbias; a.kb_bs = kb_bs;
  a.o = o; a.o_out = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = lse;
  a.bits = keep_bits;
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
                               float p_drop, const uint32_t* keep_bits, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || (dh != 8 && dh != 16)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && !keep_bits) return (int)hipErrorInvalidValue;
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
  a.bits = const_cast<uint32_t*>(keep_bits);
  fill_common(a, B, H, Lq, Lk, dh, p_drop, nullptr, 0);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return launch_bwd<8>(a, p_drop, s);
  return launch_bwd<16>(a, p_drop, s);
}
