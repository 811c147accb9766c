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
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "attn_common.h"

using namespace vaesne;

namespace {

constexpr int TK = 64;   // keys (or queries) per LDS tile

typedef float f2 __attribute__((ext_vector_type(2)));

using vaesne::ex2;
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

// broadcast-operand packed FMA: c + a * {r_d, r_d} with r_d one half of an LDS row held as
// register pairs.
//
// gfx950 erratum (measured: tools/probe/mfma_interference.py, DESIGN.md "A packed-FP32
// erratum"): a v_pk_{fma,mul,add}_f32 whose op_sel makes the LOW lane read the HIGH half
// of a source (op_sel:[0,1,0] and friends) returns wrong values while another wave on the
// CU runs v_mfma_f32_16x16x32_{f16,bf16} -- which the split-f16 attention kernels do,
// beside these kernels, on the other streams of the training step.  op_sel_hi (the HIGH
// lane reading the LOW half) is unaffected.  So the low half of a pair is broadcast by
// one v_pk_fma_f32 with op_sel_hi (fma2_lo), the high half by two scalar FMAs (fma2_hi);
// no kernel of this library contains the affected form (tests/test_isa_erratum.py).
__device__ __forceinline__ f2 fma2_lo(f2 a, f2 b, f2 c) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(c) : "v"(a), "v"(b));
  return c;
}
__device__ __forceinline__ f2 fma2_hi(f2 a, f2 b, f2 c) {
  return (f2){__builtin_fmaf(a.x, b.y, c.x), __builtin_fmaf(a.y, b.y, c.y)};
}
__device__ __forceinline__ f2 fma2_lo_u(f2 a, f2 b, f2 c) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ f2 fma2_hi_u(f2 a, f2 b, f2 c) { return fma2_hi(a, b, c); }
__device__ __forceinline__ f2 mul2_lo(f2 a, f2 b) {
  f2 r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 mul2_hi(f2 a, f2 b) { return (f2){a.x * b.y, a.y * b.y}; }
// the first FMA of a score chain: a * {b.x, b.x} + {c_H, c_H}, c = a pair of key biases
// (H = 0: its first key, read with op_sel_hi; 1: its second, two scalar FMAs)
template <int H>
__device__ __forceinline__ f2 fma2_bias(f2 a, f2 b, f2 c) {
  if (H == 0) {
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  }
  return (f2){__builtin_fmaf(a.x, b.x, c.y), __builtin_fmaf(a.y, b.x, c.y)};
}
template <int DH>
__device__ __forceinline__ f2 fma2r(f2 a, const f2 (&r)[DH / 2], int d, f2 c) {
  return (d & 1) ? fma2_hi(a, r[d >> 1], c) : fma2_lo(a, r[d >> 1], c);
}
template <int DH>
__device__ __forceinline__ f2 fma2ru(f2 a, const f2 (&r)[DH / 2], int d, f2 c) {
  return (d & 1) ? fma2_hi_u(a, r[d >> 1], c) : fma2_lo_u(a, r[d >> 1], c);
}
// Two dh-8 score chains (bias + q . k) of one or two query pairs, interleaved so each
// chain's next FMA is not right behind its last (hipcc pads what remains)
template <int HA, int HB>
__device__ __forceinline__ void qk_chains2(const f2 (&qa)[8], const f2 (&kra)[4], f2 kba,
                                           const f2 (&qb)[8], const f2 (&krb)[4], f2 kbb,
                                           f2& sa, f2& sb) {
  sa = fma2_bias<HA>(qa[0], kra[0], kba);
  sb = fma2_bias<HB>(qb[0], krb[0], kbb);
#pragma unroll
  for (int d = 1; d < 8; ++d) {
    sa = fma2r<8>(qa[d], kra, d, sa);
    sb = fma2r<8>(qb[d], krb, d, sb);
  }
}
// broadcast read of one LDS row as register pairs
template <int DH>
__device__ __forceinline__ void lrow2(const float* s, f2 (&r)[DH / 2]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 a = *reinterpret_cast<const float4*>(s + d);
    r[d / 2] = (f2){a.x, a.y};
    r[d / 2 + 1] = (f2){a.z, a.w};
  }
}

// The fused backward's two chains of one (query, key pair): s = kbias + k . q (scores,
// log2 domain) and g = v . dO
__device__ __forceinline__ void sg_chains(const f2 (&k)[8], const f2 (&v)[8], const f2 (&qr)[4],
                                          const f2 (&dr)[4], f2 kb, f2& s, f2& g) {
  s = fma2_lo_u(k[0], qr[0], kb);
  g = mul2_lo(v[0], dr[0]);
#pragma unroll
  for (int d = 1; d < 8; ++d) {
    s = fma2r<8>(k[d], qr, d, s);
    g = fma2r<8>(v[d], dr, d, g);
  }
}

// The fused backward's accumulator updates of one (query, key pair): dV += aP dO and
// dK += dS q over the 8 features
__device__ __forceinline__ void dvdk_update(f2 (&dv)[8], f2 (&dk)[8], f2 aP, f2 dS,
                                            const f2 (&dr)[4], const f2 (&qr)[4]) {
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    dv[d] = fma2r<8>(aP, dr, d, dv[d]);
    dk[d] = fma2r<8>(dS, qr, d, dk[d]);
  }
}

// The fused dQ's per-feature key sums of two queries over the lane's two key pairs (NP 2):
// F[d] = sx0 k0[d].x + sy0 k0[d].y + sx1 k1[d].x + sy1 k1[d].y
__device__ __forceinline__ void dq_sums(f2 sx0, f2 sy0, f2 sx1, f2 sy1, const f2 (&k0)[8],
                                        const f2 (&k1)[8], f2 (&F)[8]) {
#pragma unroll
  for (int d = 0; d < 8; ++d) F[d] = mul2_lo(sx0, k0[d]);
#pragma unroll
  for (int d = 0; d < 8; ++d) F[d] = fma2_hi(sy0, k0[d], F[d]);
#pragma unroll
  for (int d = 0; d < 8; ++d) F[d] = fma2_lo(sx1, k1[d], F[d]);
#pragma unroll
  for (int d = 0; d < 8; ++d) F[d] = fma2_hi(sy1, k1[d], F[d]);
}

// s[p][u] = kb[u] + q[p] . k[u] for the 8 keys of a group, x[p] = max(x[p], s[p][.]).
// dh 8: two chains per asm statement (qk_chains2): the two query pairs of one key (NP 2),
// or one query pair and two keys (NP 1).
template <int DH, int NP>
__device__ __forceinline__ void qk_group(const f2 (&q)[NP][DH], const float* ks, const float* kb,
                                         f2 (&s)[NP][8], f2 (&x)[NP]) {
  if constexpr (DH == 8 && NP == 2) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f2 kr[4];
      lrow2<8>(ks + u * 8, kr);
      const f2 kb2 = *reinterpret_cast<const f2*>(kb + (u & ~1));
      if (u & 1)
        qk_chains2<1, 1>(q[0], kr, kb2, q[1], kr, kb2, s[0][u], s[1][u]);
      else
        qk_chains2<0, 0>(q[0], kr, kb2, q[1], kr, kb2, s[0][u], s[1][u]);
      x[0] = __builtin_elementwise_max(x[0], s[0][u]);
      x[1] = __builtin_elementwise_max(x[1], s[1][u]);
    }
  } else if constexpr (DH == 8 && NP == 1) {
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      f2 k0[4], k1[4];
      lrow2<8>(ks + u * 8, k0);
      lrow2<8>(ks + (u + 1) * 8, k1);
      const f2 kb2 = *reinterpret_cast<const f2*>(kb + u);
      qk_chains2<0, 1>(q[0], k0, kb2, q[0], k1, kb2, s[0][u], s[0][u + 1]);
      x[0] = __builtin_elementwise_max(x[0], s[0][u]);
      x[0] = __builtin_elementwise_max(x[0], s[0][u + 1]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f2 kr[DH / 2];
      lrow2<DH>(ks + u * DH, kr);
      const f2 kb2 = *reinterpret_cast<const f2*>(kb + (u & ~1));
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        // acc = kb + q . k, the chain's first FMA reading the bias from its pair
        f2 acc = (u & 1) ? fma2_bias<1>(q[p][0], kr[0], kb2) : fma2_bias<0>(q[p][0], kr[0], kb2);
#pragma unroll
        for (int d = 1; d < DH; ++d) acc = fma2r<DH>(q[p][d], kr, d, acc);
        s[p][u] = acc;
        x[p] = __builtin_elementwise_max(x[p], acc);
      }
    }
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
// lane owns 2*NP queries: pair p = {i + (2p) NTT, i + (2p+1) NTT}
template <int DH, int NTT, int NP, bool DROP>
__global__ __launch_bounds__(NTT) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ __attribute__((aligned(16))) float Kb[TK];
  constexpr int R = 2 * NP;
  constexpr int QB = R * NTT;
  const int nqb = (a.Lq + QB - 1) / QB;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qb = wg % nqb;
  const int bh = wg / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  int qi[R], qc[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    qi[u] = qb * QB + u * NTT + threadIdx.x;
    qc[u] = min(qi[u], a.Lq - 1);
  }
  f2 q[NP][DH], o[NP][DH], m[NP], l[NP];
  {
    const float* qbase = a.q + (int64_t)b * a.q_bs + h * DH;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float t0[DH], t1[DH];
      ldr<DH>(qbase + (int64_t)qc[2 * p] * a.q_ls, t0);
      ldr<DH>(qbase + (int64_t)qc[2 * p + 1] * a.q_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        q[p][d] = (f2){t0[d], t1[d]} * a.scale_log2;
        o[p][d] = bc(0.f);
      }
      m[p] = bc(M_INIT);
      l[p] = bc(0.f);
    }
  }
  uint32_t rk[R];
  uint32_t skey = 0u;
  if (DROP) {
    skey = key_of(a.rng_state, a.call_id);
#pragma unroll
    for (int u = 0; u < R; ++u) rk[u] = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + qc[u]));
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;
  const int kbeg = blockIdx.y * a.kchunk, klim = min(a.Lk, kbeg + a.kchunk);
  // ASYNC (dh 8, 256 threads): the next key tile's K / V rows and key bias are loaded
  // into registers before this tile's compute and written to LDS after it
  // (issue-early / write-late): thread t < 128 holds K float4 (row t/2, half t%2),
  // t >= 128 the V float4 of row (t-128)/2, t < 64 the key bias of row t
  constexpr bool ASYNC = DH == 8 && NTT == 256;
  float4 rKV = make_float4(0.f, 0.f, 0.f, 0.f);
  float rB = -INFINITY;
  auto issue = [&](int kt) {
    const int t = threadIdx.x, half = t & 1, row = (t & 127) >> 1;
    const bool ok = kt + row < klim;
    const int64_t kc = min(kt + row, klim - 1);
    const float* src = t < 128 ? kg + kc * a.k_ls : vg + kc * a.v_ls;
    rKV = ok ? *reinterpret_cast<const float4*>(src + 4 * half) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < TK) rB = kt + t < klim ? (kbg ? kbg[kt + t] : 0.f) : -INFINITY;
  };
  if (ASYNC && kbeg < klim) issue(kbeg);

  for (int kt = kbeg; kt < klim; kt += TK) {
    __syncthreads();
    if (ASYNC) {
      const int t = threadIdx.x, half = t & 1, row = (t & 127) >> 1;
      *reinterpret_cast<float4*>((t < 128 ? Ks : Vs) + row * DH + 4 * half) = rKV;
      if (t < TK) Kb[t] = rB;
    } else {
      stage<DH, NTT>(Ks, kg, a.k_ls, kt, klim, 1.f);
      stage<DH, NTT>(Vs, vg, a.v_ls, kt, klim, 1.f);
      for (int i = threadIdx.x; i < TK; i += NTT)
        Kb[i] = kt + i < klim ? (kbg ? kbg[kt + i] : 0.f) : -INFINITY;
    }
    __syncthreads();
    if (ASYNC && kt + TK < klim) issue(kt + TK);   // next tile's loads fly under this compute
    const int kend = min(TK, klim - kt);
    uint32_t w[R];
#pragma unroll
    for (int u = 0; u < R; ++u) w[u] = 0u;
    for (int g0 = 0; g0 < kend; g0 += 8) {
      f2 s[NP][8];
      f2 x[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) x[p] = m[p];
      qk_group<DH, NP>(q, Ks + g0 * DH, Kb + g0, s, x);
      // Lazy rescaling: m is the exponent origin, moved (and o, l rescaled) only
      // when some row's running max x passes it by more than 8 (p <= 2^8, no
      // overflow) -- a wave-uniform branch taken on the first groups only.
      bool move = false;
#pragma unroll
      for (int p = 0; p < NP; ++p) move |= (x[p].x > m[p].x + 8.f) | (x[p].y > m[p].y + 8.f);
      if (__any(move)) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const f2 c = ex2(m[p] - x[p]);     // 0 from M_INIT
          m[p] = x[p];
          l[p] *= c;
#pragma unroll
          for (int d = 0; d < DH; ++d) o[p][d] *= c;
        }
      }
      f2 mu[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        mu[p] = m[p];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        f2 p0[NP], p1[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          p0[p] = ex2(s[p][u] - mu[p]);
          p1[p] = ex2(s[p][u + 1] - mu[p]);
          l[p] += p0[p] + p1[p];
        }
        if (DROP) {
          const uint32_t kpm = attn_keypair_mix(skey, (uint32_t)((kt + g0 + u) >> 1));
          bool klo[R], khi[R];
#pragma unroll
          for (int t = 0; t < R; ++t) {
            const uint32_t bits = attn_pair_bits_mixed(rk[t], kpm);
            klo[t] = (bits & 0xffffu) >= a.thr;
            khi[t] = (bits >> 16) >= a.thr;
          }
          // every row's compares first: the lane masks are read by the v_addc a few
          // instructions after they are written (no hazard wait states)
#pragma unroll
          for (int t = 0; t < R; ++t)
            w[t] = push_bit(push_bit(w[t], __builtin_amdgcn_ballot_w64(klo[t])),
                            __builtin_amdgcn_ballot_w64(khi[t]));
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            p0[p] = sel2(klo[2 * p], klo[2 * p + 1], p0[p]);
            p1[p] = sel2(khi[2 * p], khi[2 * p + 1], p1[p]);
          }
        }
        f2 v0[DH / 2], v1[DH / 2];
        lrow2<DH>(Vs + (g0 + u) * DH, v0);
        lrow2<DH>(Vs + (g0 + u + 1) * DH, v1);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            o[p][d] = fma2r<DH>(p0[p], v0, d, o[p][d]);
            o[p][d] = fma2r<DH>(p1[p], v1, d, o[p][d]);
          }
        }
      }
      if (DROP && (((g0 + 8) & 31) == 0 || g0 + 8 >= kend)) {
        const int word = (kt + g0) >> 5, n = (g0 & 31) + 8;
#pragma unroll
        for (int t = 0; t < R; ++t) {
          if (qi[t] < a.Lq) bitp[(int64_t)word * a.Lq + qi[t]] = keep_word(w[t], n);
          w[t] = 0u;
        }
      }
    }
  }
  if (a.ml) {   // split launch: un-normalised partial o and (m, l) of this key chunk
    float* ob = a.o_out + blockIdx.y * a.o_ss + (int64_t)b * a.o_bs + h * DH;
    float* mlp = a.ml + ((int64_t)blockIdx.y * a.B * a.H + bh) * a.Lq * 2;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float r0[DH], r1[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) { r0[d] = o[p][d].x; r1[d] = o[p][d].y; }
      const int i0 = qi[2 * p], i1 = qi[2 * p + 1];
      if (i0 < a.Lq) {
        str<DH>(ob + (int64_t)i0 * a.o_ls, r0);
        *reinterpret_cast<float2*>(mlp + 2 * i0) = make_float2(m[p].x, l[p].x);
      }
      if (i1 < a.Lq) {
        str<DH>(ob + (int64_t)i1 * a.o_ls, r1);
        *reinterpret_cast<float2*>(mlp + 2 * i1) = make_float2(m[p].y, l[p].y);
      }
    }
    return;
  }
  // l == 0 (every key masked) -> 0/0 = NaN, as the reference's -inf softmax
  const float ik = DROP ? a.inv_keep : 1.f;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const f2 inv = bc(ik) / l[p];
    float r0[DH], r1[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = o[p][d].x * inv.x; r1[d] = o[p][d].y * inv.y; }
    const int i0 = qi[2 * p], i1 = qi[2 * p + 1];
    if (i0 < a.Lq) {
      str<DH>(a.o_out + (int64_t)b * a.o_bs + (int64_t)i0 * a.o_ls + h * DH, r0);
      a.lse[(int64_t)bh * a.Lq + i0] = m[p].x + __log2f(l[p].x);
    }
    if (i1 < a.Lq) {
      str<DH>(a.o_out + (int64_t)b * a.o_bs + (int64_t)i1 * a.o_ls + h * DH, r1);
      a.lse[(int64_t)bh * a.Lq + i1] = m[p].y + __log2f(l[p].y);
    }
  }
}

// sum of v[0..15] over the 64 lanes of a wave; lane l returns the total of
// component l >> 2.  Transposing butterfly: each exchange level sends half of
// the live components to the partner lane group and keeps the other half, so
// the live set halves per level: permlane32 swaps (8), permlane16 swaps (4),
// DPP row_ror 8 (xor 8, 2) and half-row mirror (partner 7 - l, flips bit 2),
// then two quad-permute adds over lane bits 0, 1.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum16_spread(const float (&v)[16]) {
  float u[8], w[4], x[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) {   // lanes 0-31 keep component i, lanes 32-63 i + 8
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]),
                                                    __float_as_uint(v[i + 8]), false, false);
    u[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // lane bit 4 selects i / i + 4
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(u[i]),
                                                    __float_as_uint(u[i + 4]), false, false);
    w[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const bool b3 = (threadIdx.x >> 3) & 1, b2 = (threadIdx.x >> 2) & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)     // lane bit 3 selects i / i + 2 (partner l ^ 8 = row_ror 8)
    x[i] = (b3 ? w[i + 2] : w[i]) + dpp<0x128>(b3 ? w[i] : w[i + 2]);
  float y = (b2 ? x[1] : x[0]) + dpp<0x141>(b2 ? x[0] : x[1]);   // half-row mirror
  y += dpp<0x4e>(y);              // quad xor 2
  y += dpp<0xb1>(y);              // quad xor 1
  return y;
}

// ============================== dK, dV =====================================
// lane owns 2*NP adjacent keys key0 .. key0 + 2NP - 1 (pairs of adjacent keys);
// queries stream through LDS tiles.
// DQ (head_dim 8, the whole key axis in this workgroup): dQ is fused in.  Per
// pair of queries, each lane's dS-weighted key sums (both queries packed in one
// f2 per feature) are reduced over the wave (wave_sum16_spread) into LDS, and
// over the workgroup's waves per query tile: the dQ kernel's recomputation of
// S, P and dP is saved.
template <int DH, int NTT, int NP, bool DROP, bool DQ = false>
__global__ __launch_bounds__(NTT) void attn_bwd_kv_kernel(AttnArgs a) {
  constexpr int R = 2 * NP;
  constexpr int KB = R * NTT;
  constexpr int NWB = (KB + 31) / 32;       // bitmap words of this key block
  constexpr int NWV = NTT / 64;             // waves
  static_assert(!DQ || DH == 8, "fused dQ reduces 8 components");
  // ASYNC (dh 8, 256 threads: the decoders' launches): the next query tile's Q, dO, O,
  // lse and keep words are loaded into registers BEFORE this tile's compute and written
  // to LDS after it (issue-early / write-late), so their HBM latency hides under the
  // compute instead of stalling every wave at each tile's start
  constexpr bool ASYNC = DH == 8 && NTT == 256;
  constexpr int NWBP = NWB + (ASYNC ? 1 : 0);   // padded row: conflict-free column writes
  __shared__ __attribute__((aligned(16))) float Qs[TK * DH];
  __shared__ __attribute__((aligned(16))) float Ds_[TK * DH];   // dO tile
  __shared__ float Ls[TK], Dd[TK];
  __shared__ uint32_t Ws[TK * NWBP];
  __shared__ __attribute__((aligned(16))) float Qw[DQ ? NWV * TK * DH : 1];   // per-wave dQ
  // keep-bit lookup: 4 bits of the bitmap -> the two key pairs' 0/1 float masks
  // (one conflict-free ds_read_b128 instead of ~16 bit-extract / compare / select
  // VALU ops per query; the 16 entries fill the 64 banks exactly once)
  __shared__ float4 Mt[16];
  if (DROP && threadIdx.x < 16)
    Mt[threadIdx.x] = make_float4((float)(threadIdx.x & 1), (float)((threadIdx.x >> 1) & 1),
                                  (float)((threadIdx.x >> 2) & 1), (float)((threadIdx.x >> 3) & 1));
  const int nkb = (a.Lk + KB - 1) / KB;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int kb = wg % nkb;
  const int bh = wg / nkb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int key0 = kb * KB + R * threadIdx.x;
  f2 k[NP][DH], v[NP][DH], dk[NP][DH], dv[NP][DH], kbias[NP];
  {
    const float* kbase = a.k + (int64_t)b * a.k_bs + h * DH;
    const float* vbase = a.v + (int64_t)b * a.v_bs + h * DH;
    const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int j0 = key0 + 2 * p, j1 = j0 + 1;
      float t0[DH], t1[DH];
      ldr<DH>(kbase + (int64_t)min(j0, a.Lk - 1) * a.k_ls, t0);
      ldr<DH>(kbase + (int64_t)min(j1, a.Lk - 1) * a.k_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) k[p][d] = (f2){t0[d], t1[d]};   // the Q tile carries the scale
      ldr<DH>(vbase + (int64_t)min(j0, a.Lk - 1) * a.v_ls, t0);
      ldr<DH>(vbase + (int64_t)min(j1, a.Lk - 1) * a.v_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        v[p][d] = (f2){t0[d], t1[d]};
        dk[p][d] = bc(0.f);
        dv[p][d] = bc(0.f);
      }
      // key bias: -inf for masked or out-of-range keys -> p = 0
      kbias[p] = (f2){j0 < a.Lk ? (kbp ? kbp[j0] : 0.f) : -INFINITY,
                      j1 < a.Lk ? (kbp ? kbp[j1] : 0.f) : -INFINITY};
    }
  }
  const int wl = (R * threadIdx.x) >> 5;         // my bitmap word within the block
  const int sh = (R * threadIdx.x) & 31;         // my first bit within it
  const float* qg = a.q + (int64_t)b * a.q_bs + h * DH;
  const float* dg = a.dout + (int64_t)b * a.do_bs + h * DH;
  const float* og = a.o + (int64_t)b * a.o_bs + h * DH;
  const float* lg = a.lse + (int64_t)bh * a.Lq;
  const uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;
  const int wfirst = (kb * KB) >> 5;
  // dO is staged pre-multiplied by 1/(1-p): dV = sum keep*P*dO/(1-p) and
  // dP = keep * (V . dO)/(1-p) come out scaled; D = rowsum(dO*O) uses the raw dO.
  const int qbeg = blockIdx.y * a.qchunk, qlim = min(a.Lq, qbeg + a.qchunk);
  // ASYNC register stage: thread t < 128 holds dO and O float4 (row t/2, half t%2),
  // thread t >= 128 the Q float4 of row (t-128)/2; t < 64 the lse of row t; every
  // thread NWS keep words (word-major, 64 consecutive queries per word: coalesced)
  constexpr int NWS = ASYNC && DROP ? (TK * NWB) / NTT : 1;
  static_assert(!ASYNC || (TK * NWB) % NTT == 0, "keep words per thread");
  float4 rA = make_float4(0.f, 0.f, 0.f, 0.f), rO = rA;
  float rL = INFINITY;
  uint32_t rW[NWS];
  auto issue = [&](int qt) {     // loads of query tile qt (rows past qlim: zeros / +inf)
    const int t = threadIdx.x, half = t & 1;
    const int row = (t & 127) >> 1, qi = qt + row;
    const bool ok = qi < qlim;
    const int64_t qc = min(qi, qlim - 1);
    if (t < 128) {
      rA = ok ? *reinterpret_cast<const float4*>(dg + qc * a.do_ls + 4 * half) : make_float4(0.f, 0.f, 0.f, 0.f);
      rO = ok ? *reinterpret_cast<const float4*>(og + qc * a.o_ls + 4 * half) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      rA = ok ? *reinterpret_cast<const float4*>(qg + qc * a.q_ls + 4 * half) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (t < TK) rL = qt + t < qlim ? lg[qt + t] : INFINITY;
    if (DROP) {
#pragma unroll
      for (int j = 0; j < NWS; ++j) {
        const int idx = j * NTT + t, i = idx % TK, wv = idx / TK;
        const int word = wfirst + wv;
        rW[j] = (qt + i < qlim && word < a.nw) ? bitp[(int64_t)word * a.Lq + qt + i] : 0u;
      }
    }
  };
  auto commit = [&]() {          // the staged registers -> LDS (after a barrier)
    const int t = threadIdx.x, half = t & 1, row = (t & 127) >> 1;
    if (t < 128) {
      // D = rowsum(dO * O) in the sequential order of the fmaf chain over d = 0..7:
      // the half-1 lane continues the half-0 lane's partial sum
      float pd = fmaf(rA.x, rO.x, 0.f);
      pd = fmaf(rA.y, rO.y, pd);
      pd = fmaf(rA.z, rO.z, pd);
      pd = fmaf(rA.w, rO.w, pd);
      const float p0 = __shfl_xor(pd, 1);
      if (half) {
        float Di = fmaf(rA.x, rO.x, p0);
        Di = fmaf(rA.y, rO.y, Di);
        Di = fmaf(rA.z, rO.z, Di);
        Di = fmaf(rA.w, rO.w, Di);
        Dd[row] = Di;
      }
      const float m = a.inv_keep;
      *reinterpret_cast<float4*>(Ds_ + row * DH + 4 * half) =
          make_float4(rA.x * m, rA.y * m, rA.z * m, rA.w * m);
    } else {
      const float m = a.scale_log2;
      *reinterpret_cast<float4*>(Qs + row * DH + 4 * half) =
          make_float4(rA.x * m, rA.y * m, rA.z * m, rA.w * m);
    }
    if (t < TK) Ls[t] = rL;      // +inf for padding rows -> p = 0
    if (DROP) {
#pragma unroll
      for (int j = 0; j < NWS; ++j) {
        const int idx = j * NTT + t, i = idx % TK, wv = idx / TK;
        Ws[i * NWBP + wv] = rW[j];
      }
    }
  };
  if (ASYNC && qbeg < qlim) issue(qbeg);
  for (int qt = qbeg; qt < qlim; qt += TK) {
    __syncthreads();
    if (ASYNC) {
      commit();
    } else {
      stage<DH, NTT>(Qs, qg, a.q_ls, qt, qlim, a.scale_log2);
      stage<DH, NTT>(Ds_, dg, a.do_ls, qt, qlim, a.inv_keep);
      for (int i = threadIdx.x; i < TK; i += NTT) {
        const int qi = qt + i;
        float Di = 0.f, li = INFINITY;
        if (qi < qlim) {
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
          Ws[i * NWBP + wv] = (qi < qlim && word < a.nw) ? bitp[(int64_t)word * a.Lq + qi] : 0u;
        }
      }
    }
    __syncthreads();
    if (ASYNC && qt + TK < qlim) issue(qt + TK);   // next tile's loads fly under this compute
    const int qend = min(TK, qlim - qt);
    // two queries per trip (a padding row past qend has Ls = +inf -> p = 0 and
    // contributes nothing): explicit, as the wave reduction's cross-lane ops
    // keep the compiler from unrolling a runtime-count loop
    for (int i0 = 0; i0 < qend; i0 += 2) {
      f2 dSq[2][NP];
#pragma unroll
      for (int i = i0; i < i0 + 2; ++i) {
        f2 qr[DH / 2], dr[DH / 2];
        lrow2<DH>(Qs + i * DH, qr);
        lrow2<DH>(Ds_ + i * DH, dr);
        const f2 li = bc(Ls[i]), Di = bc(Dd[i]);
        f2 km[2];
        if (DROP) {
          const float4 t = Mt[(Ws[i * NWBP + wl] >> sh) & 15u];
          km[0] = (f2){t.x, t.y};
          km[1] = (f2){t.z, t.w};
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          f2 s, g;
          if constexpr (DH == 8) {
            sg_chains(k[p], v[p], qr, dr, kbias[p], s, g);
          } else {
            s = kbias[p];
            g = mul2_lo(v[p][0], dr[0]);
#pragma unroll
            for (int d = 0; d < DH; ++d) {
              s = fma2ru<DH>(k[p][d], qr, d, s);
              if (d > 0) g = fma2ru<DH>(v[p][d], dr, d, g);
            }
          }
          const f2 pr = ex2(s - li);
          f2 aP = pr, dS;
          if (DROP) {
            // dS = pr * (keep * g - Di) = aP * g - pr * Di: 3 packed ops, not 4
            aP = pr * km[p];
            dS = fma2(aP, g, -(pr * Di));
          } else {
            dS = pr * (g - Di);
          }
          dSq[i - i0][p] = dS;
          if constexpr (DH == 8) {
            dvdk_update(dv[p], dk[p], aP, dS, dr, qr);
          } else {
#pragma unroll
            for (int d = 0; d < DH; ++d) {
              dv[p][d] = fma2ru<DH>(aP, dr, d, dv[p][d]);
              dk[p][d] = fma2ru<DH>(dS, qr, d, dk[p][d]);
            }
          }
        }
      }
      if (DQ) {   // F[d] = {dQ_d of query i0, of query i0 + 1} over this lane's keys
        f2 F[DH];
        if constexpr (NP == 2 && DH == 8) {
          dq_sums((f2){dSq[0][0].x, dSq[1][0].x}, (f2){dSq[0][0].y, dSq[1][0].y},
                  (f2){dSq[0][1].x, dSq[1][1].x}, (f2){dSq[0][1].y, dSq[1][1].y}, k[0], k[1], F);
        } else {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const f2 sx = {dSq[0][p].x, dSq[1][p].x}, sy = {dSq[0][p].y, dSq[1][p].y};
#pragma unroll
            for (int d = 0; d < DH; ++d) {
              F[d] = p == 0 ? mul2_lo(sx, k[p][d]) : fma2_lo_u(sx, k[p][d], F[d]);
              F[d] = fma2_hi_u(sy, k[p][d], F[d]);
            }
          }
        }
        // component order: level-32 pairs (feature 2j, 2j + 1) of one query, so
        // each permlane swap reads two separate register pairs (no copies);
        // lane l ends with query (l >> 4) & 1, feature 2 b2 + 4 b3 + b5
        float c[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          c[j] = F[2 * j].x; c[j + 8] = F[2 * j + 1].x;
          c[j + 4] = F[2 * j].y; c[j + 12] = F[2 * j + 1].y;
        }
        const int l = threadIdx.x & 63;
        // the 4 lanes of a group hold the same total: all store it (no branch)
        Qw[((threadIdx.x >> 6) * TK + i0 + ((l >> 4) & 1)) * DH +
           (2 * ((l >> 2) & 1) + 4 * ((l >> 3) & 1) + ((l >> 5) & 1))] = wave_sum16_spread(c);
      }
    }
    if (DQ) {   // dQ rows of this tile: sum over the waves (the whole key axis)
      __syncthreads();
      // key block kb's share (nkb > 1: a partial slot, summed after the launch)
      float* dqb = a.dq + kb * a.dq_ss + (int64_t)b * a.dq_bs + h * DH;
      for (int idx = threadIdx.x; idx < qend * (DH / 4); idx += NTT) {
        const int i = idx / (DH / 4), c = (idx - i * (DH / 4)) * 4;
        float4 acc = *reinterpret_cast<const float4*>(Qw + i * DH + c);
#pragma unroll
        for (int wv = 1; wv < NWV; ++wv) {
          const float4 t = *reinterpret_cast<const float4*>(Qw + (wv * TK + i) * DH + c);
          acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
        }
        acc.x *= a.scale; acc.y *= a.scale; acc.z *= a.scale; acc.w *= a.scale;
        *reinterpret_cast<float4*>(dqb + (int64_t)(qt + i) * a.dq_ls + c) = acc;
      }
    }
  }
  // dK = sum_i dS_i q_i * scale = (scale / scale_log2) * sum_i dS_i Qs_i
  const float kf = a.scale / a.scale_log2;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int j0 = key0 + 2 * p, j1 = j0 + 1;
    float r0[DH], r1[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = dk[p][d].x * kf; r1[d] = dk[p][d].y * kf; }
    float* dkb = a.dk + blockIdx.y * a.dk_ss + (int64_t)b * a.dk_bs + h * DH;
    float* dvb = a.dv + blockIdx.y * a.dk_ss + (int64_t)b * a.dv_bs + h * DH;
    if (j0 < a.Lk) str<DH>(dkb + (int64_t)j0 * a.dk_ls, r0);
    if (j1 < a.Lk) str<DH>(dkb + (int64_t)j1 * a.dk_ls, r1);
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = dv[p][d].x; r1[d] = dv[p][d].y; }
    if (j0 < a.Lk) str<DH>(dvb + (int64_t)j0 * a.dv_ls, r0);
    if (j1 < a.Lk) str<DH>(dvb + (int64_t)j1 * a.dv_ls, r1);
  }
}

// ================================ dQ =======================================
template <int DH, int NTT, int NP, bool DROP>
__global__ __launch_bounds__(NTT) void attn_bwd_q_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ __attribute__((aligned(16))) float Kb[TK];
  constexpr int R = 2 * NP;
  constexpr int QB = R * NTT;
  const int nqb = (a.Lq + QB - 1) / QB;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qb = wg % nqb;
  const int bh = wg / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  int qi[R], qc[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    qi[u] = qb * QB + u * NTT + threadIdx.x;
    qc[u] = min(qi[u], a.Lq - 1);
  }
  f2 q[NP][DH], g[NP][DH], dq[NP][DH], D[NP], lse[NP];
  {
    const float* qbase = a.q + (int64_t)b * a.q_bs + h * DH;
    const float* dbase = a.dout + (int64_t)b * a.do_bs + h * DH;
    const float* obase = a.o + (int64_t)b * a.o_bs + h * DH;
    const float* lp = a.lse + (int64_t)bh * a.Lq;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float t0[DH], t1[DH], o0[DH], o1[DH];
      ldr<DH>(qbase + (int64_t)qc[2 * p] * a.q_ls, t0);
      ldr<DH>(qbase + (int64_t)qc[2 * p + 1] * a.q_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        q[p][d] = (f2){t0[d], t1[d]} * a.scale_log2;
        dq[p][d] = bc(0.f);
      }
      ldr<DH>(dbase + (int64_t)qc[2 * p] * a.do_ls, t0);
      ldr<DH>(dbase + (int64_t)qc[2 * p + 1] * a.do_ls, t1);
      ldr<DH>(obase + (int64_t)qc[2 * p] * a.o_ls, o0);
      ldr<DH>(obase + (int64_t)qc[2 * p + 1] * a.o_ls, o1);
      f2 Dp = bc(0.f);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        g[p][d] = (f2){t0[d], t1[d]};
        Dp = fma2(g[p][d], (f2){o0[d], o1[d]}, Dp);
      }
      D[p] = Dp;
      lse[p] = (f2){lp[qc[2 * p]], lp[qc[2 * p + 1]]};
    }
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  const uint32_t* bitp = DROP ? a.bits + (int64_t)bh * a.nw * a.Lq : nullptr;
  // V staged pre-multiplied by 1/(1-p): t = dO . V/(1-p) is the kept-score dP
  const int kbeg = blockIdx.y * a.kchunk, klim = min(a.Lk, kbeg + a.kchunk);
  for (int kt = kbeg; kt < klim; kt += TK) {
    __syncthreads();
    stage<DH, NTT>(Ks, kg, a.k_ls, kt, klim, 1.f);
    stage<DH, NTT>(Vs, vg, a.v_ls, kt, klim, DROP ? a.inv_keep : 1.f);
    for (int i = threadIdx.x; i < TK; i += NTT)
      Kb[i] = kt + i < klim ? (kbg ? kbg[kt + i] : 0.f) : -INFINITY;
    __syncthreads();
    const int kend = min(TK, klim - kt);
    uint32_t w[R];
#pragma unroll
    for (int u = 0; u < R; ++u) w[u] = 0xffffffffu;
    for (int j = 0; j < kend; ++j) {
      if (DROP && (j & 31) == 0) {
        const int word = (kt + j) >> 5;
#pragma unroll
        for (int u = 0; u < R; ++u) w[u] = bitp[(int64_t)word * a.Lq + qc[u]];
      }
      f2 kr[DH / 2], vr[DH / 2];
      lrow2<DH>(Ks + j * DH, kr);
      lrow2<DH>(Vs + j * DH, vr);
      const float kb = Kb[j];
      const int s = j & 31;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        f2 sc = bc(kb), t = bc(0.f);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          sc = fma2r<DH>(q[p][d], kr, d, sc);
          t = fma2r<DH>(g[p][d], vr, d, t);
        }
        const f2 pr = ex2(sc - lse[p]);
        f2 dP = t;
        if (DROP) dP = sel2((w[2 * p] >> s) & 1u, (w[2 * p + 1] >> s) & 1u, dP);
        const f2 dS = pr * (dP - D[p]);
#pragma unroll
        for (int d = 0; d < DH; ++d) dq[p][d] = fma2r<DH>(dS, kr, d, dq[p][d]);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    float r0[DH], r1[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = dq[p][d].x * a.scale; r1[d] = dq[p][d].y * a.scale; }
    const int i0 = qi[2 * p], i1 = qi[2 * p + 1];
    float* dqb = a.dq + blockIdx.y * a.dq_ss + (int64_t)b * a.dq_bs + h * DH;
    if (i0 < a.Lq) str<DH>(dqb + (int64_t)i0 * a.dq_ls, r0);
    if (i1 < a.Lq) str<DH>(dqb + (int64_t)i1 * a.dq_ls, r1);
  }
}

// ================ repeated sequences: the decoders' first block =================
// The decoders run over N = R * Bd sequences, copy r of distinct sequence b being
// sequence n = r * Bd + b (the K samples x both modalities' latents,
// SpectraVAE.py:189-192, PhotometricVAE.py:196-199).  The first block's
// self-attention reads x = embedding(wavelength | time), the SAME for all R copies
// (SpectraLayers.py:54-62, PhotometricLayers.py:59-67): scores, row maxima and
// softmax denominators are shared, only the dropout masks differ.  These kernels
// compute the shared part once per distinct sequence and loop over the copies for
// the rest:
//   forward : per copy, the keep decisions and P.V (RC copies per workgroup, the
//             scores and exponentials computed once for them);
//   backward: per copy, dP = dO.V, the keep mask and the dV terms; the copies' dS
//             are summed before dK = dS^T Q and dQ = dS K (Q, K, V are shared, so
//             their gradients are the sums over the copies anyway).
// Each copy's keep decisions are exactly those attn_fwd_kernel draws for sequence n
// and the bitmap has its layout ([n*H + h][word][query]), so the plain kernels on
// the expanded input reproduce these bit for bit (tested).
// Args: q/k/v/kbias/lse over the Bd distinct sequences (a.B = Bd), o / dout / bits
// over the N sequences (o_bs, do_bs = per-sequence strides).
// grid.x covers query blocks [qb0, qb0 + nqbs) of every (sequence, head): a launch may do
// a part of the rows (vaesne_attn_rep_fwd_part)
template <int DH, int NTT, int NP, int RC, bool DROP>
__global__ __launch_bounds__(NTT) void attn_rep_fwd_kernel(AttnArgs a, int R, int qb0, int nqbs) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ __attribute__((aligned(16))) float Kb[TK];
  constexpr int R2 = 2 * NP;              // queries per lane (pairs p = {2p, 2p + 1})
  constexpr int QB = R2 * NTT;
  constexpr int NC = DROP ? RC : 1;       // accumulator sets (no dropout: one for all copies)
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qb = qb0 + wg % nqbs;
  const int bh = wg / nqbs;               // distinct sequence x head
  const int b = bh / a.H, h = bh - b * a.H;
  const int c0 = blockIdx.y * RC;
  int qi[R2], qc[R2];
#pragma unroll
  for (int u = 0; u < R2; ++u) {
    qi[u] = qb * QB + u * NTT + threadIdx.x;
    qc[u] = min(qi[u], a.Lq - 1);
  }
  f2 q[NP][DH], o[NC][NP][DH], m[NP], l[NP];
  {
    const float* qbase = a.q + (int64_t)b * a.q_bs + h * DH;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float t0[DH], t1[DH];
      ldr<DH>(qbase + (int64_t)qc[2 * p] * a.q_ls, t0);
      ldr<DH>(qbase + (int64_t)qc[2 * p + 1] * a.q_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) q[p][d] = (f2){t0[d], t1[d]} * a.scale_log2;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int d = 0; d < DH; ++d) o[c][p][d] = bc(0.f);
      m[p] = bc(M_INIT);
      l[p] = bc(0.f);
    }
  }
  // copies past R (R % RC != 0) are computed with copy R - 1's keys and not stored
  uint32_t rk[NC][R2];
  uint32_t* bitp[NC];
  uint32_t skey = 0u;
  if (DROP) {
    skey = key_of(a.rng_state, a.call_id);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int64_t nh = (int64_t)(min(c0 + c, R - 1) * a.B + b) * a.H + h;
      bitp[c] = a.bits + nh * a.nw * a.Lq;
#pragma unroll
      for (int u = 0; u < R2; ++u) rk[c][u] = attn_row_key(skey, (uint32_t)(nh * a.Lq + qc[u]));
    }
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  for (int kt = 0; kt < a.Lk; kt += TK) {
    __syncthreads();
    stage<DH, NTT>(Ks, kg, a.k_ls, kt, a.Lk, 1.f);
    stage<DH, NTT>(Vs, vg, a.v_ls, kt, a.Lk, 1.f);
    for (int i = threadIdx.x; i < TK; i += NTT)
      Kb[i] = kt + i < a.Lk ? (kbg ? kbg[kt + i] : 0.f) : -INFINITY;
    __syncthreads();
    const int kend = min(TK, a.Lk - kt);
    uint32_t w[NC][R2];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int u = 0; u < R2; ++u) w[c][u] = 0u;
    for (int g0 = 0; g0 < kend; g0 += 8) {
      f2 s[NP][8];
      f2 x[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) x[p] = m[p];
      qk_group<DH, NP>(q, Ks + g0 * DH, Kb + g0, s, x);
      // lazy rescaling, as attn_fwd_kernel (wave-uniform, first groups only)
      bool move = false;
#pragma unroll
      for (int p = 0; p < NP; ++p) move |= (x[p].x > m[p].x + 8.f) | (x[p].y > m[p].y + 8.f);
      if (__any(move)) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const f2 cf = ex2(m[p] - x[p]);    // 0 from M_INIT
          m[p] = x[p];
          l[p] *= cf;
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int d = 0; d < DH; ++d) o[c][p][d] *= cf;
        }
      }
      f2 mu[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        mu[p] = m[p];
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        f2 p0[NP], p1[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          p0[p] = ex2(s[p][u] - mu[p]);
          p1[p] = ex2(s[p][u + 1] - mu[p]);
          l[p] += p0[p] + p1[p];
        }
        f2 v0[DH / 2], v1[DH / 2];
        lrow2<DH>(Vs + (g0 + u) * DH, v0);
        lrow2<DH>(Vs + (g0 + u + 1) * DH, v1);
        if (DROP) {
          const uint32_t kpm = attn_keypair_mix(skey, (uint32_t)((kt + g0 + u) >> 1));
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            bool klo[R2], khi[R2];
#pragma unroll
            for (int t = 0; t < R2; ++t) {
              const uint32_t bits = attn_pair_bits_mixed(rk[c][t], kpm);
              klo[t] = (bits & 0xffffu) >= a.thr;
              khi[t] = (bits >> 16) >= a.thr;
            }
#pragma unroll
            for (int t = 0; t < R2; ++t)
              w[c][t] = push_bit(push_bit(w[c][t], __builtin_amdgcn_ballot_w64(klo[t])),
                                 __builtin_amdgcn_ballot_w64(khi[t]));
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              const f2 a0 = sel2(klo[2 * p], klo[2 * p + 1], p0[p]);
              const f2 a1 = sel2(khi[2 * p], khi[2 * p + 1], p1[p]);
#pragma unroll
              for (int d = 0; d < DH; ++d) {
                o[c][p][d] = fma2r<DH>(a0, v0, d, o[c][p][d]);
                o[c][p][d] = fma2r<DH>(a1, v1, d, o[c][p][d]);
              }
            }
          }
        } else {
#pragma unroll
          for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int d = 0; d < DH; ++d) {
              o[0][p][d] = fma2r<DH>(p0[p], v0, d, o[0][p][d]);
              o[0][p][d] = fma2r<DH>(p1[p], v1, d, o[0][p][d]);
            }
        }
      }
      if (DROP && (((g0 + 8) & 31) == 0 || g0 + 8 >= kend)) {
        const int word = (kt + g0) >> 5, n = (g0 & 31) + 8;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c0 + c < R) {
#pragma unroll
            for (int t = 0; t < R2; ++t)
              if (qi[t] < a.Lq) bitp[c][(int64_t)word * a.Lq + qi[t]] = keep_word(w[c][t], n);
          }
#pragma unroll
          for (int t = 0; t < R2; ++t) w[c][t] = 0u;
        }
      }
    }
  }
  // l == 0 (every key masked) -> NaN, as the reference
  f2 inv[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) inv[p] = bc(DROP ? a.inv_keep : 1.f) / l[p];
  auto put = [&](const f2 (&oc)[NP][DH], int r) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float r0[DH], r1[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) { r0[d] = oc[p][d].x * inv[p].x; r1[d] = oc[p][d].y * inv[p].y; }
      float* ob = a.o_out + (int64_t)(r * a.B + b) * a.o_bs + h * DH;
      if (qi[2 * p] < a.Lq) str<DH>(ob + (int64_t)qi[2 * p] * a.o_ls, r0);
      if (qi[2 * p + 1] < a.Lq) str<DH>(ob + (int64_t)qi[2 * p + 1] * a.o_ls, r1);
    }
  };
  if (DROP) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c0 + c < R) put(o[c], c0 + c);
  } else {
    for (int r = 0; r < R; ++r) put(o[0], r);   // every copy the same
  }
  if (blockIdx.y == 0) {   // shared over the copies
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (qi[2 * p] < a.Lq) a.lse[(int64_t)bh * a.Lq + qi[2 * p]] = m[p].x + __log2f(l[p].x);
      if (qi[2 * p + 1] < a.Lq) a.lse[(int64_t)bh * a.Lq + qi[2 * p + 1]] = m[p].y + __log2f(l[p].y);
    }
  }
}

// Backward with dropout (head_dim 8, dQ fused as in attn_bwd_kv_kernel).  Lane owns
// 2*NP adjacent keys of a distinct sequence; query tiles of TQR queries stream
// through LDS with, per copy, its dO rows (pre-multiplied by 1/(1-p)) and keep
// words.  Per score the copies enter only through G = sum_c keep_c dO_c: dV += P G,
// dS = P (G . V - sum_c D_c).  grid.x = Bd*H*key blocks, grid.y = query chunks x copy batches (RC
// copies each); several of either write partial dK / dV (slot y) and dQ (slot
// kb * copy batches + batch) into the workspace, summed in fixed order afterwards.
constexpr int TQR = 16;
#ifndef VAESNE_REP_WPE
#define VAESNE_REP_WPE 3      // waves per SIMD the register budget is sized for (NP = 1)
#endif
template <int NTT, int NP, int RC>
__global__ __launch_bounds__(NTT) __attribute__((amdgpu_waves_per_eu(NP == 1 ? VAESNE_REP_WPE : 1)))
void attn_rep_bwd_kernel(AttnArgs a, int R, int QS) {
  constexpr int DH = 8;
  constexpr int R2 = 2 * NP;
  constexpr int KB = R2 * NTT;
  constexpr int NWB = (KB + 31) / 32;
  constexpr int NWV = NTT / 64;
  constexpr int WST = TQR + 1;                       // keep-word row stride (banks)
  __shared__ __attribute__((aligned(16))) float Qs[TQR * DH];
  __shared__ __attribute__((aligned(16))) float Dos[RC * TQR * DH];
  __shared__ float Ls[TQR], Dsum[TQR], Dc[RC * TQR];
  __shared__ uint32_t Ws[RC * NWB * WST];
  // keep-mask table: 2-bit keep pattern of a key pair -> {keep0, keep1} as 0/1 floats (one
  // bit extract and one LDS read per copy and key pair instead of 2 extracts and 2 ANDs)
  __shared__ __attribute__((aligned(8))) f2 Mk[4];
  __shared__ __attribute__((aligned(16))) float Qw[NWV * TQR * DH];
  if (threadIdx.x < 4) Mk[threadIdx.x] = (f2){(float)(threadIdx.x & 1), (float)(threadIdx.x >> 1)};
  const int nkb = (a.Lk + KB - 1) / KB;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int kb = wg % nkb;
  const int bh = wg / nkb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int qs = blockIdx.y % QS, cb = blockIdx.y / QS, ncb = gridDim.y / QS;
  const int c0 = cb * RC;
  const int key0 = kb * KB + R2 * threadIdx.x;
  f2 k[NP][DH], v[NP][DH], dk[NP][DH], dv[NP][DH], kbias[NP];
  {
    const float* kbase = a.k + (int64_t)b * a.k_bs + h * DH;
    const float* vbase = a.v + (int64_t)b * a.v_bs + h * DH;
    const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int j0 = key0 + 2 * p, j1 = j0 + 1;
      float t0[DH], t1[DH];
      ldr<DH>(kbase + (int64_t)min(j0, a.Lk - 1) * a.k_ls, t0);
      ldr<DH>(kbase + (int64_t)min(j1, a.Lk - 1) * a.k_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) k[p][d] = (f2){t0[d], t1[d]};
      ldr<DH>(vbase + (int64_t)min(j0, a.Lk - 1) * a.v_ls, t0);
      ldr<DH>(vbase + (int64_t)min(j1, a.Lk - 1) * a.v_ls, t1);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        v[p][d] = (f2){t0[d], t1[d]};
        dk[p][d] = bc(0.f);
        dv[p][d] = bc(0.f);
      }
      kbias[p] = (f2){j0 < a.Lk ? (kbp ? kbp[j0] : 0.f) : -INFINITY,
                      j1 < a.Lk ? (kbp ? kbp[j1] : 0.f) : -INFINITY};
    }
  }
  const int wl = (R2 * threadIdx.x) >> 5;
  const int sh = (R2 * threadIdx.x) & 31;
  const float* qg = a.q + (int64_t)b * a.q_bs + h * DH;
  const float* lg = a.lse + (int64_t)bh * a.Lq;
  const int wfirst = (kb * KB) >> 5;
  const int qbeg = qs * a.qchunk, qlim = min(a.Lq, qbeg + a.qchunk);
  for (int qt = qbeg; qt < qlim; qt += TQR) {
    __syncthreads();
    for (int idx = threadIdx.x; idx < TQR * (DH / 4); idx += NTT) {
      const int i = idx / (DH / 4), cc = (idx - i * (DH / 4)) * 4;
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if (qt + i < qlim) {
        val = *reinterpret_cast<const float4*>(qg + (int64_t)(qt + i) * a.q_ls + cc);
        val.x *= a.scale_log2; val.y *= a.scale_log2; val.z *= a.scale_log2; val.w *= a.scale_log2;
      }
      *reinterpret_cast<float4*>(Qs + i * DH + cc) = val;
    }
    // per copy and query: the dO row (x 1/(1-p)) and D_c = dO_c . O_c (raw dO)
    for (int idx = threadIdx.x; idx < RC * TQR; idx += NTT) {
      const int c = idx / TQR, i = idx - c * TQR;
      const int qi = qt + i;
      float x[DH], y[DH];
      float Di = 0.f;
      if (qi < qlim && c0 + c < R) {
        const int64_t n = (int64_t)(c0 + c) * a.B + b;
        ldr<DH>(a.dout + n * a.do_bs + (int64_t)qi * a.do_ls + h * DH, x);
        ldr<DH>(a.o + n * a.o_bs + (int64_t)qi * a.o_ls + h * DH, y);
#pragma unroll
        for (int d = 0; d < DH; ++d) Di = fmaf(x[d], y[d], Di);
      } else {
#pragma unroll
        for (int d = 0; d < DH; ++d) x[d] = 0.f;
      }
#pragma unroll
      for (int d = 0; d < DH; ++d) x[d] *= a.inv_keep;
      str<DH>(Dos + (c * TQR + i) * DH, x);
      Dc[c * TQR + i] = Di;
    }
    for (int idx = threadIdx.x; idx < RC * NWB * TQR; idx += NTT) {
      const int c = idx / (NWB * TQR), r = idx - c * (NWB * TQR);
      const int wv = r / TQR, i = r - wv * TQR;
      const int qi = qt + i, word = wfirst + wv;
      uint32_t wd = 0u;
      if (qi < qlim && word < a.nw && c0 + c < R) {
        const int64_t nh = (int64_t)((c0 + c) * a.B + b) * a.H + h;
        wd = a.bits[(nh * a.nw + word) * a.Lq + qi];
      }
      Ws[(c * NWB + wv) * WST + i] = wd;
    }
    for (int i = threadIdx.x; i < TQR; i += NTT)
      Ls[i] = qt + i < qlim ? lg[qt + i] : INFINITY;   // +inf for padding rows -> p = 0
    __syncthreads();
    for (int i = threadIdx.x; i < TQR; i += NTT) {
      float sD = 0.f;
      for (int c = 0; c < RC; ++c) sD += Dc[c * TQR + i];
      Dsum[i] = sD;
    }
    __syncthreads();
    const int qend = min(TQR, qlim - qt);
    for (int i0 = 0; i0 < qend; i0 += 2) {
      f2 dSq[2][NP];
#pragma unroll
      for (int i = i0; i < i0 + 2; ++i) {
        f2 qr[DH / 2];
        lrow2<DH>(Qs + i * DH, qr);
        const f2 li = bc(Ls[i]), nD = bc(-Dsum[i]);
        f2 pr[NP], acc[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          f2 s = kbias[p];
#pragma unroll
          for (int d = 0; d < DH; ++d) s = fma2ru<DH>(k[p][d], qr, d, s);
          pr[p] = ex2(s - li);
        }
        // every copy's keep word of this query first (one LDS wait, not one per copy)
        uint32_t wk[RC];
#pragma unroll
        for (int c = 0; c < RC; ++c) wk[c] = Ws[(c * NWB + wl) * WST + i];
        // G = sum over the copies of keep_c * dO_c (dO pre-scaled by 1/(1-p)), per key:
        // dV += P G and sum_c keep_c dP_c = G . V, so each copy costs its masked dO sum
        // only (8 packed FMAs per key pair) instead of its own dP and dV terms
        f2 G[NP][DH];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int d = 0; d < DH; ++d) G[p][d] = bc(0.f);
#pragma unroll
        for (int c = 0; c < RC; ++c) {
          f2 dr[DH / 2];
          lrow2<DH>(Dos + (c * TQR + i) * DH, dr);
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const f2 mk = Mk[__builtin_amdgcn_ubfe(wk[c], sh + 2 * p, 2)];   // {keep0, keep1}
#pragma unroll
            for (int d = 0; d < DH; ++d) G[p][d] = fma2ru<DH>(mk, dr, d, G[p][d]);
          }
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          // dS = P (sum_c keep_c dP_c - sum_c D_c); G . V as two half chains
          f2 g0 = G[p][0] * v[p][0], g1 = G[p][1] * v[p][1];
#pragma unroll
          for (int d = 2; d < DH; d += 2) {
            g0 = fma2(G[p][d], v[p][d], g0);
            g1 = fma2(G[p][d + 1], v[p][d + 1], g1);
          }
          acc[p] = pr[p] * ((g0 + g1) + nD);
#pragma unroll
          for (int d = 0; d < DH; ++d) dv[p][d] = fma2(pr[p], G[p][d], dv[p][d]);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          dSq[i - i0][p] = acc[p];
#pragma unroll
          for (int d = 0; d < DH; ++d) dk[p][d] = fma2ru<DH>(acc[p], qr, d, dk[p][d]);
        }
      }
      f2 F[DH];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f2 sx = {dSq[0][p].x, dSq[1][p].x}, sy = {dSq[0][p].y, dSq[1][p].y};
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          F[d] = p == 0 ? mul2_lo(sx, k[p][d]) : fma2_lo_u(sx, k[p][d], F[d]);
          F[d] = fma2_hi_u(sy, k[p][d], F[d]);
        }
      }
      float cr[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cr[j] = F[2 * j].x; cr[j + 8] = F[2 * j + 1].x;
        cr[j + 4] = F[2 * j].y; cr[j + 12] = F[2 * j + 1].y;
      }
      const int ln = threadIdx.x & 63;
      Qw[((threadIdx.x >> 6) * TQR + i0 + ((ln >> 4) & 1)) * DH +
         (2 * ((ln >> 2) & 1) + 4 * ((ln >> 3) & 1) + ((ln >> 5) & 1))] = wave_sum16_spread(cr);
    }
    __syncthreads();
    // dQ rows of this tile over this key block: slot kb * copy batches + batch
    float* dqb = a.dq + (int64_t)(kb * ncb + cb) * a.dq_ss + (int64_t)b * a.dq_bs + h * DH;
    for (int idx = threadIdx.x; idx < qend * (DH / 4); idx += NTT) {
      const int i = idx / (DH / 4), cc = (idx - i * (DH / 4)) * 4;
      float4 acc = *reinterpret_cast<const float4*>(Qw + i * DH + cc);
#pragma unroll
      for (int wv = 1; wv < NWV; ++wv) {
        const float4 t = *reinterpret_cast<const float4*>(Qw + (wv * TQR + i) * DH + cc);
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
      }
      acc.x *= a.scale; acc.y *= a.scale; acc.z *= a.scale; acc.w *= a.scale;
      *reinterpret_cast<float4*>(dqb + (int64_t)(qt + i) * a.dq_ls + cc) = acc;
    }
  }
  const float kf = a.scale / a.scale_log2;
  float* dkb = a.dk + blockIdx.y * a.dk_ss + (int64_t)b * a.dk_bs + h * DH;
  float* dvb = a.dv + blockIdx.y * a.dk_ss + (int64_t)b * a.dv_bs + h * DH;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int j0 = key0 + 2 * p, j1 = j0 + 1;
    float r0[DH], r1[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = dk[p][d].x * kf; r1[d] = dk[p][d].y * kf; }
    if (j0 < a.Lk) str<DH>(dkb + (int64_t)j0 * a.dk_ls, r0);
    if (j1 < a.Lk) str<DH>(dkb + (int64_t)j1 * a.dk_ls, r1);
#pragma unroll
    for (int d = 0; d < DH; ++d) { r0[d] = dv[p][d].x; r1[d] = dv[p][d].y; }
    if (j0 < a.Lk) str<DH>(dvb + (int64_t)j0 * a.dv_ls, r0);
    if (j1 < a.Lk) str<DH>(dvb + (int64_t)j1 * a.dv_ls, r1);
  }
}

// ======================= few queries (Lq <= 16) ===========================
// The encoders' latent queries (2*latent_len = 8 rows) attend to the whole
// light curve / spectrum (60 / 983 keys).  Query-parallel tiling leaves 56 of
// 64 lanes idle there, so these kernels go key-parallel: one 256-thread
// workgroup per (b, h, group of SQ=8 queries), each thread owns keys
// j = tid, tid+256, ..., the softmax max / sum and the output rows are block
// reductions.  Backward is ONE kernel per (b, h): dK_j / dV_j are thread-local
// sums over the (<= 16) queries, dQ a block reduction.  Dropout decisions are
// re-derived from the same counter hash (attn_pair_bits) in both directions,
// so no bitmap is written.
constexpr int SNT = 256, SNW = SNT / 64, SQ = 8;

// sum (or max) of v[0..N) over the workgroup; result in out[0..N) (LDS)
template <int N, bool MAX>
__device__ __forceinline__ void block_reduce(float (&v)[N], float* red, float* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float x = MAX ? wave_max(v[i]) : wave_sum(v[i]);
    if (lane == 0) red[w * N + i] = x;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += SNT) {
    float x = red[i];
#pragma unroll
    for (int ww = 1; ww < SNW; ++ww) x = MAX ? fmaxf(x, red[ww * N + i]) : x + red[ww * N + i];
    out[i] = x;
  }
  __syncthreads();
}

__device__ __forceinline__ bool keep_of(uint32_t rk, int j, uint32_t thr) {
  const uint32_t bits = attn_pair_bits(rk, (uint32_t)(j >> 1));
  return ((j & 1) ? (bits >> 16) : (bits & 0xffffu)) >= thr;
}

template <int DH, bool DROP>
__global__ __launch_bounds__(SNT) void attn_fwd_smallq_kernel(AttnArgs a) {
  constexpr int NV = SQ * (DH + 1);
  __shared__ float qs[SQ * DH];
  __shared__ float red[SNW * NV];
  __shared__ float res[NV];
  const int bh = blockIdx.x, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.y * SQ;
  const int nq = min(SQ, a.Lq - q0);
  if (threadIdx.x < SQ * DH) {
    const int i = threadIdx.x / DH, d = threadIdx.x - i * DH;
    qs[threadIdx.x] = i < nq ? a.q[(int64_t)b * a.q_bs + (int64_t)(q0 + i) * a.q_ls + h * DH + d] * a.scale_log2 : 0.f;
  }
  __syncthreads();
  float q[SQ][DH];
#pragma unroll
  for (int i = 0; i < SQ; ++i) lrow<DH>(qs + i * DH, q[i]);
  uint32_t rk[SQ];
  if (DROP) {
    const uint32_t skey = key_of(a.rng_state, a.call_id);
#pragma unroll
    for (int i = 0; i < SQ; ++i)
      rk[i] = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + q0 + min(i, nq - 1)));
  }
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  // pass 1: row maxima
  float m[SQ];
#pragma unroll
  for (int i = 0; i < SQ; ++i) m[i] = -INFINITY;
  for (int j = threadIdx.x; j < a.Lk; j += SNT) {
    float kr[DH];
    ldr<DH>(kg + (int64_t)j * a.k_ls, kr);
    const float kb = kbg ? kbg[j] : 0.f;
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      float sc = kb;
#pragma unroll
      for (int d = 0; d < DH; ++d) sc = fmaf(q[i][d], kr[d], sc);
      m[i] = fmaxf(m[i], sc);
    }
  }
  block_reduce<SQ, true>(m, red, res);
  float mu[SQ];
#pragma unroll
  for (int i = 0; i < SQ; ++i) {
    m[i] = res[i];
    mu[i] = m[i] == -INFINITY ? 0.f : m[i];    // fully masked row -> l = 0 -> NaN output
  }
  __syncthreads();
  // pass 2: l (undropped) and o (dropped) partial sums
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  for (int j = threadIdx.x; j < a.Lk; j += SNT) {
    float kr[DH], vr[DH];
    ldr<DH>(kg + (int64_t)j * a.k_ls, kr);
    ldr<DH>(vg + (int64_t)j * a.v_ls, vr);
    const float kb = kbg ? kbg[j] : 0.f;
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      float sc = kb;
#pragma unroll
      for (int d = 0; d < DH; ++d) sc = fmaf(q[i][d], kr[d], sc);
      float p = ex2(sc - mu[i]);
      acc[i] += p;
      if (DROP && !keep_of(rk[i], j, a.thr)) p = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) acc[SQ + i * DH + d] = fmaf(p, vr[d], acc[SQ + i * DH + d]);
    }
  }
  block_reduce<NV, false>(acc, red, res);
  const float ik = DROP ? a.inv_keep : 1.f;
  if (threadIdx.x < nq * DH) {
    const int i = threadIdx.x / DH, d = threadIdx.x - i * DH;
    a.o_out[(int64_t)b * a.o_bs + (int64_t)(q0 + i) * a.o_ls + h * DH + d] = res[SQ + threadIdx.x] * ik / res[i];
  }
  if (threadIdx.x < nq) {
    const int i = threadIdx.x;
    a.lse[(int64_t)bh * a.Lq + q0 + i] = m[i] + __log2f(res[i]);
  }
}

template <int DH, bool DROP>
__global__ __launch_bounds__(SNT) void attn_bwd_smallq_kernel(AttnArgs a) {
  constexpr int SQ = 64 / DH;   // query group: dQ partials SQ*DH = 64 registers
  __shared__ float qs[SQ * DH], gs[SQ * DH], lsh[SQ], Dsh[SQ];
  __shared__ float red[SNW * SQ * DH];
  __shared__ float res[SQ * DH];
  const int bh = blockIdx.x, b = bh / a.H, h = bh - b * a.H;
  const float* kg = a.k + (int64_t)b * a.k_bs + h * DH;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * DH;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  const float ik = DROP ? a.inv_keep : 1.f;
  const float kf = a.scale / a.scale_log2;
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;
  for (int q0 = 0; q0 < a.Lq; q0 += SQ) {
    const int nq = min(SQ, a.Lq - q0);
    __syncthreads();
    if (threadIdx.x < SQ * DH) {
      const int i = threadIdx.x / DH, d = threadIdx.x - i * DH;
      const int64_t r = q0 + i;
      qs[threadIdx.x] = i < nq ? a.q[(int64_t)b * a.q_bs + r * a.q_ls + h * DH + d] * a.scale_log2 : 0.f;
      gs[threadIdx.x] = i < nq ? a.dout[(int64_t)b * a.do_bs + r * a.do_ls + h * DH + d] : 0.f;
    }
    if (threadIdx.x < SQ) {
      const int i = threadIdx.x;
      float D = 0.f, l = INFINITY;    // padding rows: p = 0
      if (i < nq) {
        float x[DH], y[DH];
        ldr<DH>(a.dout + (int64_t)b * a.do_bs + (int64_t)(q0 + i) * a.do_ls + h * DH, x);
        ldr<DH>(a.o + (int64_t)b * a.o_bs + (int64_t)(q0 + i) * a.o_ls + h * DH, y);
#pragma unroll
        for (int d = 0; d < DH; ++d) D = fmaf(x[d], y[d], D);
        l = a.lse[(int64_t)bh * a.Lq + q0 + i];
      }
      Dsh[i] = D;
      lsh[i] = l;
    }
    __syncthreads();
    // q / dO rows are re-read per key as LDS broadcasts (keeps dh=16 in registers)
    float dq[SQ * DH], lse[SQ], D[SQ];
    uint32_t rk[SQ];
#pragma unroll
    for (int i = 0; i < SQ; ++i) {
      lse[i] = lsh[i];
      D[i] = Dsh[i];
      if (DROP) rk[i] = attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + q0 + min(i, nq - 1)));
    }
#pragma unroll
    for (int i = 0; i < SQ * DH; ++i) dq[i] = 0.f;
    for (int j = threadIdx.x; j < a.Lk; j += SNT) {
      float kr[DH], vr[DH], dk[DH], dv[DH];
      ldr<DH>(kg + (int64_t)j * a.k_ls, kr);
      ldr<DH>(vg + (int64_t)j * a.v_ls, vr);
      const float kb = kbg ? kbg[j] : 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
#pragma unroll
      for (int i = 0; i < SQ; ++i) {
        float qi[DH], gi[DH];
        lrow<DH>(qs + i * DH, qi);
        lrow<DH>(gs + i * DH, gi);
        float sc = kb, dp = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          sc = fmaf(qi[d], kr[d], sc);
          dp = fmaf(gi[d], vr[d], dp);
        }
        const float p = ex2(sc - lse[i]);
        float aP = p * ik, dP = dp * ik;
        if (DROP && !keep_of(rk[i], j, a.thr)) { aP = 0.f; dP = 0.f; }
        const float dS = p * (dP - D[i]);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          dv[d] = fmaf(aP, gi[d], dv[d]);
          dk[d] = fmaf(dS, qi[d], dk[d]);
          dq[i * DH + d] = fmaf(dS, kr[d], dq[i * DH + d]);
        }
      }
      float* dkp = a.dk + (int64_t)b * a.dk_bs + (int64_t)j * a.dk_ls + h * DH;
      float* dvp = a.dv + (int64_t)b * a.dv_bs + (int64_t)j * a.dv_ls + h * DH;
#pragma unroll
      for (int d = 0; d < DH; ++d) dk[d] *= kf;
      if (q0 > 0) {   // this thread owns key j in every query group: plain RMW
        float ok[DH], ov[DH];
        ldr<DH>(dkp, ok);
        ldr<DH>(dvp, ov);
#pragma unroll
        for (int d = 0; d < DH; ++d) { dk[d] += ok[d]; dv[d] += ov[d]; }
      }
      str<DH>(dkp, dk);
      str<DH>(dvp, dv);
    }
    block_reduce<SQ * DH, false>(dq, red, res);
    if (threadIdx.x < nq * DH) {
      const int i = threadIdx.x / DH, d = threadIdx.x - i * DH;
      a.dq[(int64_t)b * a.dq_bs + (int64_t)(q0 + i) * a.dq_ls + h * DH + d] = res[threadIdx.x] * a.scale;
    }
  }
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
  a.kchunk = Lk; a.qchunk = Lq;
}

// Geometry: rows per lane R = 2*NP (NP = 2 amortises each LDS read over four
// rows) and workgroup size NTT in {256, 128, 64}.  Of (NP=2: 256,128,64; NP=1:
// 256,128,64), the geometries yielding >= 1024 workgroups (4 per CU) compete on
// row-slot efficiency; the small encoder grids (B*H = 64) fall through to NP=1
// / 64 threads.
struct Geo { int nt, np; };
// forced geometry: vaesne_attn_force_geometry() (tests: every geometry is reachable on
// small shapes); nt = 0 -> auto
Geo g_forced{0, 0};
// geometry of the split launches (grids that leave a split in place): 256 x 2 (staging
// shared by 4 waves; A/B 9.52 -> 9.49 ms per step against the row-slot rule)
constexpr Geo kSplitGeo{256, 2};
Geo pick_geo(int64_t bh, int L) {
  if (g_forced.nt > 0) return g_forced;
  // among geometries with >= 1024 workgroups, the one wasting the fewest row
  // slots (short sequences: the photometry decoder's 60 tokens x 1024 (b, h)
  // fill 60 of 1024 rows at 256x2 but 60 of 128 at 64x1); ties keep the order
  const int nts[3] = {256, 128, 64};
  Geo best{64, 1};
  double best_eff = -1.0;
  for (int np = 2; np >= 1; --np)
    for (int i = 0; i < 3; ++i) {
      const int nt = nts[i], rows = 2 * np * nt;
      const int64_t nb = (L + rows - 1) / rows;
      const double eff = (double)L / (double)(rows * nb);
      if (bh * nb >= 1024 && eff > best_eff + 1e-9) { best = {nt, np}; best_eff = eff; }
    }
  if (L >= 256) {   // this pick would be split (< 2048 waves): the split geometry
    const int64_t waves = bh * ((L + 2 * best.np * best.nt - 1) / (2 * best.np * best.nt)) *
                          (best.nt / 64);
    if (waves < 2048) return kSplitGeo;
  }
  return best;
}

int64_t waves_of(int64_t bh, int L);

// Split launches for grids too small to fill the chip (the encoder's 983-token
// context self-attention: B*H = 64 sequences -> 512 one-wave workgroups): the
// streamed axis (keys for the forward / dQ, queries for dK / dV) is cut into
// `n` chunks of a multiple of 64 (= TK and two keep-bitmap words), each chunk a
// grid row; partial results go to the workspace and a fixed-order combine
// kernel finishes them (bitwise reproducible).
struct Split { int n, chunk; };
// target waves of a split launch (2048 / 8192 measured slower in the step)
constexpr int64_t kSplitWaves = 4096;
Split pick_split(int64_t waves, int L) {
  Split sp{1, L};
  if (waves >= 2048 || L < 256) return sp;
  int n = (int)std::min<int64_t>(16, (kSplitWaves + waves - 1) / waves);
  n = std::min(n, L / 128);
  if (n <= 1) return sp;
  sp.chunk = ((L + n - 1) / n + 63) / 64 * 64;
  sp.n = (L + sp.chunk - 1) / sp.chunk;
  return sp;
}
int64_t waves_of(int64_t bh, int L) {
  const Geo g = pick_geo(bh, L);
  return bh * ((L + 2 * g.np * g.nt - 1) / (2 * g.np * g.nt)) * (g.nt / 64);
}

// o = sum_c o_c 2^(m_c - M) * ik / L,  L = sum_c l_c 2^(m_c - M),  lse = M + log2 L
template <int DH>
__global__ void attn_fwd_combine_kernel(const float* __restrict__ po, int64_t o_ss,
                                        const float* __restrict__ ml, int n, int B, int H, int Lq,
                                        float ik, float* __restrict__ o, int64_t o_bs,
                                        int64_t o_ls, float* __restrict__ lse) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t BHL = (int64_t)B * H * Lq;
  if (t >= BHL) return;
  const int q = (int)(t % Lq);
  const int64_t bh = t / Lq;
  const int h = (int)(bh % H), b = (int)(bh / H);
  float M = -INFINITY;
  for (int c = 0; c < n; ++c) M = fmaxf(M, ml[(c * BHL + t) * 2]);
  const float Mu = M == -INFINITY ? 0.f : M;
  float L = 0.f, acc[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = 0.f;
  for (int c = 0; c < n; ++c) {
    const float w = ex2(ml[(c * BHL + t) * 2] - Mu);
    L = fmaf(ml[(c * BHL + t) * 2 + 1], w, L);
    float r[DH];
    ldr<DH>(po + c * o_ss + ((int64_t)b * Lq + q) * (H * DH) + h * DH, r);
#pragma unroll
    for (int d = 0; d < DH; ++d) acc[d] = fmaf(w, r[d], acc[d]);
  }
  const float sc = ik / L;   // L == 0 (every key masked): NaN, as the reference
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] *= sc;
  str<DH>(o + (int64_t)b * o_bs + (int64_t)q * o_ls + h * DH, acc);
  lse[t] = M + __log2f(L);
}

// out[b, l, e] = sum_c ws[c][b, l, e]  (dense [B, L, E] chunks, stride ss)
__global__ void attn_sum_chunks_kernel(const float* __restrict__ ws, int64_t ss, int n, int B,
                                       int L, int E, float* __restrict__ out, int64_t bs,
                                       int64_t ls) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * L * E) return;
  const int e = (int)(t % E);
  const int64_t bl = t / E;
  const int l = (int)(bl % L), b = (int)(bl / L);
  float v = 0.f;
  for (int c = 0; c < n; ++c) v += ws[c * ss + t];
  out[(int64_t)b * bs + (int64_t)l * ls + e] = v;
}

// attn_sum_chunks_kernel with 4 adjacent features per thread (16-byte loads / stores)
__global__ void attn_sum_chunks4_kernel(const float* __restrict__ ws, int64_t ss, int n, int B,
                                        int L, int E, float* __restrict__ out, int64_t bs,
                                        int64_t ls) {
  const int64_t t = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (t >= (int64_t)B * L * E) return;
  const int e = (int)(t % E);
  const int64_t bl = t / E;
  const int l = (int)(bl % L), b = (int)(bl / L);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < n; ++c) {
    const float4 w = *reinterpret_cast<const float4*>(ws + c * ss + t);
    v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
  }
  *reinterpret_cast<float4*>(out + (int64_t)b * bs + (int64_t)l * ls + e) = v;
}

// out = sum of n dense [B, L, E] chunks (stride ss) -- same per-element order either way
void launch_sum_chunks(const float* ws, int64_t ss, int n, int B, int L, int E, float* out,
                       int64_t bs, int64_t ls, hipStream_t s) {
  const int64_t total = (int64_t)B * L * E;
  if (E % 4 == 0 && ss % 4 == 0 && bs % 4 == 0 && ls % 4 == 0 && (uintptr_t)ws % 16 == 0 &&
      (uintptr_t)out % 16 == 0)
    hipLaunchKernelGGL(attn_sum_chunks4_kernel, dim3((unsigned)((total / 4 + 255) / 256)),
                       dim3(256), 0, s, ws, ss, n, B, L, E, out, bs, ls);
  else
    hipLaunchKernelGGL(attn_sum_chunks_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256),
                       0, s, ws, ss, n, B, L, E, out, bs, ls);
}

// the split-f16 matrix-core kernels (attention_sf16.hip) for head_dim 8 unless a test forces
// a packed-VALU geometry
bool use_sf16(int dh, int64_t bh, int Lq, int Lk) {
  return g_forced.nt == 0 && sf16_path(dh, bh, Lq, Lk);
}
// the repeated-sequence kernels: split-f16 unless a packed-VALU geometry is forced (the plain
// path's rule, so a forced geometry selects the VALU kernels on both paths)
bool use_rep_sf16(int L, int R) { return g_forced.nt == 0 && sf16_rep_path(L, R); }

// Keep-bitmap layout guard: each forward records which kernel family (layout) and shape wrote
// a bitmap; a backward that would read it with the other family -- a geometry override
// flipped between the two calls -- fails with hipErrorInvalidValue instead of reading the
// wrong bits.  Host side only (a captured graph replays both as captured).
enum BitsFamily { kBitsValu = 1, kBitsSf16 = 2 };
struct BitsTag { int fam, B, H, Lq, Lk; };
std::mutex g_bits_mu;
std::unordered_map<const void*, BitsTag> g_bits;
void bits_record(const void* bits, int fam, int B, int H, int Lq, int Lk) {
  if (!bits) return;
  std::lock_guard<std::mutex> lk(g_bits_mu);
  if (g_bits.size() > 65536) g_bits.clear();
  g_bits[bits] = {fam, B, H, Lq, Lk};
}
bool bits_check(const void* bits, int fam, int B, int H, int Lq, int Lk) {
  if (!bits) return true;
  std::lock_guard<std::mutex> lk(g_bits_mu);
  const auto it = g_bits.find(bits);
  if (it == g_bits.end()) return true;   // written elsewhere (the caller's own bitmap)
  const BitsTag& t = it->second;
  return t.fam == fam && t.B == B && t.H == H && t.Lq == Lq && t.Lk == Lk;
}

// workspace of a split launch (bytes; 0 = no split for this shape)
int64_t fwd_ws_floats(int B, int H, int Lq, int Lk, int dh, Split& sp) {
  sp = {1, Lk};
  if (Lq <= 2 * SQ || use_sf16(dh, (int64_t)B * H, Lq, Lk)) return 0;
  sp = pick_split(waves_of((int64_t)B * H, Lq), Lk);
  if (sp.n <= 1) return 0;
  return (int64_t)sp.n * B * Lq * H * dh + (int64_t)sp.n * B * H * Lq * 2;
}
// key blocks of the dK/dV launch (the fused dQ's partial count)
int kv_blocks(int64_t bh, int Lk, int dh) {
  const Geo g = pick_geo(bh, Lk);
  return (Lk + 2 * g.np * g.nt - 1) / (2 * g.np * g.nt);
}
// floats of the dQ region: per-key-chunk partials of the dQ kernel, or (head_dim
// 8, dQ fused into the dK/dV kernel) one partial per key block when there are
// several; the larger of the two so either path fits
int64_t bwd_dq_floats(int B, int H, int Lq, int Lk, int dh, const Split& sq) {
  const int64_t unfused = (int64_t)(sq.n > 1 ? sq.n : 0) * B * Lq * H * dh;
  const int nkb = kv_blocks((int64_t)B * H, Lk, dh);
  const int64_t fused = dh == 8 && nkb > 1 ? (int64_t)nkb * B * Lq * H * dh : 0;
  return std::max(unfused, fused);
}
int64_t bwd_ws_floats(int B, int H, int Lq, int Lk, int dh, Split& sq, Split& sk) {
  sq = {1, Lk};   // dQ: key chunks
  sk = {1, Lq};   // dK/dV: query chunks
  if (Lq <= 2 * SQ) return 0;
  if (use_sf16(dh, (int64_t)B * H, Lq, Lk)) return sf16_bwd_ws_floats(B, H, Lq, Lk);
  sq = pick_split(waves_of((int64_t)B * H, Lq), Lk);
  sk = pick_split(waves_of((int64_t)B * H, Lk), Lq);
  return bwd_dq_floats(B, H, Lq, Lk, dh, sq) +
         (int64_t)(sk.n > 1 ? sk.n : 0) * B * Lk * H * dh * 2;
}

#define VAESNE_GEO_SWITCH(G, CALL)                                                     \
  if (G.np == 2) {                                                                     \
    constexpr int NP = 2;                                                              \
    switch (G.nt) {                                                                    \
      case 256: { constexpr int NTT = 256; CALL; break; }                              \
      case 128: { constexpr int NTT = 128; CALL; break; }                              \
      default: { constexpr int NTT = 64; CALL; break; }                                \
    }                                                                                  \
  } else {                                                                             \
    constexpr int NP = 1;                                                              \
    switch (G.nt) {                                                                    \
      case 256: { constexpr int NTT = 256; CALL; break; }                              \
      case 128: { constexpr int NTT = 128; CALL; break; }                              \
      default: { constexpr int NTT = 64; CALL; break; }                                \
    }                                                                                  \
  }

template <int DHV>
int launch_fwd(const AttnArgs& a, float p_drop, float* ws, hipStream_t s) {
  if (a.Lq <= 2 * SQ) {
    dim3 grid((unsigned)((int64_t)a.B * a.H), (unsigned)((a.Lq + SQ - 1) / SQ));
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_fwd_smallq_kernel<DHV, true>), grid, dim3(SNT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_fwd_smallq_kernel<DHV, false>), grid, dim3(SNT), 0, s, a);
    VAESNE_CHECK_LAUNCH();
    return 0;
  }
  if (use_sf16(DHV, (int64_t)a.B * a.H, a.Lq, a.Lk)) return sf16_fwd(a, p_drop, s);
  Split sp;
  const int64_t wsf = fwd_ws_floats(a.B, a.H, a.Lq, a.Lk, DHV, sp);
  AttnArgs c = a;
  if (wsf > 0 && ws) {   // chunked keys: partial o / (m, l) into the workspace
    c.kchunk = sp.chunk;
    c.o_out = ws; c.o_bs = (int64_t)a.Lq * a.H * DHV; c.o_ls = (int64_t)a.H * DHV;
    c.o_ss = (int64_t)a.B * a.Lq * a.H * DHV;
    c.ml = ws + sp.n * c.o_ss;
  } else {
    sp = {1, a.Lk};
  }
  const Geo g = pick_geo((int64_t)a.B * a.H, a.Lq);
  VAESNE_GEO_SWITCH(g, {
    const int nqb = (a.Lq + 2 * NP * NTT - 1) / (2 * NP * NTT);
    dim3 grid((unsigned)((int64_t)a.B * a.H * nqb), (unsigned)sp.n);
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_fwd_kernel<DHV, NTT, NP, true>), grid, dim3(NTT), 0, s, c);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<DHV, NTT, NP, false>), grid, dim3(NTT), 0, s, c);
  })
  VAESNE_CHECK_LAUNCH();
  if (sp.n > 1) {
    const int64_t n = (int64_t)a.B * a.H * a.Lq;
    hipLaunchKernelGGL((attn_fwd_combine_kernel<DHV>), dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, s, c.o_out, c.o_ss, c.ml, sp.n, a.B, a.H, a.Lq,
                       p_drop > 0.f ? a.inv_keep : 1.f, a.o_out, a.o_bs, a.o_ls, a.lse);
    VAESNE_CHECK_LAUNCH();
  }
  return 0;
}

// part: 1 = dK/dV kernel, 2 = dQ kernel, 3 = both (the few-query path is one
// fused kernel and runs for any nonzero part)
template <int DHV>
int launch_bwd(const AttnArgs& a, float p_drop, int part, float* ws, hipStream_t s) {
  if (a.Lq <= 2 * SQ) {
    dim3 grid((unsigned)((int64_t)a.B * a.H));
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_bwd_smallq_kernel<DHV, true>), grid, dim3(SNT), 0, s, a);
    else
      hipLaunchKernelGGL((attn_bwd_smallq_kernel<DHV, false>), grid, dim3(SNT), 0, s, a);
    VAESNE_CHECK_LAUNCH();
    return 0;
  }
  // the split-f16 backward is one fused kernel: every part runs it whole
  if (use_sf16(DHV, (int64_t)a.B * a.H, a.Lq, a.Lk)) return sf16_bwd(a, p_drop, ws, s);
  Split sq, sk;
  const int64_t wsf = bwd_ws_floats(a.B, a.H, a.Lq, a.Lk, DHV, sq, sk);
  if (wsf == 0 || !ws) { sq = {1, a.Lk}; sk = {1, a.Lq}; }
  const int E = a.H * DHV;
  float* ws_dq = ws;
  float* ws_dkv = ws && wsf > 0 ? ws + bwd_dq_floats(a.B, a.H, a.Lq, a.Lk, DHV, sq) : nullptr;
  // fused dK/dV/dQ (head_dim 8): one key block covers the whole key axis (dQ
  // written directly), or several write dQ partials into the workspace
  const int nkb = kv_blocks((int64_t)a.B * a.H, a.Lk, DHV);
  const bool fuse = DHV == 8 && part == 3 && (nkb == 1 || (ws && wsf > 0));
  if (part & 1) {
    AttnArgs c = a;
    if (sk.n > 1) {   // chunked queries: partial dK / dV per chunk
      c.qchunk = sk.chunk;
      c.dk = ws_dkv; c.dk_bs = (int64_t)a.Lk * E; c.dk_ls = E;
      c.dv = ws_dkv + (int64_t)sk.n * a.B * a.Lk * E; c.dv_bs = c.dk_bs; c.dv_ls = E;
      c.dk_ss = (int64_t)a.B * a.Lk * E;
    }
    if (fuse && nkb > 1) {   // fused dQ over several key blocks: partial per block
      c.dq = ws_dq; c.dq_bs = (int64_t)a.Lq * E; c.dq_ls = E;
      c.dq_ss = (int64_t)a.B * a.Lq * E;
    }
    const Geo gk = pick_geo((int64_t)a.B * a.H, a.Lk);
    VAESNE_GEO_SWITCH(gk, {
      const int nkb = (a.Lk + 2 * NP * NTT - 1) / (2 * NP * NTT);
      dim3 grid((unsigned)((int64_t)a.B * a.H * nkb), (unsigned)sk.n);
      if (fuse) {
        if (p_drop > 0.f)
          hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, NP, true, DHV == 8>), grid, dim3(NTT),
                             0, s, c);
        else
          hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, NP, false, DHV == 8>), grid,
                             dim3(NTT), 0, s, c);
      } else if (p_drop > 0.f) {
        hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, NP, true>), grid, dim3(NTT), 0, s, c);
      } else {
        hipLaunchKernelGGL((attn_bwd_kv_kernel<DHV, NTT, NP, false>), grid, dim3(NTT), 0, s, c);
      }
    })
    VAESNE_CHECK_LAUNCH();
    if (sk.n > 1) {
      launch_sum_chunks(c.dk, c.dk_ss, sk.n, a.B, a.Lk, E, a.dk, a.dk_bs, a.dk_ls, s);
      VAESNE_CHECK_LAUNCH();
      launch_sum_chunks(c.dv, c.dk_ss, sk.n, a.B, a.Lk, E, a.dv, a.dv_bs, a.dv_ls, s);
      VAESNE_CHECK_LAUNCH();
    }
    if (fuse && nkb > 1) {
      launch_sum_chunks(c.dq, c.dq_ss, nkb, a.B, a.Lq, E, a.dq, a.dq_bs, a.dq_ls, s);
      VAESNE_CHECK_LAUNCH();
    }
  }
  if ((part & 2) && !fuse) {
    AttnArgs c = a;
    if (sq.n > 1) {   // chunked keys: partial dQ per chunk
      c.kchunk = sq.chunk;
      c.dq = ws_dq; c.dq_bs = (int64_t)a.Lq * E; c.dq_ls = E;
      c.dq_ss = (int64_t)a.B * a.Lq * E;
    }
    const Geo gq = pick_geo((int64_t)a.B * a.H, a.Lq);
    VAESNE_GEO_SWITCH(gq, {
      const int nqb = (a.Lq + 2 * NP * NTT - 1) / (2 * NP * NTT);
      dim3 grid((unsigned)((int64_t)a.B * a.H * nqb), (unsigned)sq.n);
      if (p_drop > 0.f)
        hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, NTT, NP, true>), grid, dim3(NTT), 0, s, c);
      else
        hipLaunchKernelGGL((attn_bwd_q_kernel<DHV, NTT, NP, false>), grid, dim3(NTT), 0, s, c);
    })
    VAESNE_CHECK_LAUNCH();
    if (sq.n > 1) {
      launch_sum_chunks(c.dq, c.dq_ss, sq.n, a.B, a.Lq, E, a.dq, a.dq_bs, a.dq_ls, s);
      VAESNE_CHECK_LAUNCH();
    }
  }
  return 0;
}

// ---- repeated sequences (attn_rep_*): configuration and plans ----
// forward: fnt threads x 2 queries per lane, frc copies per workgroup (frc sets of
// 8 packed accumulators); backward: bnt threads x 2*bnp keys per lane, brc copies
// per staged tile, query chunks sized so the grid has ~bwgs workgroups.
// forward fnp query pairs per lane.  vaesne_attn_rep_config() overrides (tests).
struct RepCfg { int fnt, frc, bnt, bnp, brc, bwgs, fnp; };
// bwgs 768: the block-1 backward now runs beside the encoders' backward chain (since the
// latent gradient sums moved into their own kernels), and half the workgroups leave that
// latency-bound chain more free slots (step A/B 8.79 vs 8.82 ms, profiles/r04_ab/rep_bwgs.txt)
const RepCfg kRepDefault{0, 2, 256, 1, 16, 768, 1};
RepCfg g_rep = kRepDefault;
bool rep_cfg_ok(const RepCfg& c) {
  return (c.fnt == 0 || c.fnt == 64 || c.fnt == 128 || c.fnt == 256) &&
         (c.frc == 2 || c.frc == 4 || c.frc == 8) && (c.bnt == 128 || c.bnt == 256) &&
         (c.bnp == 1 || c.bnp == 2) && (c.brc == 8 || c.brc == 16) && c.bwgs > 0 &&
         (c.fnp == 1 || (c.fnp == 2 && c.frc <= 4));
}
int rep_fwd_nt(int64_t bh, int L, int cb, int np) {
  if (g_rep.fnt > 0) return g_rep.fnt;
  // fewest wasted query slots among grids of >= 1024 workgroups (else 64 threads)
  const int nts[3] = {256, 128, 64};
  int best = 64;
  double best_eff = -1.0;
  for (int nt : nts) {
    const int rows = 2 * np * nt;
    const int64_t nb = (L + rows - 1) / rows;
    const double eff = (double)L / (double)(rows * nb);
    if (bh * nb * cb >= 1024 && eff > best_eff + 1e-9) { best = nt; best_eff = eff; }
  }
  return best;
}
struct RepPlan { int nkb, QS, chunk, CB; int64_t dkv_floats, dq_floats, dsum_floats, std_floats; };
RepPlan rep_bwd_plan(int Bd, int R, int H, int L, float p_drop) {
  RepPlan pl{};
  const int E = H * 8;
  if (p_drop <= 0.f) {   // no dropout: copies identical -> one plain backward on sum_r dO_r
    Split sq, sk;
    pl.dsum_floats = (int64_t)Bd * L * E;
    pl.std_floats = bwd_ws_floats(Bd, H, L, L, 8, sq, sk);
    return pl;
  }
  if (use_rep_sf16(L, R)) {   // query-chunk partials of dK / dV only (dQ complete)
    pl.dkv_floats = sf16_rep_bwd_ws_floats(Bd, H, L);
    return pl;
  }
  const int KB = 2 * g_rep.bnp * g_rep.bnt;
  pl.nkb = (L + KB - 1) / KB;
  pl.CB = (R + g_rep.brc - 1) / g_rep.brc;
  const int64_t per = (int64_t)Bd * H * pl.nkb * pl.CB;
  const int tiles = (L + TQR - 1) / TQR;
  int qs = (int)std::max<int64_t>(1, (g_rep.bwgs + per / 2) / per);
  qs = std::min(qs, tiles);
  pl.chunk = (tiles + qs - 1) / qs * TQR;
  pl.QS = (L + pl.chunk - 1) / pl.chunk;
  pl.dkv_floats = pl.QS * pl.CB > 1 ? 2 * (int64_t)pl.QS * pl.CB * Bd * L * E : 0;
  pl.dq_floats = pl.nkb * pl.CB > 1 ? (int64_t)pl.nkb * pl.CB * Bd * L * E : 0;
  return pl;
}

// query blocks [p0 * nqb / np_, p1 * nqb / np_) of the launch geometry
int launch_rep_fwd(const AttnArgs& a, int R, float p_drop, int p0, int p1, int np_, hipStream_t s) {
  if (use_rep_sf16(a.Lq, R)) return sf16_rep_fwd(a, R, p_drop, p0, p1, np_, s);
  const bool drop = p_drop > 0.f;
  const int rc = drop ? g_rep.frc : 1;
  const int cb = drop ? (R + rc - 1) / rc : 1;
  const int np = drop ? g_rep.fnp : 1;
  const int nt = rep_fwd_nt((int64_t)a.B * a.H, a.Lq, cb, np);
  const int nqb = (a.Lq + 2 * np * nt - 1) / (2 * np * nt);
  const int qb0 = (int)((int64_t)p0 * nqb / np_), qb1 = (int)((int64_t)p1 * nqb / np_);
  const int nqbs = qb1 - qb0;
  if (nqbs <= 0) return 0;
  const dim3 grid((unsigned)((int64_t)a.B * a.H * nqbs), (unsigned)cb);
#define VAESNE_REP_FWD(NT)                                                                        \
  if (!drop) hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 1, 1, false>), grid, dim3(NT), 0, s, a, R, qb0, nqbs); \
  else if (np == 2 && rc == 2) hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 2, 2, true>), grid, dim3(NT), 0, s, a, R, qb0, nqbs); \
  else if (np == 2) hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 2, 4, true>), grid, dim3(NT), 0, s, a, R, qb0, nqbs); \
  else if (rc == 2) hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 1, 2, true>), grid, dim3(NT), 0, s, a, R, qb0, nqbs); \
  else if (rc == 4) hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 1, 4, true>), grid, dim3(NT), 0, s, a, R, qb0, nqbs); \
  else hipLaunchKernelGGL((attn_rep_fwd_kernel<8, NT, 1, 8, true>), grid, dim3(NT), 0, s, a, R, qb0, nqbs);
  if (nt == 256) { VAESNE_REP_FWD(256) } else if (nt == 128) { VAESNE_REP_FWD(128) } else { VAESNE_REP_FWD(64) }
#undef VAESNE_REP_FWD
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int launch_rep_bwd(const AttnArgs& a, int R, float p_drop, float* ws, hipStream_t s) {
  const int E = a.H * 8;
  const RepPlan pl = rep_bwd_plan(a.B, R, a.H, a.Lq, p_drop);
  if (p_drop <= 0.f) {
    // every copy's O and P are the same: dS summed over copies = P (V.sum_r dO_r - sum_r D_r),
    // sum_r D_r = O . sum_r dO_r -- the plain backward of (qkv, O, sum_r dO_r)
    float* dsum = ws;
    launch_sum_chunks(a.dout, (int64_t)a.B * a.do_bs, R, a.B, a.Lq, E, dsum, (int64_t)a.Lq * E, (int64_t)E, s);
    VAESNE_CHECK_LAUNCH();
    AttnArgs c = a;
    c.dout = dsum; c.do_bs = (int64_t)a.Lq * E; c.do_ls = E;
    return launch_bwd<8>(c, 0.f, 3, pl.std_floats > 0 ? ws + pl.dsum_floats : nullptr, s);
  }
  if (use_rep_sf16(a.Lq, R)) return sf16_rep_bwd(a, R, ws, s);
  AttnArgs c = a;
  c.qchunk = pl.chunk;
  float* wdkv = ws;
  float* wdq = ws + pl.dkv_floats;
  if (pl.dkv_floats > 0) {
    c.dk = wdkv; c.dk_bs = (int64_t)a.Lk * E; c.dk_ls = E;
    c.dv = wdkv + (int64_t)pl.QS * pl.CB * a.B * a.Lk * E; c.dv_bs = c.dk_bs; c.dv_ls = E;
    c.dk_ss = (int64_t)a.B * a.Lk * E;
  } else {
    c.dk_ss = 0;
  }
  if (pl.dq_floats > 0) {
    c.dq = wdq; c.dq_bs = (int64_t)a.Lq * E; c.dq_ls = E;
    c.dq_ss = (int64_t)a.B * a.Lq * E;
  } else {
    c.dq_ss = 0;
  }
  const dim3 grid((unsigned)((int64_t)a.B * a.H * pl.nkb), (unsigned)(pl.QS * pl.CB));
#define VAESNE_REP_BWD(NT, NP)                                                                     \
  if (g_rep.brc == 16) hipLaunchKernelGGL((attn_rep_bwd_kernel<NT, NP, 16>), grid, dim3(NT), 0, s, c, R, pl.QS); \
  else hipLaunchKernelGGL((attn_rep_bwd_kernel<NT, NP, 8>), grid, dim3(NT), 0, s, c, R, pl.QS);
  if (g_rep.bnt == 256) {
    if (g_rep.bnp == 2) { VAESNE_REP_BWD(256, 2) } else { VAESNE_REP_BWD(256, 1) }
  } else {
    if (g_rep.bnp == 2) { VAESNE_REP_BWD(128, 2) } else { VAESNE_REP_BWD(128, 1) }
  }
#undef VAESNE_REP_BWD
  VAESNE_CHECK_LAUNCH();
  if (pl.dkv_floats > 0) {
    launch_sum_chunks(c.dk, c.dk_ss, pl.QS * pl.CB, a.B, a.Lk, E, a.dk, a.dk_bs, a.dk_ls, s);
    VAESNE_CHECK_LAUNCH();
    launch_sum_chunks(c.dv, c.dk_ss, pl.QS * pl.CB, a.B, a.Lk, E, a.dv, a.dv_bs, a.dv_ls, s);
    VAESNE_CHECK_LAUNCH();
  }
  if (pl.dq_floats > 0) {
    launch_sum_chunks(c.dq, c.dq_ss, pl.nkb * pl.CB, a.B, a.Lq, E, a.dq, a.dq_bs, a.dq_ls, s);
    VAESNE_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace

VAESNE_API int vaesne_attn_rep_config(int fnt, int frc, int bnt, int bnp, int brc, int bwgs,
                                      int fnp) {
  if (fnt < 0) { g_rep = kRepDefault; return 0; }
  const RepCfg c{fnt, frc, bnt, bnp, brc, bwgs, fnp};
  if (!rep_cfg_ok(c)) return (int)hipErrorInvalidValue;
  g_rep = c;
  return 0;
}

VAESNE_API int vaesne_attn_rep_sf16_config(int frc, int bwgs) { return sf16_rep_config(frc, bwgs); }

VAESNE_API int64_t vaesne_attn_rep_workspace(int Bd, int R, int H, int L, int dh, float p_drop) {
  if (Bd <= 0 || R <= 0 || L <= 2 * SQ || dh != 8) return 0;
  const RepPlan pl = rep_bwd_plan(Bd, R, H, L, p_drop);
  return (pl.dkv_floats + pl.dq_floats + pl.dsum_floats + pl.std_floats) * (int64_t)sizeof(float);
}

namespace {
bool rep_args(AttnArgs& a, const float* qkv, int64_t qkv_bs, int64_t qkv_ls, const float* kbias,
              int64_t kb_bs, int Bd, int H, int L, int dh, float p_drop, const int64_t* rng_state,
              uint32_t call_id) {
  const int E = H * dh;
  a.q = qkv; a.k = qkv + E; a.v = qkv + 2 * E;
  a.q_bs = a.k_bs = a.v_bs = qkv_bs;
  a.q_ls = a.k_ls = a.v_ls = qkv_ls;
  a.kbias = kbias; a.kb_bs = kb_bs;
  fill_common(a, Bd, H, L, L, dh, p_drop, rng_state, call_id);
  return aligned16(a.q, qkv_ls) && aligned16(a.k, qkv_ls) && aligned16(a.v, qkv_ls);
}
}  // namespace

VAESNE_API int vaesne_attn_rep_fwd_part(const float* qkv, int64_t qkv_bs, int64_t qkv_ls,
                                        const float* kbias, int64_t kb_bs, float* o, int64_t o_bs,
                                        int64_t o_ls, float* lse, int Bd, int R, int H, int L,
                                        int dh, float p_drop, const int64_t* rng_state,
                                        uint32_t call_id, uint32_t* keep_bits, int p0, int p1,
                                        int nparts, void* stream) {
  if (Bd <= 0 || R <= 0 || L <= 0) return 0;
  if (nparts < 1 || p0 < 0 || p1 > nparts || p0 > p1) return (int)hipErrorInvalidValue;
  if (dh != 8 || L <= 2 * SQ || !rep_cfg_ok(g_rep)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && (!keep_bits || !rng_state)) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  if (!rep_args(a, qkv, qkv_bs, qkv_ls, kbias, kb_bs, Bd, H, L, dh, p_drop, rng_state, call_id) ||
      !aligned16(o, o_ls))
    return (int)hipErrorInvalidValue;
  a.o = o; a.o_out = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = lse;
  a.bits = keep_bits;
  if (p_drop > 0.f) bits_record(keep_bits, use_rep_sf16(L, R) ? kBitsSf16 : kBitsValu, R * Bd, H, L, L);
  return launch_rep_fwd(a, R, p_drop, p0, p1, nparts, (hipStream_t)stream);
}

VAESNE_API int vaesne_attn_rep_fwd(const float* qkv, int64_t qkv_bs, int64_t qkv_ls,
                                   const float* kbias, int64_t kb_bs, float* o, int64_t o_bs,
                                   int64_t o_ls, float* lse, int Bd, int R, int H, int L, int dh,
                                   float p_drop, const int64_t* rng_state, uint32_t call_id,
                                   uint32_t* keep_bits, void* stream) {
  return vaesne_attn_rep_fwd_part(qkv, qkv_bs, qkv_ls, kbias, kb_bs, o, o_bs, o_ls, lse, Bd, R, H,
                                  L, dh, p_drop, rng_state, call_id, keep_bits, 0, 1, 1, stream);
}

VAESNE_API int vaesne_attn_rep_bwd(const float* qkv, int64_t qkv_bs, int64_t qkv_ls,
                                   const float* kbias, int64_t kb_bs, const float* o, int64_t o_bs,
                                   int64_t o_ls, const float* lse, const float* dout,
                                   float* dqkv, int Bd, int R, int H, int L, int dh, float p_drop,
                                   const int64_t* rng_state, uint32_t call_id,
                                   const uint32_t* keep_bits, float* workspace, void* stream) {
  if (Bd <= 0 || R <= 0 || L <= 0) return 0;
  if (dh != 8 || L <= 2 * SQ || !rep_cfg_ok(g_rep)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && !keep_bits) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && !bits_check(keep_bits, use_rep_sf16(L, R) ? kBitsSf16 : kBitsValu, R * Bd, H, L, L))
    return (int)hipErrorInvalidValue;
  if (vaesne_attn_rep_workspace(Bd, R, H, L, dh, p_drop) > 0 && !workspace)
    return (int)hipErrorInvalidValue;
  const int E = H * dh;
  AttnArgs a{};
  if (!rep_args(a, qkv, qkv_bs, qkv_ls, kbias, kb_bs, Bd, H, L, dh, p_drop, rng_state, call_id) ||
      !aligned16(o, o_ls) || !aligned16(dout, E) || !aligned16(dqkv, qkv_ls))
    return (int)hipErrorInvalidValue;
  a.o = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = const_cast<float*>(lse);
  a.dout = dout; a.do_bs = (int64_t)L * E; a.do_ls = E;        // dense [R*Bd, L, E]
  a.dq = dqkv; a.dk = dqkv + E; a.dv = dqkv + 2 * E;
  a.dq_bs = a.dk_bs = a.dv_bs = qkv_bs;
  a.dq_ls = a.dk_ls = a.dv_ls = qkv_ls;
  a.bits = const_cast<uint32_t*>(keep_bits);
  return launch_rep_bwd(a, R, p_drop, workspace, (hipStream_t)stream);
}

VAESNE_API int vaesne_attn_force_geometry(int nt, int np) {
  if (nt == 0) { g_forced = {0, 0}; return 0; }
  if ((nt != 64 && nt != 128 && nt != 256) || (np != 1 && np != 2)) return (int)hipErrorInvalidValue;
  g_forced = {nt, np};
  return 0;
}

VAESNE_API int vaesne_mask_bias(const uint8_t* mask, int64_t n, float* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mask_bias_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, mask, n, out);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int64_t vaesne_attn_keep_bits_size(int B, int H, int Lq, int Lk) {
  // either kernel family's layout fits (the split-f16 one pads queries to 16, keys to 128)
  return std::max((int64_t)B * H * ((Lk + 31) / 32) * Lq * (int64_t)sizeof(uint32_t),
                  sf16_bits_bytes(B, H, Lq, Lk));
}

VAESNE_API int64_t vaesne_attn_workspace(int B, int H, int Lq, int Lk, int dh, int bwd) {
  if (B <= 0 || Lq <= 0 || Lk <= 0) return 0;
  Split a, b;
  const int64_t f = bwd ? bwd_ws_floats(B, H, Lq, Lk, dh, a, b) : fwd_ws_floats(B, H, Lq, Lk, dh, a);
  return f * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_attn_fwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const float* kbias, int64_t kb_bs, float* o,
                               int64_t o_bs, int64_t o_ls, float* lse, int B, int H, int Lq,
                               int Lk, int dh, float p_drop, const int64_t* rng_state,
                               uint32_t call_id, uint32_t* keep_bits, float* workspace,
                               void* stream) {
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
  if (p_drop > 0.f && Lq > 2 * SQ)
    bits_record(keep_bits, use_sf16(dh, (int64_t)B * H, Lq, Lk) ? kBitsSf16 : kBitsValu, B, H, Lq, Lk);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return launch_fwd<8>(a, p_drop, workspace, s);
  return launch_fwd<16>(a, p_drop, workspace, s);
}

namespace {
int attn_bwd_impl(const float* q, int64_t q_bs, int64_t q_ls, const float* k, int64_t k_bs,
                  int64_t k_ls, const float* v, int64_t v_bs, int64_t v_ls, const float* kbias,
                  int64_t kb_bs, const float* o, int64_t o_bs, int64_t o_ls, const float* lse,
                  const float* dout, int64_t do_bs, int64_t do_ls, float* dq, int64_t dq_bs,
                  int64_t dq_ls, float* dk, int64_t dk_bs, int64_t dk_ls, float* dv,
                  int64_t dv_bs, int64_t dv_ls, int B, int H, int Lq, int Lk, int dh,
                  float p_drop, const int64_t* rng_state, uint32_t call_id,
                  const uint32_t* keep_bits, float* workspace, int part, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || (dh != 8 && dh != 16)) return (int)hipErrorInvalidValue;
  // query-tiled kernels read the forward's keep bitmap; the few-query kernel
  // re-derives the decisions from rng_state / call_id
  if (p_drop > 0.f && (Lq > 2 * SQ ? !keep_bits : !rng_state)) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls) ||
      !aligned16(dout, do_ls) || !aligned16(dq, dq_ls) || !aligned16(dk, dk_ls) ||
      !aligned16(dv, dv_ls))
    return (int)hipErrorInvalidValue;
  // one fused kernel (the few-query path, the split-f16 path) writes dq, dk and dv whichever
  // part is asked for: all three must be given
  if ((Lq <= 2 * SQ || use_sf16(dh, (int64_t)B * H, Lq, Lk)) && (!dq || !dk || !dv))
    return (int)hipErrorInvalidValue;
  // the bitmap must come from the kernel family this backward reads it with
  if (p_drop > 0.f && Lq > 2 * SQ &&
      !bits_check(keep_bits, use_sf16(dh, (int64_t)B * H, Lq, Lk) ? kBitsSf16 : kBitsValu, B, H, Lq, Lk))
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
  fill_common(a, B, H, Lq, Lk, dh, p_drop, rng_state, call_id);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return launch_bwd<8>(a, p_drop, part, workspace, s);
  return launch_bwd<16>(a, p_drop, part, workspace, s);
}
}  // namespace

#define VAESNE_ATTN_BWD_PARAMS                                                                  \
  const float *q, int64_t q_bs, int64_t q_ls, const float *k, int64_t k_bs, int64_t k_ls,      \
      const float *v, int64_t v_bs, int64_t v_ls, const float *kbias, int64_t kb_bs,          \
      const float *o, int64_t o_bs, int64_t o_ls, const float *lse, const float *dout,        \
      int64_t do_bs, int64_t do_ls, float *dq, int64_t dq_bs, int64_t dq_ls, float *dk,       \
      int64_t dk_bs, int64_t dk_ls, float *dv, int64_t dv_bs, int64_t dv_ls, int B, int H,    \
      int Lq, int Lk, int dh, float p_drop, const int64_t *rng_state, uint32_t call_id,       \
      const uint32_t *keep_bits, float *workspace
#define VAESNE_ATTN_BWD_ARGS                                                                    \
  q, q_bs, q_ls, k, k_bs, k_ls, v, v_bs, v_ls, kbias, kb_bs, o, o_bs, o_ls, lse, dout, do_bs,  \
      do_ls, dq, dq_bs, dq_ls, dk, dk_bs, dk_ls, dv, dv_bs, dv_ls, B, H, Lq, Lk, dh, p_drop,   \
      rng_state, call_id, keep_bits, workspace

VAESNE_API int vaesne_attn_bwd(VAESNE_ATTN_BWD_PARAMS, void* stream) {
  return attn_bwd_impl(VAESNE_ATTN_BWD_ARGS, 3, stream);
}
VAESNE_API int vaesne_attn_bwd_kv(VAESNE_ATTN_BWD_PARAMS, void* stream) {
  return attn_bwd_impl(VAESNE_ATTN_BWD_ARGS, 1, stream);
}
VAESNE_API int vaesne_attn_bwd_q(VAESNE_ATTN_BWD_PARAMS, void* stream) {
  return attn_bwd_impl(VAESNE_ATTN_BWD_ARGS, 2, stream);
}
