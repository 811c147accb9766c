// Masked multi-head attention core for VAESNe (head_dim 8; 16 also built):
// the arithmetic of torch.nn.MultiheadAttention's slow path as the reference
// calls it (util_layers.py:289,297,301 -> torch/nn/functional.py:6559-6594):
//     S = (q / sqrt(dh)) k^T ;  S[:, j] = -inf where key_padding_mask[j]
//     P = softmax(S) ;  A = Dropout_p(P) ;  O = A v
// The score matrix never touches HBM (flash-style online softmax).  Scores are
// kept in the log2 domain (q pre-multiplied by log2(e)/sqrt(dh)) so every
// exponential is one v_exp_f32.  lse is saved per (batch, head, query) for the
// backward, which recomputes P.
//
// Layout: q/k/v/o are row-major token matrices with a per-batch stride and a
// per-row stride (e.g. the packed in-projection output [B, L, 3E] is read in
// place); head h owns columns [h*dh, (h+1)*dh).  kpm is [B, Lk] uint8
// (1 = ignore the key), or null.
//
// Kernels (all fp32, VALU; one query / key per lane, K/V or Q/dO tiles staged
// through LDS and read as broadcast float4s):
//   attn_fwd     : grid (B*H*query-blocks); QPT queries per lane.
//   attn_bwd_pre : D = rowsum(dO * O) per (b, h, q)  (valid with dropout:
//                  sum_j P_ij dP_ij = dO_i . O_i).
//   attn_bwd_kv  : key-parallel, two adjacent keys per lane: dK, dV.
//   attn_bwd_q   : query-parallel: dQ.
// Dropout: one 32-bit hash per (row, key pair) gives the two 16-bit keep
// draws; fwd, bwd_kv and bwd_q regenerate identical masks.
#include "common.h"

using namespace vaesne;

namespace {

constexpr int NT = 256;
constexpr int TK = 64;   // keys per LDS tile (fwd / dq)
constexpr int TQ = 64;   // queries per LDS tile (dkv)
constexpr int CH = 16;   // keys per online-softmax update

struct AttnArgs {
  const float* q; int64_t q_bs, q_ls;
  const float* k; int64_t k_bs, k_ls;
  const float* v; int64_t v_bs, v_ls;
  const uint8_t* kpm; int64_t m_bs;
  const float* o; int64_t o_bs, o_ls;      // fwd output / bwd input
  float* o_out;                            // fwd output pointer (same strides as o)
  float* lse;                              // [B, H, Lq] log2 domain
  const float* dout; int64_t do_bs, do_ls;
  float* D;                                // [B, H, Lq]
  float* dq; int64_t dq_bs, dq_ls;
  float* dk; int64_t dk_bs, dk_ls;
  float* dv; int64_t dv_bs, dv_ls;
  int B, H, Lq, Lk;
  float scale;        // 1/sqrt(dh)
  float scale_log2;   // log2(e)/sqrt(dh)
  float p_drop; uint32_t thr; float inv_keep;
  const int64_t* rng_state; uint32_t call_id;
};

template <int DH>
__device__ __forceinline__ void ld(const float* __restrict__ p, float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 t = *reinterpret_cast<const float4*>(p + d);
    r[d] = t.x; r[d + 1] = t.y; r[d + 2] = t.z; r[d + 3] = t.w;
  }
}
template <int DH>
__device__ __forceinline__ void st(float* __restrict__ p, const float (&r)[DH]) {
#pragma unroll
  for (int d = 0; d < DH; d += 4)
    *reinterpret_cast<float4*>(p + d) = make_float4(r[d], r[d + 1], r[d + 2], r[d + 3]);
}
template <int DH>
__device__ __forceinline__ float dot(const float (&a)[DH], const float* __restrict__ b) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 t = *reinterpret_cast<const float4*>(b + d);
    s = fmaf(a[d], t.x, s);
    s = fmaf(a[d + 1], t.y, s);
    s = fmaf(a[d + 2], t.z, s);
    s = fmaf(a[d + 3], t.w, s);
  }
  return s;
}
template <int DH>
__device__ __forceinline__ void axpy(float (&y)[DH], float a, const float* __restrict__ x) {
#pragma unroll
  for (int d = 0; d < DH; d += 4) {
    float4 t = *reinterpret_cast<const float4*>(x + d);
    y[d] = fmaf(a, t.x, y[d]);
    y[d + 1] = fmaf(a, t.y, y[d + 1]);
    y[d + 2] = fmaf(a, t.z, y[d + 2]);
    y[d + 3] = fmaf(a, t.w, y[d + 3]);
  }
}

// cooperative load of one key tile: Ks/Vs [TK][DH], Mb [TK] (0 or -inf)
template <int DH>
__device__ __forceinline__ void load_kv_tile(const AttnArgs& a, int b, int h, int kt, float* Ks,
                                             float* Vs, float* Mb) {
  constexpr int V4 = DH / 4;
  for (int idx = threadIdx.x; idx < TK * V4 * 2; idx += NT) {
    int kk = idx / (2 * V4);
    int part = idx - kk * 2 * V4;
    int key = kt + kk;
    float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
    bool isv = part >= V4;
    int c = (isv ? part - V4 : part) * 4;
    if (key < a.Lk) {
      const float* src = isv ? a.v + (int64_t)b * a.v_bs + (int64_t)key * a.v_ls + h * DH + c
                             : a.k + (int64_t)b * a.k_bs + (int64_t)key * a.k_ls + h * DH + c;
      val = *reinterpret_cast<const float4*>(src);
    }
    *reinterpret_cast<float4*>((isv ? Vs : Ks) + kk * DH + c) = val;
  }
  if (threadIdx.x < TK) {
    int key = kt + threadIdx.x;
    bool ok = key < a.Lk && !(a.kpm && a.kpm[(int64_t)b * a.m_bs + key]);
    Mb[threadIdx.x] = ok ? 0.f : -INFINITY;
  }
}

template <int DH, int QPT, bool DROP>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ float Mb[TK];
  const int nqb = (a.Lq + NT * QPT - 1) / (NT * QPT);
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;

  float q[QPT][DH], o[QPT][DH], m[QPT], l[QPT];
  uint32_t rkey[QPT];
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    int qi = qb * NT * QPT + j * NT + threadIdx.x;
    int qc = qi < a.Lq ? qi : a.Lq - 1;
    ld<DH>(a.q + (int64_t)b * a.q_bs + (int64_t)qc * a.q_ls + h * DH, q[j]);
#pragma unroll
    for (int d = 0; d < DH; ++d) { q[j][d] *= a.scale_log2; o[j][d] = 0.f; }
    m[j] = -INFINITY;
    l[j] = 0.f;
    rkey[j] = DROP ? attn_row_key(skey, (uint32_t)((int64_t)bh * a.Lq + qc)) : 0u;
  }

  for (int kt = 0; kt < a.Lk; kt += TK) {
    __syncthreads();
    load_kv_tile<DH>(a, b, h, kt, Ks, Vs, Mb);
    __syncthreads();
    const int kend = min(TK, a.Lk - kt);
    for (int c0 = 0; c0 < kend; c0 += CH) {
#pragma unroll
      for (int j = 0; j < QPT; ++j) {
        float s[CH];
        float cm = -INFINITY;
#pragma unroll
        for (int kk = 0; kk < CH; ++kk) {
          s[kk] = Mb[c0 + kk] + dot<DH>(q[j], Ks + (c0 + kk) * DH);
          cm = fmaxf(cm, s[kk]);
        }
        const float mn = fmaxf(m[j], cm);
        const float mu = mn == -INFINITY ? 0.f : mn;
        const float corr = exp2f(m[j] - mu);
        m[j] = mn;
        l[j] *= corr;
#pragma unroll
        for (int d = 0; d < DH; ++d) o[j][d] *= corr;
#pragma unroll
        for (int kk = 0; kk < CH; kk += 2) {
          float p0 = exp2f(s[kk] - mu);
          float p1 = exp2f(s[kk + 1] - mu);
          l[j] += p0 + p1;
          if (DROP) {
            uint32_t bits = attn_pair_bits(rkey[j], (uint32_t)((kt + c0 + kk) >> 1));
            p0 = (bits & 0xffffu) >= a.thr ? p0 : 0.f;
            p1 = (bits >> 16) >= a.thr ? p1 : 0.f;
          }
          axpy<DH>(o[j], p0, Vs + (c0 + kk) * DH);
          axpy<DH>(o[j], p1, Vs + (c0 + kk + 1) * DH);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    int qi = qb * NT * QPT + j * NT + threadIdx.x;
    if (qi >= a.Lq) continue;
    const float inv = (DROP ? a.inv_keep : 1.f) / l[j];  // l == 0 (all keys masked) -> NaN, as the reference
#pragma unroll
    for (int d = 0; d < DH; ++d) o[j][d] *= inv;
    st<DH>(a.o_out + (int64_t)b * a.o_bs + (int64_t)qi * a.o_ls + h * DH, o[j]);
    a.lse[(int64_t)bh * a.Lq + qi] = m[j] + __log2f(l[j]);
  }
}

template <int DH>
__global__ __launch_bounds__(NT) void attn_bwd_pre_kernel(AttnArgs a) {
  int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x;
  int64_t total = (int64_t)a.B * a.H * a.Lq;
  if (t >= total) return;
  int qi = (int)(t % a.Lq);
  int64_t bh = t / a.Lq;
  int b = (int)(bh / a.H), h = (int)(bh - (int64_t)b * a.H);
  float x[DH], y[DH];
  ld<DH>(a.o + (int64_t)b * a.o_bs + (int64_t)qi * a.o_ls + h * DH, x);
  ld<DH>(a.dout + (int64_t)b * a.do_bs + (int64_t)qi * a.do_ls + h * DH, y);
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < DH; ++d) s = fmaf(x[d], y[d], s);
  a.D[t] = s;
}

// key-parallel backward: lane owns keys 2*tid, 2*tid+1 of a 512-key block
template <int DH, bool DROP>
__global__ __launch_bounds__(NT) void attn_bwd_kv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Qs[TQ * DH];
  __shared__ __attribute__((aligned(16))) float Os[TQ * DH];  // dO tile
  __shared__ float Ls[TQ], Ds[TQ];
  __shared__ uint32_t Rk[TQ];
  constexpr int KB = 2 * NT;
  const int nkb = (a.Lk + KB - 1) / KB;
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb;
  const int b = bh / a.H, h = bh - b * a.H;
  const int key0 = kb * KB + 2 * threadIdx.x;
  const uint32_t kp = (uint32_t)(key0 >> 1);
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;

  float kr[2][DH], vr[2][DH], dk[2][DH], dv[2][DH];
  bool valid[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    int key = key0 + u;
    valid[u] = key < a.Lk && !(a.kpm && a.kpm[(int64_t)b * a.m_bs + key]);
    int kc = key < a.Lk ? key : a.Lk - 1;
    ld<DH>(a.k + (int64_t)b * a.k_bs + (int64_t)kc * a.k_ls + h * DH, kr[u]);
    ld<DH>(a.v + (int64_t)b * a.v_bs + (int64_t)kc * a.v_ls + h * DH, vr[u]);
#pragma unroll
    for (int d = 0; d < DH; ++d) { dk[u][d] = 0.f; dv[u][d] = 0.f; }
  }
  const bool any_valid = valid[0] || valid[1];

  for (int qt = 0; qt < a.Lq; qt += TQ) {
    __syncthreads();
    constexpr int V4 = DH / 4;
    for (int idx = threadIdx.x; idx < TQ * V4 * 2; idx += NT) {
      int qq = idx / (2 * V4);
      int part = idx - qq * 2 * V4;
      int qi = qt + qq;
      bool isd = part >= V4;
      int c = (isd ? part - V4 : part) * 4;
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if (qi < a.Lq) {
        if (isd) {
          val = *reinterpret_cast<const float4*>(a.dout + (int64_t)b * a.do_bs +
                                                 (int64_t)qi * a.do_ls + h * DH + c);
        } else {
          val = *reinterpret_cast<const float4*>(a.q + (int64_t)b * a.q_bs + (int64_t)qi * a.q_ls +
                                                 h * DH + c);
          val.x *= a.scale_log2; val.y *= a.scale_log2; val.z *= a.scale_log2; val.w *= a.scale_log2;
        }
      }
      *reinterpret_cast<float4*>((isd ? Os : Qs) + qq * DH + c) = val;
    }
    if (threadIdx.x < TQ) {
      int qi = qt + threadIdx.x;
      bool ok = qi < a.Lq;
      int64_t row = (int64_t)bh * a.Lq + qi;
      Ls[threadIdx.x] = ok ? a.lse[row] : INFINITY;
      Ds[threadIdx.x] = ok ? a.D[row] : 0.f;
      Rk[threadIdx.x] = DROP ? attn_row_key(skey, (uint32_t)row) : 0u;
    }
    __syncthreads();
    if (!any_valid) continue;
    const int qend = min(TQ, a.Lq - qt);
    for (int i = 0; i < qend; ++i) {
      float qv[DH], dov[DH];
#pragma unroll
      for (int d = 0; d < DH; d += 4) {
        float4 t = *reinterpret_cast<const float4*>(Qs + i * DH + d);
        qv[d] = t.x; qv[d + 1] = t.y; qv[d + 2] = t.z; qv[d + 3] = t.w;
        float4 w = *reinterpret_cast<const float4*>(Os + i * DH + d);
        dov[d] = w.x; dov[d + 1] = w.y; dov[d + 2] = w.z; dov[d + 3] = w.w;
      }
      const float li = Ls[i], Di = Ds[i];
      uint32_t bits = DROP ? attn_pair_bits(Rk[i], kp) : 0u;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float s = 0.f, dA = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          s = fmaf(qv[d], kr[u][d], s);
          dA = fmaf(dov[d], vr[u][d], dA);
        }
        float p = valid[u] ? exp2f(s - li) : 0.f;
        float aP = p, dP = dA;
        if (DROP) {
          bool keep = ((u == 0 ? (bits & 0xffffu) : (bits >> 16)) >= a.thr);
          aP = keep ? p * a.inv_keep : 0.f;
          dP = keep ? dA * a.inv_keep : 0.f;
        }
        float dS = p * (dP - Di);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          dv[u][d] = fmaf(aP, dov[d], dv[u][d]);
          dk[u][d] = fmaf(dS, qv[d], dk[u][d]);
        }
      }
    }
  }
  // dK = sum_i dS_i * q_i * scale = (scale / scale_log2) * sum_i dS_i * Qs_i
  const float kfac = a.scale / a.scale_log2;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    int key = key0 + u;
    if (key >= a.Lk) continue;
#pragma unroll
    for (int d = 0; d < DH; ++d) dk[u][d] *= kfac;
    st<DH>(a.dk + (int64_t)b * a.dk_bs + (int64_t)key * a.dk_ls + h * DH, dk[u]);
    st<DH>(a.dv + (int64_t)b * a.dv_bs + (int64_t)key * a.dv_ls + h * DH, dv[u]);
  }
}

template <int DH, int QPT, bool DROP>
__global__ __launch_bounds__(NT) void attn_bwd_q_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) float Ks[TK * DH];
  __shared__ __attribute__((aligned(16))) float Vs[TK * DH];
  __shared__ float Mb[TK];
  const int nqb = (a.Lq + NT * QPT - 1) / (NT * QPT);
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / a.H, h = bh - b * a.H;
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;

  float q[QPT][DH], dov[QPT][DH], dq[QPT][DH], lse[QPT], Dv[QPT];
  uint32_t rkey[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    int qi = qb * NT * QPT + j * NT + threadIdx.x;
    int qc = qi < a.Lq ? qi : a.Lq - 1;
    int64_t row = (int64_t)bh * a.Lq + qc;
    ld<DH>(a.q + (int64_t)b * a.q_bs + (int64_t)qc * a.q_ls + h * DH, q[j]);
    ld<DH>(a.dout + (int64_t)b * a.do_bs + (int64_t)qc * a.do_ls + h * DH, dov[j]);
#pragma unroll
    for (int d = 0; d < DH; ++d) { q[j][d] *= a.scale_log2; dq[j][d] = 0.f; }
    lse[j] = a.lse[row];
    Dv[j] = a.D[row];
    rkey[j] = DROP ? attn_row_key(skey, (uint32_t)row) : 0u;
  }
  for (int kt = 0; kt < a.Lk; kt += TK) {
    __syncthreads();
    load_kv_tile<DH>(a, b, h, kt, Ks, Vs, Mb);
    __syncthreads();
    const int kend = min(TK, a.Lk - kt);
    for (int kk = 0; kk < kend; kk += 2) {
#pragma unroll
      for (int j = 0; j < QPT; ++j) {
        uint32_t bits = DROP ? attn_pair_bits(rkey[j], (uint32_t)((kt + kk) >> 1)) : 0u;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float* kp = Ks + (kk + u) * DH;
          const float* vp = Vs + (kk + u) * DH;
          float s = Mb[kk + u] + dot<DH>(q[j], kp);
          float dA = dot<DH>(dov[j], vp);
          float p = exp2f(s - lse[j]);
          float dP = dA;
          if (DROP) {
            bool keep = ((u == 0 ? (bits & 0xffffu) : (bits >> 16)) >= a.thr);
            dP = keep ? dA * a.inv_keep : 0.f;
          }
          float dS = p * (dP - Dv[j]);
          axpy<DH>(dq[j], dS, kp);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    int qi = qb * NT * QPT + j * NT + threadIdx.x;
    if (qi >= a.Lq) continue;
#pragma unroll
    for (int d = 0; d < DH; ++d) dq[j][d] *= a.scale;
    st<DH>(a.dq + (int64_t)b * a.dq_bs + (int64_t)qi * a.dq_ls + h * DH, dq[j]);
  }
}

bool aligned16(const void* p, int64_t ls) {
  return ((uintptr_t)p % 16 == 0) && (ls % 4 == 0);
}

template <int DH>
int fwd_dh(AttnArgs& a, hipStream_t s) {
  constexpr int QPT = 2;
  int nqb = (a.Lq + NT * QPT - 1) / (NT * QPT);
  dim3 grid((unsigned)((int64_t)a.B * a.H * nqb));
  if (a.p_drop > 0.f)
    hipLaunchKernelGGL((attn_fwd_kernel<DH, QPT, true>), grid, dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<DH, QPT, false>), grid, dim3(NT), 0, s, a);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

template <int DH>
int bwd_dh(AttnArgs& a, hipStream_t s) {
  int64_t rows = (int64_t)a.B * a.H * a.Lq;
  hipLaunchKernelGGL((attn_bwd_pre_kernel<DH>), dim3((unsigned)((rows + NT - 1) / NT)), dim3(NT),
                     0, s, a);
  VAESNE_CHECK_LAUNCH();
  const int nkb = (a.Lk + 2 * NT - 1) / (2 * NT);
  dim3 gkv((unsigned)((int64_t)a.B * a.H * nkb));
  constexpr int QPT = 1;
  const int nqb = (a.Lq + NT * QPT - 1) / (NT * QPT);
  dim3 gq((unsigned)((int64_t)a.B * a.H * nqb));
  if (a.p_drop > 0.f) {
    hipLaunchKernelGGL((attn_bwd_kv_kernel<DH, true>), gkv, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_q_kernel<DH, QPT, true>), gq, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_kv_kernel<DH, false>), gkv, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_q_kernel<DH, QPT, false>), gq, dim3(NT), 0, s, a);
  }
  VAESNE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

VAESNE_API int vaesne_attn_fwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const uint8_t* kpm, int64_t m_bs, float* o,
                               int64_t o_bs, int64_t o_ls, float* lse, int B, int H, int Lq,
                               int Lk, int dh, float p_drop, const int64_t* rng_state,
                               uint32_t call_id, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls))
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.q_bs = q_bs; a.q_ls = q_ls;
  a.k = k; a.k_bs = k_bs; a.k_ls = k_ls;
  a.v = v; a.v_bs = v_bs; a.v_ls = v_ls;
  a.kpm = kpm; a.m_bs = m_bs;
  a.o = o; a.o_out = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = lse;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.scale = 1.0f / sqrtf((float)dh);
  a.scale_log2 = a.scale * 1.4426950408889634f;
  a.p_drop = p_drop; a.thr = drop_thr16(p_drop);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.rng_state = rng_state; a.call_id = call_id;
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return fwd_dh<8>(a, s);
  if (dh == 16) return fwd_dh<16>(a, s);
  return (int)hipErrorInvalidValue;
}

VAESNE_API int64_t vaesne_attn_bwd_workspace(int B, int H, int Lq) {
  return (int64_t)B * H * Lq * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_attn_bwd(const float* q, int64_t q_bs, int64_t q_ls, const float* k,
                               int64_t k_bs, int64_t k_ls, const float* v, int64_t v_bs,
                               int64_t v_ls, const uint8_t* kpm, int64_t m_bs, const float* o,
                               int64_t o_bs, int64_t o_ls, const float* lse, const float* dout,
                               int64_t do_bs, int64_t do_ls, float* dq, int64_t dq_bs,
                               int64_t dq_ls, float* dk, int64_t dk_bs, int64_t dk_ls, float* dv,
                               int64_t dv_bs, int64_t dv_ls, int B, int H, int Lq, int Lk, int dh,
                               float p_drop, const int64_t* rng_state, uint32_t call_id,
                               float* workspace, void* stream) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0) return (int)hipErrorInvalidValue;
  if (!aligned16(q, q_ls) || !aligned16(k, k_ls) || !aligned16(v, v_ls) || !aligned16(o, o_ls) ||
      !aligned16(dout, do_ls) || !aligned16(dq, dq_ls) || !aligned16(dk, dk_ls) ||
      !aligned16(dv, dv_ls))
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.q = q; a.q_bs = q_bs; a.q_ls = q_ls;
  a.k = k; a.k_bs = k_bs; a.k_ls = k_ls;
  a.v = v; a.v_bs = v_bs; a.v_ls = v_ls;
  a.kpm = kpm; a.m_bs = m_bs;
  a.o = o; a.o_bs = o_bs; a.o_ls = o_ls;
  a.lse = const_cast<float*>(lse);
  a.dout = dout; a.do_bs = do_bs; a.do_ls = do_ls;
  a.D = workspace;
  a.dq = dq; a.dq_bs = dq_bs; a.dq_ls = dq_ls;
  a.dk = dk; a.dk_bs = dk_bs; a.dk_ls = dk_ls;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_ls = dv_ls;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.scale = 1.0f / sqrtf((float)dh);
  a.scale_log2 = a.scale * 1.4426950408889634f;
  a.p_drop = p_drop; a.thr = drop_thr16(p_drop);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.rng_state = rng_state; a.call_id = call_id;
  hipStream_t s = (hipStream_t)stream;
  if (dh == 8) return bwd_dh<8>(a, s);
  if (dh == 16) return bwd_dh<16>(a, s);
  return (int)hipErrorInvalidValue;
}
