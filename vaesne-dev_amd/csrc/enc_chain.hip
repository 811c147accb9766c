// Fused latent-token chain of the VAESNe encoders: every TransformerBlock of
// photometricTransformerEncoder / spectraTransformerEncoder
// (PhotometricLayers.py:141-142, SpectraLayers.py:135-136 -> util_layers.py:285-309)
// on the T learned bottleneck tokens, with the data tokens as cross-attention context:
//
//   qkv = x Wi^T + bi;   O = Drop(softmax(q k^T / sqrt(8))) v      (T x T, 4 heads)
//   x1  = LN1(x + Drop(O Wo1^T + bo1));   q = x1 Wq^T + bq          (Wq = in_proj rows [0, 32))
//   c   = Drop(softmax(q k_ctx^T / sqrt(8) + kbias)) v_ctx           (T x Lk, 4 heads)
//   x2  = LN2(x1 + Drop(c Wo2^T + bo2))
//   y   = LN3(x2 + Drop(W2 gelu(W1 x2 + b1) + b2))
//
// for all nb blocks in ONE launch (forward) and ONE launch (backward).  The chain
// of one sequence is T = 8 tokens x 32 features: one workgroup per sequence,
// thread (token, feature), weights staged per block in LDS, cross-token sums
// through LDS, per-token sums through DPP / permlane half-wave reductions.  The
// context's k | v projections (in_proj rows [32, 96)) are wide token-wise GEMMs
// over B * Lk tokens: the caller runs them (vaesne_linear_*) before the forward
// and after the backward; this backward writes d(k|v) per sequence.
// blockIdx.y selects one of up to two GROUPS (the photometry and the spectra
// encoder: one launch covers both chains, which a captured graph would otherwise
// run one after the other).
//
// Numerics and dropout streams are those of the per-op path (vaesne_attn_fwd's
// few-query kernel, vaesne_enc_block PRE / POST): the same counter hashes on the
// same (call id, row, element) coordinates, so with the same call ids the keep
// masks are bit-identical and results agree to fp32 rounding.
//
// Backward: the forward saves every activation of the chain (~15 KB per block and
// sequence); the backward runs the blocks in reverse, re-hashes the keep masks and
// writes per-sequence weight-gradient partials [B][nb * PBLK] (fixed-order column
// sums over B, now or deferred: bitwise reproducible, no atomics).
#include "common.h"

using namespace vaesne;

namespace {

constexpr int E = 32, H = 4, DH = 8, E3 = 96, NT = 512, TMAX = 8, LP = 33;
// thread layout: wave w (8) = token w of the sequence in the per-token phases; lane l:
// feature f = l & 31, half hf = l >> 5 (the halves split every dot product and combine
// with one permlane32 swap, so both halves hold the token's 32 features)
constexpr int NSL = 16;       // key slices of the cross-attention forward (32 query-heads x 16)
constexpr int KTF = 128;      // keys per tile, cross-attention forward
constexpr int KTB = 128;      // keys per tile, cross-attention backward (128 keys x 4 heads)
constexpr int DSP = KTB + 1;  // dS row pitch
constexpr int GMAX = 2;

// saved activations, per (sequence, block), floats; rows [TMAX][...]
constexpr int S_XIN = 0, S_QKV = 256, S_PN = 1024, S_O = 1280, S_XH1 = 1536, S_RS1 = 1792,
              S_X1 = 1800, S_QS = 2056, S_C = 2312, S_LSE = 2568, S_XH2 = 2600, S_RS2 = 2856,
              S_X2 = 2864, S_H1 = 3120, S_XH3 = 3376, S_RS3 = 3632, SAVE_BLK = 3648;

// per-block gradient layout (partials and gflat alike), the 18 tensors in order
constexpr int O_WI = 0, O_BI = 3072, O_WO1 = 3168, O_BO1 = 4192, O_G1 = 4224, O_BE1 = 4256,
              O_WC = 4288, O_BC = 7360, O_WO2 = 7456, O_BO2 = 8480, O_G2 = 8512, O_BE2 = 8544,
              O_W1 = 8576, O_B1 = 9600, O_W2 = 9632, O_B2 = 10656, O_G3 = 10688, O_BE3 = 10720,
              PBLK = 10752;
enum WIdx { W_I = 0, B_I, W_O1, B_O1, G_1, BE_1, W_C, B_C, W_O2, B_O2, G_2, BE_2, W_1, B_1,
            W_2, B_2, G_3, BE_3 };

#ifdef VAESNE_CHAIN_PROFILE
// per-phase timestamps (tools/chain_phases.py): [fwd/bwd][group][sequence][block][mark]
__device__ unsigned long long g_chain_prof[2][GMAX][64][VAESNE_ENC_CHAIN_MAXB][8];
#define PT(dir, k)                                                                    \
  do {                                                                                \
    if (threadIdx.x == 0 && b < 64) g_chain_prof[dir][blockIdx.y][b][blk][k] = wall_clock64(); \
  } while (0)
#else
#define PT(dir, k) \
  do {             \
  } while (0)
#endif

struct Grp {
  vaesne_enc_chain_group d;
  uint32_t thr_sa, thr_res, thr_ca;
  float ik_sa, ik_res, ik_ca;
  float scale, scale_log2, kf;   // 1/sqrt(dh), its log2(e) multiple, scale / scale_log2
};
struct Args {
  Grp g[GMAX];
};

struct __attribute__((aligned(16))) Wts {
  float Wi[E3 * LP], Wo1[E * LP], Wq[E * LP], Wo2[E * LP], W1[E * LP], W2[E * LP];
  float bi[E3], bo1[E], g1[E], be1[E], bq[E], bo2[E], g2[E], be2[E], b1[E], b2[E], g3[E], be3[E];
};

// a block's weights into LDS (matrices at pitch LP): every global load is issued
// before the first LDS store, so the staging costs one memory latency
// (parameters may be views into an unpadded flat buffer: scalar loads, coalesced)
__device__ __forceinline__ void stage(Wts& w, const float* const* p) {
  const int t = threadIdx.x;
  constexpr int NR = (3 * E * E + 5 * E * E) / NT;     // 16 matrix floats per thread
  float m[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = t + r * NT;                           // over [Wi | Wo1 | Wq | Wo2 | W1 | W2]
    const int mi = i < 3 * E * E ? 0 : 1 + ((i - 3 * E * E) >> 10);
    const int o = i < 3 * E * E ? i : (i - 3 * E * E) & 1023;
    const float* src = mi == 0 ? p[W_I] : mi == 1 ? p[W_O1] : mi == 2 ? p[W_C]
                     : mi == 3 ? p[W_O2] : mi == 4 ? p[W_1] : p[W_2];
    m[r] = src[o];
  }
  // vectors: bi [96] then 11 x [32] (bo1 g1 be1 bq bo2 g2 be2 b1 b2 g3 be3)
  const int vid[11] = {B_O1, G_1, BE_1, B_C, B_O2, G_2, BE_2, B_1, B_2, G_3, BE_3};
  float v = 0.f;
  if (t < 3 * E) v = p[B_I][t];
  else if (t < 3 * E + 11 * E) v = p[vid[(t - 3 * E) >> 5]][(t - 3 * E) & 31];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = t + r * NT;
    const int mi = i < 3 * E * E ? 0 : 1 + ((i - 3 * E * E) >> 10);
    const int o = i < 3 * E * E ? i : (i - 3 * E * E) & 1023;
    float* dst = mi == 0 ? w.Wi : mi == 1 ? w.Wo1 : mi == 2 ? w.Wq : mi == 3 ? w.Wo2
               : mi == 4 ? w.W1 : w.W2;
    dst[(o >> 5) * LP + (o & 31)] = m[r];
  }
  float* vd[12] = {w.bi, w.bo1, w.g1, w.be1, w.bq, w.bo2, w.g2, w.be2, w.b1, w.b2, w.g3, w.be3};
  if (t < 3 * E) vd[0][t] = v;
  else if (t < 3 * E + 11 * E) vd[1 + ((t - 3 * E) >> 5)][(t - 3 * E) & 31] = v;
}

// this half's share of sum_k W[o][k] x[k] (k in [16 hf, 16 hf + 16)), both halves
// combined: W in LDS (pitch LP), x an LDS row (broadcast reads); two accumulators
__device__ __forceinline__ float dot_row(const float* W, int o, const float* x, int hf) {
  const float* wr = W + o * LP + 16 * hf;
  const float* xr = x + 16 * hf;
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; k += 8) {
    const float4 x0 = *reinterpret_cast<const float4*>(xr + k);
    const float4 x1 = *reinterpret_cast<const float4*>(xr + k + 4);
    a0 = fmaf(wr[k], x0.x, a0); a1 = fmaf(wr[k + 1], x0.y, a1);
    a0 = fmaf(wr[k + 2], x0.z, a0); a1 = fmaf(wr[k + 3], x0.w, a1);
    a0 = fmaf(wr[k + 4], x1.x, a0); a1 = fmaf(wr[k + 5], x1.y, a1);
    a0 = fmaf(wr[k + 6], x1.z, a0); a1 = fmaf(wr[k + 7], x1.w, a1);
  }
  return xsum32(a0 + a1);
}
// sum_o W[o][k] g[o] over N outputs (backward data), split over the halves likewise
template <int N>
__device__ __forceinline__ float dot_col(const float* W, int k, const float* g, int hf) {
  constexpr int NH = N / 2;
  const float* gr = g + NH * hf;
  const float* wc = W + NH * hf * LP + k;
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int o = 0; o < NH; o += 4) {
    const float4 gv = *reinterpret_cast<const float4*>(gr + o);
    a0 = fmaf(wc[o * LP], gv.x, a0);
    a1 = fmaf(wc[(o + 1) * LP], gv.y, a1);
    a0 = fmaf(wc[(o + 2) * LP], gv.z, a0);
    a1 = fmaf(wc[(o + 3) * LP], gv.w, a1);
  }
  return xsum32(a0 + a1);
}

// sum over the 32 lanes of a half-wave (one token's features): DPP within each
// 16-lane row, then the row pair (lane ^ 16)
__device__ __forceinline__ float hsum32(float v) {
  v += dpp_mov<0x128>(v);   // row_ror 8
  v += dpp_mov<0x124>(v);   // row_ror 4
  v += dpp_mov<0x4e>(v);    // quad xor 2
  v += dpp_mov<0xb1>(v);    // quad xor 1
  return xsum16(v);
}
// sum / max over aligned groups of 8 lanes: quad xor 1, 2, then the half-row mirror
__device__ __forceinline__ float gsum8(float v) {
  v += dpp_mov<0xb1>(v);
  v += dpp_mov<0x4e>(v);
  return v + dpp_mov<0x141>(v);
}
__device__ __forceinline__ float gmax8(float v) {
  v = fmaxf(v, dpp_mov<0xb1>(v));
  v = fmaxf(v, dpp_mov<0x4e>(v));
  return fmaxf(v, dpp_mov<0x141>(v));
}

// LayerNorm of one token (the lane's feature v); returns x_hat, sets rstd
__device__ __forceinline__ float ln_fwd(float v, float& rstd) {
  const float mu = hsum32(v) * (1.f / E);
  const float d = v - mu;
  rstd = rsqrtf(hsum32(d * d) * (1.f / E) + 1e-5f);
  return d * rstd;
}
// d(LN input) from d(LN output) g
__device__ __forceinline__ float ln_bwd(float g, float xh, float gamma, float rstd) {
  const float gg = g * gamma;
  const float a = hsum32(gg) * (1.f / E);
  const float b = hsum32(gg * xh) * (1.f / E);
  return rstd * (gg - a - xh * b);
}

__device__ __forceinline__ uint32_t site_key(uint32_t key, uint32_t site) {
  return mix32(key ^ (0x632be5abu * (site + 1)));   // = decoder_block.hip site_key
}
// residual-dropout keep decision of element (row, f) at a site
__device__ __forceinline__ bool res_keep(uint32_t skey, int64_t row, int f, uint32_t thr) {
  return (rand_u32(skey, (uint64_t)row * E + f) & 0xffffu) >= thr;
}
// attention-probability keep decision (= attention.hip keep_of)
__device__ __forceinline__ bool attn_keep(uint32_t rk, int j, uint32_t thr) {
  const uint32_t bits = attn_pair_bits(rk, (uint32_t)(j >> 1));
  return ((j & 1) ? (bits >> 16) : (bits & 0xffffu)) >= thr;
}

__device__ __forceinline__ float ex2f_(float x) { return __builtin_amdgcn_exp2f(x); }

// ============================== forward ====================================
struct __attribute__((aligned(16))) FwdSmem {
  Wts w;
  float X[TMAX * E], QKV[TMAX * E3], PD[H * TMAX * TMAX], O[TMAX * E], X1[TMAX * E],
      QS[TMAX * E], C[TMAX * E], X2[TMAX * E], GL[TMAX * E];
  float red[NSL][32][10];
  float Kt[KTF * E], Vt[KTF * E], Kb[KTF];
};

__global__ __launch_bounds__(NT) void enc_chain_fwd_kernel(Args args) {
  __shared__ FwdSmem S;
  const Grp& G = args.g[blockIdx.y];
  const vaesne_enc_chain_group& a = G.d;
  const int b = blockIdx.x;
  if (b >= a.B) return;
  const int tid = threadIdx.x, tok = tid >> 6, lane = tid & 63, f = lane & 31, hf = lane >> 5;
  const int T = a.T;
  const bool act = tok < T;
  const bool wr = act && hf == 0;              // the lane that stores the token's feature f
  const int tf = tok * E + f;                  // (token, feature) index of [TMAX][E] rows
  const int64_t row = (int64_t)b * T + (act ? tok : T - 1);
  if (hf == 0) S.X[tf] = act ? a.x0[((int64_t)b * T + tok) * E + f] : 0.f;
  for (int blk = 0; blk < a.nb; ++blk) {
    float* sv = a.save + ((int64_t)b * a.nb + blk) * SAVE_BLK;
    __syncthreads();
    PT(0, 0);
    stage(S.w, a.w[blk]);
    __syncthreads();
    PT(0, 1);
    const float xin = S.X[tf];
    if (wr) sv[S_XIN + tf] = xin;
    // ---- self-attention in-projection
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int o = c * E + f;
      const float v = S.w.bi[o] + dot_row(S.w.Wi, o, S.X + tok * E, hf);
      if (hf == 0) S.QKV[tok * E3 + o] = v;
      if (wr) sv[S_QKV + tok * E3 + o] = v;
    }
    __syncthreads();
    PT(0, 2);
    // ---- self-attention over the T tokens: lane (query tok, head h, key j)
    {
      const int h = (lane >> 3) & 3, j = lane & 7;
      const bool valid = act && j < T;
      float s = -INFINITY;
      if (valid) {
        s = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d)
          s = fmaf(S.QKV[tok * E3 + h * DH + d] * G.scale_log2, S.QKV[j * E3 + E + h * DH + d], s);
      }
      const float m = gmax8(s);
      const float p = valid ? ex2f_(s - m) : 0.f;
      const float l = gsum8(p);
      const float pn = valid ? p / l : 0.f;
      float pd = pn * G.ik_sa;
      if (G.thr_sa && valid) {
        const uint32_t rk = attn_row_key(key_of(a.rng, a.call_id[blk][0]),
                                         (uint32_t)(((int64_t)b * H + h) * T + tok));
        if (!attn_keep(rk, j, G.thr_sa)) pd = 0.f;
      }
      if (hf == 0) {
        S.PD[(h * TMAX + tok) * TMAX + j] = valid ? pd : 0.f;
        sv[S_PN + (h * TMAX + tok) * TMAX + j] = pn;
      }
    }
    __syncthreads();
    {
      const int h = f >> 3;
      float o = 0.f;
      for (int j = 0; j < T; ++j) o = fmaf(S.PD[(h * TMAX + tok) * TMAX + j], S.QKV[j * E3 + 2 * E + f], o);
      if (hf == 0) S.O[tf] = o;
      if (wr) sv[S_O + tf] = o;
    }
    __syncthreads();
    PT(0, 3);
    // ---- PRE: out-projection, residual dropout (site 0), LN1, cross q
    {
      float v = S.w.bo1[f] + dot_row(S.w.Wo1, f, S.O + tok * E, hf);
      if (G.thr_res && !res_keep(site_key(key_of(a.rng, a.call_id[blk][1]), 0), row, f, G.thr_res))
        v = 0.f;
      else
        v *= G.ik_res;
      float rs;
      const float xh = ln_fwd(v + xin, rs);
      const float x1 = fmaf(xh, S.w.g1[f], S.w.be1[f]);
      if (hf == 0) S.X1[tf] = x1;
      if (wr) {
        sv[S_XH1 + tf] = xh;
        sv[S_X1 + tf] = x1;
        if (f == 0) sv[S_RS1 + tok] = rs;
      }
    }
    __syncthreads();
    {
      const float q = S.w.bq[f] + dot_row(S.w.Wq, f, S.X1 + tok * E, hf);
      if (hf == 0) S.QS[tf] = q * G.scale_log2;
      if (wr) sv[S_QS + tf] = q * G.scale_log2;
    }
    __syncthreads();
    PT(0, 4);
    // ---- cross-attention over the Lk context tokens: lane (query-head qh, key slice ks).
    // K / V / key-bias tiles of KTF keys are staged in LDS; the next tile's loads are in
    // flight while the current one is computed.  Online softmax per tile (one rescale
    // per tile and lane), then the NSL slices are merged in a fixed order.
    {
      const int qh = tid & 31, ks = tid >> 5, i = qh >> 2, h = qh & 3;
      const bool qa = i < T;
      float qv[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) qv[d] = S.QS[i * E + h * DH + d];
      const float* kvb = a.kv[blk] + (int64_t)b * a.Lk * 2 * E;
      const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kbias_bs : nullptr;
      uint32_t rk = 0u;
      if (G.thr_ca)
        rk = attn_row_key(key_of(a.rng, a.call_id[blk][2]),
                          (uint32_t)(((int64_t)b * H + h) * T + (qa ? i : T - 1)));
      float m = -INFINITY, l = 0.f, o[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = 0.f;
      constexpr int NR = KTF * 2 * E / 4 / NT;      // float4 loads per thread per tile
      float4 pf[NR];
      float pkb = 0.f;
      auto load_tile = [&](int j0) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int idx = tid + NT * r, key = j0 + (idx >> 4);
          pf[r] = key < a.Lk ? *reinterpret_cast<const float4*>(kvb + (int64_t)key * 2 * E + (idx & 15) * 4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (tid < KTF) pkb = (j0 + tid < a.Lk && kbp) ? kbp[j0 + tid] : 0.f;
      };
      load_tile(0);
      for (int j0 = 0; j0 < a.Lk; j0 += KTF) {
        __syncthreads();                      // the previous tile's readers are done
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int idx = tid + NT * r, kl = idx >> 4, c = (idx & 15) * 4;
          *reinterpret_cast<float4*>((c < E ? S.Kt : S.Vt) + kl * E + (c & (E - 1))) = pf[r];
        }
        if (tid < KTF) S.Kb[tid] = pkb;
        __syncthreads();
        if (j0 + KTF < a.Lk) load_tile(j0 + KTF);
        const int nk = min(KTF, a.Lk - j0);
        float sc[KTF / NSL];
        float mt = -INFINITY;
#pragma unroll
        for (int n = 0; n < KTF / NSL; ++n) {
          const int jj = ks + NSL * n;
          float x = -INFINITY;
          if (jj < nk) {
            const float4 k0 = *reinterpret_cast<const float4*>(S.Kt + jj * E + h * DH);
            const float4 k1 = *reinterpret_cast<const float4*>(S.Kt + jj * E + h * DH + 4);
            x = S.Kb[jj];
            x = fmaf(qv[0], k0.x, x); x = fmaf(qv[1], k0.y, x); x = fmaf(qv[2], k0.z, x);
            x = fmaf(qv[3], k0.w, x); x = fmaf(qv[4], k1.x, x); x = fmaf(qv[5], k1.y, x);
            x = fmaf(qv[6], k1.z, x); x = fmaf(qv[7], k1.w, x);
          }
          sc[n] = x;
          mt = fmaxf(mt, x);
        }
        if (mt > m) {
          const float c = m == -INFINITY ? 0.f : ex2f_(m - mt);
          l *= c;
#pragma unroll
          for (int d = 0; d < DH; ++d) o[d] *= c;
          m = mt;
        }
        const float mu = m == -INFINITY ? 0.f : m;   // all keys so far masked: p = 0
#pragma unroll
        for (int n = 0; n < KTF / NSL; ++n) {
          const int jj = ks + NSL * n;
          if (jj < nk) {
            float p = ex2f_(sc[n] - mu);
            l += p;
            if (G.thr_ca && !attn_keep(rk, j0 + jj, G.thr_ca)) p = 0.f;
            const float4 v0 = *reinterpret_cast<const float4*>(S.Vt + jj * E + h * DH);
            const float4 v1 = *reinterpret_cast<const float4*>(S.Vt + jj * E + h * DH + 4);
            o[0] = fmaf(p, v0.x, o[0]); o[1] = fmaf(p, v0.y, o[1]); o[2] = fmaf(p, v0.z, o[2]);
            o[3] = fmaf(p, v0.w, o[3]); o[4] = fmaf(p, v1.x, o[4]); o[5] = fmaf(p, v1.y, o[5]);
            o[6] = fmaf(p, v1.z, o[6]); o[7] = fmaf(p, v1.w, o[7]);
          }
        }
      }
      S.red[ks][qh][0] = m;
      S.red[ks][qh][1] = l;
#pragma unroll
      for (int d = 0; d < DH; ++d) S.red[ks][qh][2 + d] = o[d];
      __syncthreads();
      if (tid < 32 * DH) {       // lane (qh, feature d) merges the slices in order
        const int q2 = tid >> 3, d = tid & 7, i2 = q2 >> 2, h2 = q2 & 3;
        float M = S.red[0][q2][0];
#pragma unroll
        for (int k = 1; k < NSL; ++k) M = fmaxf(M, S.red[k][q2][0]);
        float lt = 0.f, ot = 0.f;
#pragma unroll
        for (int k = 0; k < NSL; ++k) {
          const float mk = S.red[k][q2][0];
          const float fk = mk == -INFINITY ? 0.f : ex2f_(mk - M);
          lt = fmaf(S.red[k][q2][1], fk, lt);
          ot = fmaf(S.red[k][q2][2 + d], fk, ot);
        }
        const bool q2a = i2 < T;
        const float c = q2a ? ot * G.ik_ca / lt : 0.f;   // every key masked: 0/0 = NaN
        S.C[i2 * E + h2 * DH + d] = c;
        if (q2a) {
          sv[S_C + i2 * E + h2 * DH + d] = c;
          if (d == 0) sv[S_LSE + q2] = M + __log2f(lt);
        }
      }
    }
    __syncthreads();
    PT(0, 5);
    // ---- POST: out-projection, dropout (site 1), LN2, FFN, dropout (site 2), LN3
    const uint32_t kpost = G.thr_res ? key_of(a.rng, a.call_id[blk][3]) : 0u;
    {
      float v = S.w.bo2[f] + dot_row(S.w.Wo2, f, S.C + tok * E, hf);
      if (G.thr_res && !res_keep(site_key(kpost, 1), row, f, G.thr_res)) v = 0.f;
      else v *= G.ik_res;
      float rs;
      const float xh = ln_fwd(v + S.X1[tf], rs);
      const float x2 = fmaf(xh, S.w.g2[f], S.w.be2[f]);
      if (hf == 0) S.X2[tf] = x2;
      if (wr) {
        sv[S_XH2 + tf] = xh;
        sv[S_X2 + tf] = x2;
        if (f == 0) sv[S_RS2 + tok] = rs;
      }
    }
    __syncthreads();
    {
      const float h1 = S.w.b1[f] + dot_row(S.w.W1, f, S.X2 + tok * E, hf);
      if (hf == 0) S.GL[tf] = gelu_erf(h1);
      if (wr) sv[S_H1 + tf] = h1;
    }
    __syncthreads();
    {
      float v = S.w.b2[f] + dot_row(S.w.W2, f, S.GL + tok * E, hf);
      if (G.thr_res && !res_keep(site_key(kpost, 2), row, f, G.thr_res)) v = 0.f;
      else v *= G.ik_res;
      float rs;
      const float xh = ln_fwd(v + S.X2[tf], rs);
      const float y = fmaf(xh, S.w.g3[f], S.w.be3[f]);
      if (wr) {
        sv[S_XH3 + tf] = xh;
        if (f == 0) sv[S_RS3 + tok] = rs;
      }
      __syncthreads();      // every lane is done reading X for this block
      if (hf == 0) S.X[tf] = act ? y : 0.f;
    }
    PT(0, 6);
  }
  __syncthreads();
  if (wr) a.y[((int64_t)b * T + tok) * E + f] = S.X[tf];
}

// ============================== backward ===================================
struct __attribute__((aligned(16))) BwdSmem {
  Wts w;
  float DY[TMAX * E], GL3[TMAX * E], DF[TMAX * E], GLU[TMAX * E], DH1[TMAX * E],
      GL2[TMAX * E], DA2[TMAX * E], DC[TMAX * E], DQ[TMAX * E], GL1[TMAX * E], DA1[TMAX * E],
      DO[TMAX * E], DQKV[TMAX * E3], PD[H * TMAX * TMAX], DSS[H * TMAX * TMAX];
  float SV[SAVE_BLK];   // this block's saved activations
  float lse[32], Dq[32];
  uint32_t rk[32];
  float DS[32 * DSP];
  float Kt[KTB * E];    // key tile; after the last tile, the dq reduction [16][32][8]
};

// out[o][k] = sum_{t < T} G[t][o] X[t][k] (o < NO, k < 32); out row-major [NO][32]
template <int NO>
__device__ __forceinline__ void outer_sum(const float* G, int gp, const float* X, int T,
                                          float* out) {
  for (int idx = threadIdx.x; idx < NO * 8; idx += NT) {
    const int o = idx >> 3, k4 = (idx & 7) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t = 0; t < T; ++t) {
      const float g = G[t * gp + o];
      const float4 x = *reinterpret_cast<const float4*>(X + t * E + k4);
      acc.x = fmaf(g, x.x, acc.x); acc.y = fmaf(g, x.y, acc.y);
      acc.z = fmaf(g, x.z, acc.z); acc.w = fmaf(g, x.w, acc.w);
    }
    *reinterpret_cast<float4*>(out + o * E + k4) = acc;
  }
}
// out[o] = sum_{t < T} G[t][o] for the thread's o (the bias gradients)
__device__ __forceinline__ void col_sum1(const float* G, int gp, int o, int T, float* out) {
  float acc = 0.f;
  for (int t = 0; t < T; ++t) acc += G[t * gp + o];
  out[o] = acc;
}
// LayerNorm affine gradients: dg[f] = sum_t G[t][f] xh[t][f], db[f] = sum_t G[t][f]
__device__ __forceinline__ void ln_sums1(const float* G, const float* XH, int f, int T, float* dg,
                                         float* db) {
  float a = 0.f, c = 0.f;
  for (int t = 0; t < T; ++t) {
    a = fmaf(G[t * E + f], XH[t * E + f], a);
    c += G[t * E + f];
  }
  dg[f] = a;
  db[f] = c;
}

__global__ __launch_bounds__(NT) void enc_chain_bwd_kernel(Args args) {
  __shared__ BwdSmem S;
  const Grp& G = args.g[blockIdx.y];
  const vaesne_enc_chain_group& a = G.d;
  const int b = blockIdx.x;
  if (b >= a.B) return;
  const int tid = threadIdx.x, tok = tid >> 6, lane = tid & 63, f = lane & 31, hf = lane >> 5;
  const int T = a.T;
  const bool act = tok < T;
  const int tf = tok * E + f;
  const int64_t row = (int64_t)b * T + (act ? tok : T - 1);
  if (hf == 0) S.DY[tf] = act ? a.dy[((int64_t)b * T + tok) * E + f] : 0.f;
  for (int blk = a.nb - 1; blk >= 0; --blk) {
    const float* sv = a.save + ((int64_t)b * a.nb + blk) * SAVE_BLK;
    float* wp = a.wpart + ((int64_t)b * a.nb + blk) * PBLK;
    __syncthreads();
    PT(1, 0);
    {   // weights and this block's saved activations: all loads in flight at once
      constexpr int NRS = (SAVE_BLK / 4 + NT - 1) / NT;
      float4 r4[NRS];
#pragma unroll
      for (int r = 0; r < NRS; ++r) {
        const int i = tid + NT * r;
        if (i < SAVE_BLK / 4) r4[r] = reinterpret_cast<const float4*>(sv)[i];
      }
      stage(S.w, a.w[blk]);
#pragma unroll
      for (int r = 0; r < NRS; ++r) {
        const int i = tid + NT * r;
        if (i < SAVE_BLK / 4) reinterpret_cast<float4*>(S.SV)[i] = r4[r];
      }
    }
    __syncthreads();
    PT(1, 1);
    const uint32_t kpost = G.thr_res ? key_of(a.rng, a.call_id[blk][3]) : 0u;
    const uint32_t kpre = G.thr_res ? key_of(a.rng, a.call_id[blk][1]) : 0u;
    float acc;
    // ---- LN3, FFN, LN2 (POST backward)
    {
      const float g = S.DY[tf];
      const float dz = ln_bwd(g, S.SV[S_XH3 + tf], S.w.g3[f], S.SV[S_RS3 + tok]);
      acc = dz;                                             // d x2 (residual)
      float df = dz * G.ik_res;
      if (G.thr_res && !res_keep(site_key(kpost, 2), row, f, G.thr_res)) df = 0.f;
      if (hf == 0) {
        S.GL3[tf] = g;
        S.DF[tf] = act ? df : 0.f;
        S.GLU[tf] = act ? gelu_erf(S.SV[S_H1 + tf]) : 0.f;
      }
    }
    __syncthreads();
    {
      const float dgl = dot_col<E>(S.w.W2, f, S.DF + tok * E, hf);
      if (hf == 0) S.DH1[tf] = act ? dgl * gelu_erf_grad(S.SV[S_H1 + tf]) : 0.f;
    }
    __syncthreads();
    acc += dot_col<E>(S.w.W1, f, S.DH1 + tok * E, hf);     // d x2 total
    if (hf == 0) S.GL2[tf] = act ? acc : 0.f;
    {
      const float dz = ln_bwd(acc, S.SV[S_XH2 + tf], S.w.g2[f], S.SV[S_RS2 + tok]);
      acc = dz;                                             // d x1 (residual)
      float da = dz * G.ik_res;
      if (G.thr_res && !res_keep(site_key(kpost, 1), row, f, G.thr_res)) da = 0.f;
      if (hf == 0) S.DA2[tf] = act ? da : 0.f;
    }
    __syncthreads();
    {
      const float dc = dot_col<E>(S.w.Wo2, f, S.DA2 + tok * E, hf);
      if (hf == 0) S.DC[tf] = act ? dc : 0.f;
    }
    __syncthreads();
    PT(1, 2);
    // ---- cross-attention backward: d q -> S.DQ, d(k|v) of this sequence -> a.dkv[blk].
    // Per key tile, lane (key, head) runs the T queries of its head; dS goes to LDS for
    // the dq contraction by lane (query-head, key slice).
    if (tid < 32) {
      const int qh = tid, i = qh >> 2, h = qh & 3;
      float D = 0.f;
      if (i < T) {
#pragma unroll
        for (int d = 0; d < DH; ++d)
          D = fmaf(S.DC[i * E + h * DH + d], S.SV[S_C + i * E + h * DH + d], D);
      }
      S.Dq[qh] = D;
      S.lse[qh] = i < T ? S.SV[S_LSE + qh] : 0.f;
      S.rk[qh] = G.thr_ca ? attn_row_key(key_of(a.rng, a.call_id[blk][2]),
                                          (uint32_t)(((int64_t)b * H + h) * T + (i < T ? i : T - 1)))
                          : 0u;
    }
    __syncthreads();
    {
      const float* kvb = a.kv[blk] + (int64_t)b * a.Lk * 2 * E;
      float* dkvb = a.dkv[blk] + (int64_t)b * a.Lk * 2 * E;
      const float* kbp = a.kbias ? a.kbias + (int64_t)b * a.kbias_bs : nullptr;
      const int h = tid >> 7, jl = tid & (KTB - 1);           // per-key phase
      const int qh = tid & 31, js = tid >> 5, hq = qh & 3;    // dq phase: 16 slices of 8 keys
      const bool qok = (qh >> 2) < T;
      float dqa[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) dqa[d] = 0.f;
      // this lane's k | v row slices of the next tile are loaded while the current
      // tile is computed
      float4 pk0, pk1, pv0, pv1;
      float pkb;
      auto load_kv = [&](int j) {
        pk0 = pk1 = pv0 = pv1 = make_float4(0.f, 0.f, 0.f, 0.f);
        pkb = 0.f;
        if (j < a.Lk) {
          const float* r = kvb + (int64_t)j * 2 * E + h * DH;
          pk0 = *reinterpret_cast<const float4*>(r);
          pk1 = *reinterpret_cast<const float4*>(r + 4);
          pv0 = *reinterpret_cast<const float4*>(r + E);
          pv1 = *reinterpret_cast<const float4*>(r + E + 4);
          if (kbp) pkb = kbp[j];
        }
      };
      load_kv(jl);
      for (int j0 = 0; j0 < a.Lk; j0 += KTB) {
        const int j = j0 + jl;
        const bool kok = j < a.Lk;
        float k[DH], v[DH], dk[DH], dv[DH];
        const float kb = pkb;
        {
          const float4 k0 = pk0, k1 = pk1, v0 = pv0, v1 = pv1;
          k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w;
          k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
          v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
          v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
          *reinterpret_cast<float4*>(S.Kt + jl * E + h * DH) = k0;
          *reinterpret_cast<float4*>(S.Kt + jl * E + h * DH + 4) = k1;
        }
        if (j0 + KTB < a.Lk) load_kv(j + KTB);
#pragma unroll
        for (int d = 0; d < DH; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
        for (int i = 0; i < T; ++i) {
          const int q = i * 4 + h;
          const float4 qa0 = *reinterpret_cast<const float4*>(S.SV + S_QS + i * E + h * DH);
          const float4 qa1 = *reinterpret_cast<const float4*>(S.SV + S_QS + i * E + h * DH + 4);
          const float4 g0 = *reinterpret_cast<const float4*>(S.DC + i * E + h * DH);
          const float4 g1 = *reinterpret_cast<const float4*>(S.DC + i * E + h * DH + 4);
          const float qv[DH] = {qa0.x, qa0.y, qa0.z, qa0.w, qa1.x, qa1.y, qa1.z, qa1.w};
          const float gv[DH] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
          float s = kb, dp = 0.f;
#pragma unroll
          for (int d = 0; d < DH; ++d) {
            s = fmaf(qv[d], k[d], s);
            dp = fmaf(gv[d], v[d], dp);
          }
          const float p = ex2f_(s - S.lse[q]);
          float aP = p * G.ik_ca, dP = dp * G.ik_ca;
          if (G.thr_ca && !attn_keep(S.rk[q], j, G.thr_ca)) { aP = 0.f; dP = 0.f; }
          const float ds = kok ? p * (dP - S.Dq[q]) : 0.f;
#pragma unroll
          for (int d = 0; d < DH; ++d) {
            dv[d] = fmaf(aP, gv[d], dv[d]);
            dk[d] = fmaf(ds, qv[d], dk[d]);
          }
          S.DS[q * DSP + jl] = ds;
        }
        if (kok) {
          float* r = dkvb + (int64_t)j * 2 * E + h * DH;
          *reinterpret_cast<float4*>(r) = make_float4(dk[0] * G.kf, dk[1] * G.kf, dk[2] * G.kf, dk[3] * G.kf);
          *reinterpret_cast<float4*>(r + 4) = make_float4(dk[4] * G.kf, dk[5] * G.kf, dk[6] * G.kf, dk[7] * G.kf);
          *reinterpret_cast<float4*>(r + E) = make_float4(dv[0], dv[1], dv[2], dv[3]);
          *reinterpret_cast<float4*>(r + E + 4) = make_float4(dv[4], dv[5], dv[6], dv[7]);
        }
        __syncthreads();
        if (qok) {
          const int n1 = min(8, a.Lk - j0 - js * 8);
          for (int n = 0; n < n1; ++n) {
            const int jj = js * 8 + n;
            const float dsv = S.DS[qh * DSP + jj];
            const float4 k0 = *reinterpret_cast<const float4*>(S.Kt + jj * E + hq * DH);
            const float4 k1 = *reinterpret_cast<const float4*>(S.Kt + jj * E + hq * DH + 4);
            dqa[0] = fmaf(dsv, k0.x, dqa[0]); dqa[1] = fmaf(dsv, k0.y, dqa[1]);
            dqa[2] = fmaf(dsv, k0.z, dqa[2]); dqa[3] = fmaf(dsv, k0.w, dqa[3]);
            dqa[4] = fmaf(dsv, k1.x, dqa[4]); dqa[5] = fmaf(dsv, k1.y, dqa[5]);
            dqa[6] = fmaf(dsv, k1.z, dqa[6]); dqa[7] = fmaf(dsv, k1.w, dqa[7]);
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int d = 0; d < DH; ++d) S.Kt[(js * 32 + qh) * DH + d] = dqa[d];
      __syncthreads();
      if (tid < 32 * DH) {
        const int q2 = tid >> 3, d = tid & 7, i2 = q2 >> 2, h2 = q2 & 3;
        float t = S.Kt[q2 * DH + d];
#pragma unroll
        for (int k = 1; k < KTB / 8; ++k) t += S.Kt[(k * 32 + q2) * DH + d];
        S.DQ[i2 * E + h2 * DH + d] = i2 < T ? t * G.scale : 0.f;
      }
    }
    __syncthreads();
    PT(1, 3);
    // ---- PRE backward: cross q projection, LN1, out-projection
    acc += dot_col<E>(S.w.Wq, f, S.DQ + tok * E, hf);      // d x1 total
    if (hf == 0) S.GL1[tf] = act ? acc : 0.f;
    {
      const float dz = ln_bwd(acc, S.SV[S_XH1 + tf], S.w.g1[f], S.SV[S_RS1 + tok]);
      acc = dz;                                             // d x (residual)
      float da = dz * G.ik_res;
      if (G.thr_res && !res_keep(site_key(kpre, 0), row, f, G.thr_res)) da = 0.f;
      if (hf == 0) S.DA1[tf] = act ? da : 0.f;
    }
    __syncthreads();
    {
      const float dO = dot_col<E>(S.w.Wo1, f, S.DA1 + tok * E, hf);
      if (hf == 0) S.DO[tf] = act ? dO : 0.f;
    }
    __syncthreads();
    PT(1, 4);
    // ---- self-attention backward: lane (query tok, head h, key j)
    {
      const int h = (lane >> 3) & 3, j = lane & 7;
      const bool valid = act && j < T;
      const float pn = valid ? S.SV[S_PN + (h * TMAX + tok) * TMAX + j] : 0.f;
      float dpd = 0.f;
      if (valid) {
#pragma unroll
        for (int d = 0; d < DH; ++d)
          dpd = fmaf(S.DO[tok * E + h * DH + d], S.SV[S_QKV + j * E3 + 2 * E + h * DH + d], dpd);
      }
      bool kp = true;
      if (G.thr_sa && valid) {
        const uint32_t rk = attn_row_key(key_of(a.rng, a.call_id[blk][0]),
                                         (uint32_t)(((int64_t)b * H + h) * T + tok));
        kp = attn_keep(rk, j, G.thr_sa);
      }
      const float dp = kp ? dpd * G.ik_sa : 0.f;
      const float D = gsum8(pn * dp);
      if (hf == 0) {
        S.DSS[(h * TMAX + tok) * TMAX + j] = valid ? pn * (dp - D) : 0.f;
        S.PD[(h * TMAX + tok) * TMAX + j] = (valid && kp) ? pn * G.ik_sa : 0.f;
      }
    }
    __syncthreads();
    {
      const int h = f >> 3;
      float dq = 0.f, dk = 0.f, dv = 0.f;
      for (int j = 0; j < T; ++j) {
        dq = fmaf(S.DSS[(h * TMAX + tok) * TMAX + j], S.SV[S_QKV + j * E3 + E + f], dq);
        dk = fmaf(S.DSS[(h * TMAX + j) * TMAX + tok], S.SV[S_QKV + j * E3 + f], dk);
        dv = fmaf(S.PD[(h * TMAX + j) * TMAX + tok], S.DO[j * E + f], dv);
      }
      if (hf == 0) {
        S.DQKV[tok * E3 + f] = act ? dq * G.scale : 0.f;
        S.DQKV[tok * E3 + E + f] = act ? dk * G.scale : 0.f;
        S.DQKV[tok * E3 + 2 * E + f] = act ? dv : 0.f;
      }
    }
    __syncthreads();
    PT(1, 5);
    acc += dot_col<E3>(S.w.Wi, f, S.DQKV + tok * E3, hf);  // d x total (block input)
    // ---- this sequence's weight-gradient partials
    outer_sum<E3>(S.DQKV, E3, S.SV + S_XIN, T, wp + O_WI);
    outer_sum<E>(S.DA1, E, S.SV + S_O, T, wp + O_WO1);
    outer_sum<E>(S.DQ, E, S.SV + S_X1, T, wp + O_WC);
    outer_sum<E>(S.DA2, E, S.SV + S_C, T, wp + O_WO2);
    outer_sum<E>(S.DH1, E, S.SV + S_X2, T, wp + O_W1);
    outer_sum<E>(S.DF, E, S.GLU, T, wp + O_W2);
    if (tid < E3) col_sum1(S.DQKV, E3, tid, T, wp + O_BI);
    else if (tid < E3 + E) col_sum1(S.DA1, E, tid - E3, T, wp + O_BO1);
    else if (tid < E3 + 2 * E) col_sum1(S.DQ, E, tid - E3 - E, T, wp + O_BC);
    else if (tid < E3 + 3 * E) col_sum1(S.DA2, E, tid - E3 - 2 * E, T, wp + O_BO2);
    else if (tid < E3 + 4 * E) col_sum1(S.DH1, E, tid - E3 - 3 * E, T, wp + O_B1);
    else if (tid < E3 + 5 * E) col_sum1(S.DF, E, tid - E3 - 4 * E, T, wp + O_B2);
    else if (tid < E3 + 6 * E) ln_sums1(S.GL1, S.SV + S_XH1, tid - E3 - 5 * E, T, wp + O_G1, wp + O_BE1);
    else if (tid < E3 + 7 * E) ln_sums1(S.GL2, S.SV + S_XH2, tid - E3 - 6 * E, T, wp + O_G2, wp + O_BE2);
    else if (tid < E3 + 8 * E) ln_sums1(S.GL3, S.SV + S_XH3, tid - E3 - 7 * E, T, wp + O_G3, wp + O_BE3);
    __syncthreads();
    PT(1, 6);
    if (hf == 0) S.DY[tf] = act ? acc : 0.f;
  }
  __syncthreads();
  if (act && hf == 0) a.dx0[((int64_t)b * T + tok) * E + f] = S.DY[tf];
}

Grp make_grp(const vaesne_enc_chain_group& d) {
  Grp g{};
  g.d = d;
  g.thr_sa = drop_thr16(d.p_attn);
  g.thr_res = drop_thr16(d.p_res);
  g.thr_ca = drop_thr16(d.p_cross);
  g.ik_sa = d.p_attn > 0.f ? 1.f / (1.f - d.p_attn) : 1.f;
  g.ik_res = d.p_res > 0.f ? 1.f / (1.f - d.p_res) : 1.f;
  g.ik_ca = d.p_cross > 0.f ? 1.f / (1.f - d.p_cross) : 1.f;
  g.scale = 1.0f / sqrtf((float)DH);            // = vaesne_attn_* (attention.hip)
  g.scale_log2 = g.scale * 1.4426950408889634f;
  g.kf = g.scale / g.scale_log2;
  return g;
}

int check(const vaesne_enc_chain_group& d, bool bwd) {
  if (d.B <= 0 || d.T < 1 || d.T > TMAX || d.Lk < 1 || d.nb < 1 || d.nb > VAESNE_ENC_CHAIN_MAXB)
    return (int)hipErrorInvalidValue;
  if (!d.save || (!bwd && (!d.x0 || !d.y))) return (int)hipErrorInvalidValue;
  if ((d.p_attn > 0.f || d.p_res > 0.f || d.p_cross > 0.f) && !d.rng) return (int)hipErrorInvalidValue;
  for (int blk = 0; blk < d.nb; ++blk) {
    for (int i = 0; i < 18; ++i)
      if (!d.w[blk][i]) return (int)hipErrorInvalidValue;
    if (!d.kv[blk] || (bwd && !d.dkv[blk])) return (int)hipErrorInvalidValue;
  }
  if (bwd && (!d.dy || !d.dx0 || !d.wpart || !d.gflat)) return (int)hipErrorInvalidValue;
  return 0;
}

int launch(int G, const vaesne_enc_chain_group* groups, bool bwd, hipStream_t s) {
  if (G < 1 || !groups) return (int)hipErrorInvalidValue;
  for (int g0 = 0; g0 < G; g0 += GMAX) {
    Args args{};
    int n = min(GMAX, G - g0), Bmax = 0;
    for (int i = 0; i < n; ++i) {
      const int rc = check(groups[g0 + i], bwd);
      if (rc) return rc;
      args.g[i] = make_grp(groups[g0 + i]);
      Bmax = max(Bmax, groups[g0 + i].B);
    }
    if (bwd) hipLaunchKernelGGL(enc_chain_bwd_kernel, dim3(Bmax, n), dim3(NT), 0, s, args);
    else hipLaunchKernelGGL(enc_chain_fwd_kernel, dim3(Bmax, n), dim3(NT), 0, s, args);
    VAESNE_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace

VAESNE_API int vaesne_enc_chain_layout(int* save_blk, int* pblk, int* offsets) {
  if (save_blk) *save_blk = SAVE_BLK;
  if (pblk) *pblk = PBLK;
  if (offsets) {
    const int off[18] = {O_WI, O_BI, O_WO1, O_BO1, O_G1, O_BE1, O_WC, O_BC, O_WO2,
                         O_BO2, O_G2, O_BE2, O_W1, O_B1, O_W2, O_B2, O_G3, O_BE3};
    for (int i = 0; i < 18; ++i) offsets[i] = off[i];
  }
  return 0;
}

VAESNE_API int vaesne_enc_chain_fwd(int G, const vaesne_enc_chain_group* groups, void* stream) {
  return launch(G, groups, false, (hipStream_t)stream);
}

VAESNE_API int vaesne_enc_chain_bwd(int G, const vaesne_enc_chain_group* groups,
                                    vaesne_colsum_list* defer, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = launch(G, groups, true, s);
  if (rc) return rc;
  // per block: [Wi .. be1, Wq rows] | [bq] | [Wo2 .. be3]; the k|v rows of the cross
  // in_proj (and their biases) come from the caller's context-projection gradient
  const int reg[3][2] = {{0, O_WC + E * E}, {O_BC, O_BC + E}, {O_WO2, PBLK}};
  for (int g = 0; g < G; ++g) {
    const vaesne_enc_chain_group& d = groups[g];
    const int64_t ld = (int64_t)d.nb * PBLK;
    for (int blk = 0; blk < d.nb; ++blk)
      for (int r = 0; r < 3; ++r) {
        const int64_t off = (int64_t)blk * PBLK + reg[r][0];
        rc = colsum_or_defer(defer, d.wpart + off, ld, d.B, reg[r][1] - reg[r][0], d.gflat + off, 0, s);
        if (rc) return rc;
      }
  }
  return 0;
}

#ifdef VAESNE_CHAIN_PROFILE
VAESNE_API int vaesne_enc_chain_profile_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_prof), sizeof(g_chain_prof));
}
#endif
