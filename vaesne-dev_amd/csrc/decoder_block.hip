// Fused decoder-block tail of VAESNe (TransformerBlock.forward after the masked
// self-attention core, util_layers.py:285-309, as used by the decoders
// spectraTransformerDecoder SpectraLayers.py:55-63 and
// photometricTransformerDecoder PhotometricLayers.py:66-68):
//
//   a1 = O Wo1^T + bo1                   self-attn out_proj
//   x1 = LN1(x + Drop(a1))
//   q  = x1 Wq^T + bq                    cross-attn in_proj rows [0, E)
//   c  = Drop(softmax(q k^T / sqrt(dh))) v   over the Lc <= 8 context tokens
//                                        (k, v = projected decoder context, unmasked)
//   a2 = c Wo2^T + bo2;   x2 = LN2(x1 + Drop(a2))
//   f  = W2 gelu(W1 x2 + b1) + b2;   y = LN3(x2 + Drop(f))
//   [qkv_next = y Wn^T + bn]             the NEXT block's self-attn in_proj
//
// E = 32, H = 4, dh = 8, ff = 32 (every cannon script).  One launch replaces
// ~20 op-level launches (and ~40 in the backward) and all their HBM round trips.
//
// Layout ("feature layout" of v_mfma_f32_32x32x2_f32): a wave owns 32 tokens;
// lane l holds token t = l & 31 and the 16 features F(r, h) = (r&3) + 8(r>>2) + 4h,
// h = l >> 5, r = 0..15 — exactly the rows an MFMA accumulator D[o][t] gives
// lane l.  So y = W x is 16 MFMAs with A = W (from LDS) and B = x straight from
// the previous accumulator: no shuffles between layers.  LayerNorm = 16 in-lane
// adds + one cross-half swap; each head's 8 dims are regs 4hd..4hd+3 of both halves.
//
// Backward: recompute the forward in registers, run the chain in reverse, and
// accumulate every weight gradient dW = sum_t g_t x_t^T with MFMAs whose
// contraction runs over the wave's 32 tokens (operands staged in LDS rows).
// Per-workgroup partials -> fixed-order column sums (bitwise reproducible),
// launched at once or deferred to the backward pass's batched flush.
// Context (k, v) gradients are per sequence: a workgroup only ever covers
// tokens of ONE sequence, so they accumulate in the same way.
#include "common.h"

using namespace vaesne;

namespace {

constexpr int E = 32, H = 4, DH = 8, LP = 33;  // LP: padded LDS row (floats)
constexpr int NW = 4, NT = 256;               // waves / threads per workgroup
constexpr int LCMAX = 8;

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int F(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f16v mfma(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

struct Tail {
  // activations
  const float* x;      // [M, 32] block input (residual stream)
  const float* O;      // [M, 32] self-attention core output
  const float* kvc;    // [Nseq, Lc, 64] projected context: k | v
  int M, L, Lc;        // tokens, tokens per sequence, context tokens
  // weights (row-major nn.Linear [out, in]) and vectors
  const float *Wo1, *bo1, *g1, *be1, *Wq, *bq, *Wo2, *bo2, *g2, *be2;
  const float *W1, *b1, *W2, *b2, *g3, *be3, *Wn, *bn;   // Wn/bn may be null
  float p_drop;        // residual / attention-probability dropout
  uint32_t thr; float inv_keep;
  const int64_t* rng; uint32_t call_id;
  int chunk;           // tokens per workgroup (multiple of 128)
  uint32_t* masks;     // [M][4] dropout keep masks written by fwd, read by bwd (or null:
                       // bwd re-hashes): word s < 3 = residual site s, 16 bits per half
                       // (half 0 low), word 3 = cross-attention keep bits
  // forward outputs
  float* y;            // [M, 32]
  float* qkv;          // [M, 96] (if Wn)
  // backward
  const float* dy;     // [M, 32]
  const float* dqkv;   // [M, 96] (if Wn)
  float* dx;           // [M, 32]
  float* dO;           // [M, 32]
  float* wpart;        // [G][WPART] per-workgroup partials (gflat itself when G == 1)
  float* dkvc;         // [Nseq, Lc, 64] context k | v gradients (two-kernel path scratch)
  const float* ctx;    // [Nseq, Lc, 32] context tokens (k | v projected in the kernels)
  float* dctx;         // [Nseq, Lc, 32] their gradient (backward)
  int mode;            // MODE_FULL (decoder block tail) / MODE_PRE / MODE_POST (encoder halves)
};

// dropout scale of bit `bit` of a keep word: ik where set, +0 where clear.  Bit
// arithmetic instead of a lane mask per bit + select (the fused backward kept those
// masks in SGPR pairs and spilled them into VGPR lanes).  Callers launder the word
// right before use so the 16 scales are not all computed early and held.
__device__ __forceinline__ float keep_sc(uint32_t k, int bit, float ik) {
  return __int_as_float(((int)(k << (31 - bit)) >> 31) & __float_as_int(ik));
}
__device__ __forceinline__ uint32_t opaque(uint32_t k) {
  asm volatile("" : "+v"(k));
  return k;
}

// Encoder blocks (util_layers.py:285-309 with the cross-attention over the
// ~60 / 984 data tokens, too many for the in-register cross attention of the
// tail) run as two halves around the external cross-attention kernel:
//   PRE : a1 = O Wo1^T + bo1, x1 = LN1(x + Drop(a1)), q = x1 Wq^T + bq
//   POST: a2 = c Wo2^T + bo2, x2 = LN2(x1 + Drop(a2)), FFN, y = LN3(x2 + Drop(f)),
//         [qkv_next = y Wn^T + bn]
// over the B * latent tokens (one "sequence" of M rows), replacing ~10 forward and
// ~25 backward op-level launches per block (graph launches of tiny kernels cost
// ~5 us each).
enum Mode { MODE_FULL = 0, MODE_PRE = 1, MODE_POST = 2 };

// --- LDS image of the weights --------------------------------------------
struct __attribute__((aligned(16))) Smem {
  float Wo1[E * LP], Wq[E * LP], Wo2[E * LP], W1[E * LP], W2[E * LP], Wn[3 * E * LP];
  float bo1[E], bq[E], bo2[E], b1[E], b2[E], bn[3 * E];
  float g1[E], be1[E], g2[E], be2[E], g3[E], be3[E];
  float kv[LCMAX * 2 * E];
  float ctxs[LCMAX * E];
};

// Prologue staging: every global load of the weights in flight before the LDS stores (the
// strided-loop form waited for each load in turn: ~40 dependent L2 round trips per
// workgroup before the first token)
template <int ROWS>
__device__ __forceinline__ void load_w(const float* src, float (&r)[ROWS * E / NT]) {
  static_assert(ROWS * E % NT == 0, "whole rounds of the workgroup");
#pragma unroll
  for (int j = 0; j < ROWS * E / NT; ++j) r[j] = src[threadIdx.x + j * NT];
}
template <int ROWS>
__device__ __forceinline__ void store_w(float* dst, const float (&r)[ROWS * E / NT]) {
#pragma unroll
  for (int j = 0; j < ROWS * E / NT; ++j) {
    const int i = threadIdx.x + j * NT;
    dst[(i / E) * LP + (i % E)] = r[j];
  }
}
// NV vectors of n floats (n <= NT): thread t < n stages element t of each; a null source
// stages zeros
template <int NV>
__device__ __forceinline__ void stage_vecs(float* const (&dst)[NV], const float* const (&src)[NV],
                                           int n) {
  if (threadIdx.x < n) {
    float r[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) r[v] = src[v] ? src[v][threadIdx.x] : 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) dst[v][threadIdx.x] = r[v];
  }
}
constexpr int MW = E * E / NT;   // per-thread elements of a 32 x 32 weight

__device__ __forceinline__ void stage_all(Smem& S, const Tail& a, bool next) {
  float w0[MW], w1[MW], w2[MW], w3[MW], w4[MW], wn[3 * MW];
  load_w<E>(a.Wo1, w0); load_w<E>(a.Wq, w1); load_w<E>(a.Wo2, w2);
  load_w<E>(a.W1, w3); load_w<E>(a.W2, w4);
  if (next) load_w<3 * E>(a.Wn, wn);
  stage_vecs<11>({S.bo1, S.bq, S.bo2, S.b1, S.b2, S.g1, S.be1, S.g2, S.be2, S.g3, S.be3},
                 {a.bo1, a.bq, a.bo2, a.b1, a.b2, a.g1, a.be1, a.g2, a.be2, a.g3, a.be3}, E);
  if (next) stage_vecs<1>({S.bn}, {a.bn}, 3 * E);
  store_w<E>(S.Wo1, w0); store_w<E>(S.Wq, w1); store_w<E>(S.Wo2, w2);
  store_w<E>(S.W1, w3); store_w<E>(S.W2, w4);
  if (next) store_w<3 * E>(S.Wn, wn);
}

// The sequence's projected context k | v into S.kv: the cross in_proj rows [E, 3E)
// (util_layers.py:301; a.Wq / a.bq point at row 0 of the in_proj weight / bias) on
// its Lc <= 8 context tokens, which also land in S.ctxs.  512 outputs: weights read
// straight from L2, no launch of their own.
__device__ void ctx_kv(Smem& S, const Tail& a, int seq) {
  for (int i = threadIdx.x; i < a.Lc * E; i += NT) S.ctxs[i] = a.ctx[(int64_t)seq * a.Lc * E + i];
  __syncthreads();
  for (int i = threadIdx.x; i < a.Lc * 2 * E; i += NT) {
    const int j = i >> 6, c = i & 63;
    const float* w = a.Wq + (int64_t)(E + c) * E;
    float wr[E];   // the weight row's loads all in flight together (dword loads: the row may
                   // be a view into an optimizer's flat buffer, 4-byte aligned only)
#pragma unroll
    for (int k = 0; k < E; ++k) wr[k] = w[k];
    float acc = a.bq[E + c];
#pragma unroll
    for (int k = 0; k < E; ++k) acc = fmaf(S.ctxs[j * E + k], wr[k], acc);
    S.kv[i] = acc;
  }
}

// y[r] = b[F(r,h)] + sum_k W[F(r,h)][k] x[k]      (x, y in feature layout)
__device__ __forceinline__ void mv(const float* W, const float* b, const float (&x)[16],
                                   float (&y)[16], int lane) {
  const int o = lane & 31, h = lane >> 5;
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = b ? b[F(r, h)] : 0.f;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma(W[o * LP + F(s, h)], x[s], acc);
#pragma unroll
  for (int r = 0; r < 16; ++r) y[r] = acc[r];
}
// mv on the f16 matrix cores with split products (the attention kernels' scheme,
// attention_sf16.hip): W and x carried as hi = f16(v), lo = f16(v - hi); y = b + Wh xh + Wl xh
// + Wh xl with fp32 accumulation (2^-20 relative per product) in six v_mfma_f32_32x32x16_f16
// instead of sixteen v_mfma_f32_32x32x2_f32 (3/16 of the matrix-core time).  For the decoder
// tails' forward chain (and its recompute in the backward), whose operands are LayerNorm
// outputs, attention / cross-attention outputs and GELU values: O(1), inside f16's range
// (the encoder halves keep mv: the fused encoder chain is pinned to them bit for bit).
// MFMA K = 16: lane half h carries its own 8 features F(8m + e, h), e = 0..7, of group m in
// both operands (A: W[o][.], B: x_t[.]), so no cross-lane movement; each dword pairs two
// features of ONE precision (a dword mixing a hi and a lo product of one value loses the lo)
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t pk_hi16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, h2v));
}
__device__ __forceinline__ uint32_t pk_lo16(float a, float b, uint32_t hi) {
  const f2v h = __builtin_convertvector(__builtin_bit_cast(h2v, hi), f2v);
  return pk_hi16(a - h.x, b - h.y);
}
__device__ __forceinline__ f16v mfma16(u4v a, u4v b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b),
                                                c, 0, 0, 0);
}
__device__ __forceinline__ void mv16(const float* W, const float* b, const float (&x)[16],
                                     float (&y)[16], int lane) {
  const int o = lane & 31, h = lane >> 5;
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = b ? b[F(r, h)] : 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    u4v wh, wl, xh, xl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float w0 = W[o * LP + F(8 * m + 2 * i, h)], w1 = W[o * LP + F(8 * m + 2 * i + 1, h)];
      wh[i] = pk_hi16(w0, w1);
      wl[i] = pk_lo16(w0, w1, wh[i]);
      xh[i] = pk_hi16(x[8 * m + 2 * i], x[8 * m + 2 * i + 1]);
      xl[i] = pk_lo16(x[8 * m + 2 * i], x[8 * m + 2 * i + 1], xh[i]);
    }
    acc = mfma16(wh, xh, acc);
    acc = mfma16(wl, xh, acc);
    acc = mfma16(wh, xl, acc);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) y[r] = acc[r];
}
// y (+)= W^T g   (backward data):  y[k] = sum_o W[o][k] g[o]
__device__ __forceinline__ void mvt(const float* W, const float (&g)[16], f16v& acc, int lane) {
  const int i = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma(W[F(s, h) * LP + i], g[s], acc);
}

__device__ __forceinline__ void load_row(const float* p, int64_t row, int h, float (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float4 t = *reinterpret_cast<const float4*>(p + row * E + 8 * g + 4 * h);
    v[4 * g] = t.x; v[4 * g + 1] = t.y; v[4 * g + 2] = t.z; v[4 * g + 3] = t.w;
  }
}
__device__ __forceinline__ void store_row(float* p, int64_t row, int ld, int off, int h,
                                          const float (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(p + row * ld + off + 8 * g + 4 * h) =
        make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}

// LayerNorm over the 32 features of a token (16 in-lane + the other half-wave)
__device__ __forceinline__ void layernorm(float (&v)[16], float& rstd, float (&xh)[16]) {
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += v[r];
  s = xsum32(s);
  const float mu = s * (1.f / E);
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) { float d = v[r] - mu; q = fmaf(d, d, q); }
  q = xsum32(q);
  rstd = rsqrtf(q * (1.f / E) + 1e-5f);
#pragma unroll
  for (int r = 0; r < 16; ++r) xh[r] = (v[r] - mu) * rstd;
}
// d(LN input) from d(LN output) g (gamma already applied by caller? no: raw)
__device__ __forceinline__ void layernorm_bwd(const float (&g)[16], const float (&xh)[16],
                                              const float* gamma, float rstd, int h,
                                              float (&dv)[16]) {
  float a = 0.f, b = 0.f;
  float gg[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    gg[r] = g[r] * gamma[F(r, h)];
    a += gg[r];
    b = fmaf(gg[r], xh[r], b);
  }
  a = xsum32(a);
  b = xsum32(b);
  a *= (1.f / E);
  b *= (1.f / E);
#pragma unroll
  for (int r = 0; r < 16; ++r) dv[r] = rstd * (gg[r] - a - xh[r] * b);
}

// residual-dropout keep scales for one site, element (row, F(r,h))
__device__ __forceinline__ void drop_res(uint32_t key, int64_t row, int h, uint32_t thr,
                                         float inv_keep, float (&sc)[16]) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    uint32_t bits = rand_u32(key, (uint64_t)row * E + F(r, h));
    sc[r] = (bits & 0xffffu) >= thr ? inv_keep : 0.f;
  }
}
// the decoder tails' residual dropout: one 32-bit hash per PAIR of adjacent features
// (F(2k, h), F(2k, h) + 1), the attention kernels' two-round 24-bit-multiply hash over the
// row's key (attn_pair_bits; 16-bit decisions, p_eff = round(65536 p) / 65536): 1 row
// hash + 8 pair hashes per lane and site instead of 16 two-round 32-bit-multiply
// rand_u32.  (The encoder halves keep drop_res: the fused encoder chain matches them.)
__device__ __forceinline__ void drop_res_pairs(uint32_t key, int64_t row, int h, uint32_t thr,
                                               float inv_keep, float (&sc)[16]) {
  const uint32_t rk = attn_row_key(key, (uint32_t)row);
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    const uint32_t bits = attn_pair_bits(rk, (uint32_t)(F(r, h) >> 1));
    sc[r] = (bits & 0xffffu) >= thr ? inv_keep : 0.f;
    sc[r + 1] = (bits >> 16) >= thr ? inv_keep : 0.f;
  }
}
__device__ __forceinline__ uint32_t site_key(uint32_t key, uint32_t site) {
  return mix32(key ^ (0x632be5abu * (site + 1)));
}

__device__ __forceinline__ float gelu(float x) { return gelu_erf(x); }

// head hd's pre-dropout attention probabilities p[j] of one token over the Lc
// context tokens -- the same arithmetic, in the same order, as cross_fwd (the
// backward recomputes them instead of keeping 32 registers live)
template <int LC>
__device__ __forceinline__ void cross_probs(const float* kv, int Lc, const float (&q)[16], int h,
                                            int hd, float (&p)[LC]) {
  const float scale = 0.35355339059327373f;  // 1/sqrt(8)
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < LC; ++j) {
    float part = 0.f;
    if (j < Lc) {
      const float* kj = kv + j * 2 * E + 8 * hd + 4 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i) part = fmaf(q[4 * hd + i], kj[i], part);
    }
    part = xsum32(part);
    p[j] = j < Lc ? part * scale : -INFINITY;
    mx = fmaxf(mx, p[j]);
  }
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < LC; ++j) {
    float e = j < Lc ? __expf(p[j] - mx) : 0.f;
    p[j] = e;
    l += e;
  }
  const float il = 1.f / l;
#pragma unroll
  for (int j = 0; j < LC; ++j) p[j] *= il;
}

// cross attention of one token over the Lc context tokens (all heads):
// p[hd][j] (pre-dropout), keep bits, c (feature layout)
// have_km: keepm already holds the keep bits (stored by the forward); else hash
template <int LC>
__device__ __forceinline__ void cross_fwd(const float* kv, int Lc, const float (&q)[16], int h,
                                          uint32_t akey, int64_t row, bool drop, uint32_t thr,
                                          float inv_keep, float (&p)[H][LC], uint32_t& keepm,
                                          float (&c)[16], bool have_km = false) {
  if (!have_km) keepm = 0u;
  // keep decisions: one hash per (head, pair of context tokens) over the row's key
  const uint32_t rk = (drop && !have_km) ? attn_row_key(akey, (uint32_t)row) : 0u;
#pragma unroll
  for (int hd = 0; hd < H; ++hd) {
    cross_probs<LC>(kv, Lc, q, h, hd, p[hd]);
#pragma unroll
    for (int i = 0; i < 4; ++i) c[4 * hd + i] = 0.f;
    uint32_t pb = 0u;
#pragma unroll
    for (int j = 0; j < LC; ++j) {
      const float pj = p[hd][j];
      float pd = pj;
      if (drop && !have_km && (j & 1) == 0)
        pb = attn_pair_bits(rk, (uint32_t)(hd * (LCMAX / 2) + (j >> 1)));
      if (drop && j < Lc) {
        bool kp;
        if (have_km) {
          kp = (keepm >> (hd * LCMAX + j)) & 1u;
        } else {
          kp = ((j & 1) ? (pb >> 16) : (pb & 0xffffu)) >= thr;
          keepm |= (kp ? 1u : 0u) << (hd * LCMAX + j);
        }
        pd = kp ? pj * inv_keep : 0.f;
      } else if (!have_km) {
        keepm |= 1u << (hd * LCMAX + j);
      }
      if (j < Lc) {
        const float* vj = kv + j * 2 * E + E + 8 * hd + 4 * h;
#pragma unroll
        for (int i = 0; i < 4; ++i) c[4 * hd + i] = fmaf(pd, vj[i], c[4 * hd + i]);
      }
    }
  }
}

// ============================== forward ====================================
template <int LC, bool NEXT, bool DROP>
__global__ __launch_bounds__(NT) void dec_tail_fwd(Tail a) {
  __shared__ Smem S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int chunks = (a.L + a.chunk - 1) / a.chunk;
  const int seq = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  stage_all(S, a, NEXT);
  ctx_kv(S, a, seq);
  __syncthreads();
  const uint32_t key = DROP ? key_of(a.rng, a.call_id) : 0u;
  const int t0 = ch * a.chunk, t1 = min(a.L, t0 + a.chunk);
  // issue-early / write-late: a tile's O and x rows are loaded while the previous tile
  // finishes (before its next-block projections), not at the top of its own chain
  auto row_of = [&](int tt) {
    const int tok = tt + (lane & 31);
    return (int64_t)seq * a.L + (tok < t1 ? tok : t1 - 1);
  };
  float nO[16], nX[16];
  if (t0 + wave * 32 < t1) {
    load_row(a.O, row_of(t0 + wave * 32), h, nO);
    load_row(a.x, row_of(t0 + wave * 32), h, nX);
  }
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = row_of(tt);
    float xin[16], v[16], xh[16], rs;
#pragma unroll
    for (int r = 0; r < 16; ++r) { v[r] = nO[r]; xin[r] = nX[r]; }
    mv16(S.Wo1, S.bo1, v, v, lane);                          // a1
    uint16_t* m16 = reinterpret_cast<uint16_t*>(a.masks) + row * 8 + h;
    const bool keep_masks = DROP && a.masks != nullptr && valid;
    if (DROP) {
      float sc[16];
      drop_res_pairs(site_key(key, 0), row, h, a.thr, a.inv_keep, sc);
      uint32_t m = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; m |= (sc[r] != 0.f ? 1u : 0u) << r; }
      if (keep_masks) m16[0] = (uint16_t)m;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) xin[r] = fmaf(xh[r], S.g1[F(r, h)], S.be1[F(r, h)]);  // x1
    float q[16], c[16], p[H][LC];
    uint32_t km;
    mv16(S.Wq, S.bq, xin, q, lane);
    cross_fwd<LC>(S.kv, a.Lc, q, h, site_key(key, 3), row, DROP, a.thr, a.inv_keep, p, km, c);
    mv16(S.Wo2, S.bo2, c, v, lane);                           // a2
    if (DROP) {
      float sc[16];
      drop_res_pairs(site_key(key, 1), row, h, a.thr, a.inv_keep, sc);
      uint32_t m = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; m |= (sc[r] != 0.f ? 1u : 0u) << r; }
      if (keep_masks) { m16[2] = (uint16_t)m; if (h) a.masks[row * 4 + 3] = km; }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) xin[r] = fmaf(xh[r], S.g2[F(r, h)], S.be2[F(r, h)]);  // x2
    mv16(S.W1, S.b1, xin, v, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = gelu(v[r]);
    mv16(S.W2, S.b2, v, v, lane);                             // f
    if (DROP) {
      float sc[16];
      drop_res_pairs(site_key(key, 2), row, h, a.thr, a.inv_keep, sc);
      uint32_t m = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; m |= (sc[r] != 0.f ? 1u : 0u) << r; }
      if (keep_masks) m16[4] = (uint16_t)m;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaf(xh[r], S.g3[F(r, h)], S.be3[F(r, h)]);    // y
    if (valid) store_row(a.y, row, E, 0, h, v);
    if (tt + NW * 32 < t1) {
      load_row(a.O, row_of(tt + NW * 32), h, nO);
      load_row(a.x, row_of(tt + NW * 32), h, nX);
    }
    if (NEXT) {
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float o[16];
        mv16(S.Wn + cc * E * LP, S.bn + cc * E, v, o, lane);
        if (valid) store_row(a.qkv, row, 3 * E, cc * E, h, o);
      }
    }
  }
}

// ============================== backward ===================================
// Phase (a), dec_tail_bwd_data: per token, recompute the forward, run the chain
// in reverse, write dx / dO and the per-token vectors the weight gradients need
// into a scratch buffer laid out [vector][M][32] (SoA, coalesced rows).
// Phase (b), dec_tail_wgrad: per workgroup (one sequence chunk) contract those
// vectors over tokens with MFMAs -> per-workgroup partials -> column sums.
enum Vec {
  V_DA1 = 0, V_DQ, V_DA2, V_DF1, V_DF2, V_X1, V_C, V_X2, V_GL,
  V_DLN1, V_DLN1X, V_DLN2, V_DLN2X, V_DLN3, V_DLN3X, V_Q, V_DC, V_DS, V_PD, NVEC
};

// a wave's 16-float-per-lane row parked in LDS ([16][64], lane-contiguous:
// conflict-free); the asm memory clobber keeps the compiler from forwarding the
// value in registers, which is the point
__device__ __forceinline__ void park(float (*slot)[64], const float (&v)[16], int lane) {
#pragma unroll
  for (int r = 0; r < 16; ++r) slot[r][lane] = v[r];
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void unpark(float (*slot)[64], float (&v)[16], int lane) {
  asm volatile("" ::: "memory");
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = slot[r][lane];
}

// MASKS: the forward's stored keep masks are read (else re-hashed; compiled
// apart so the common path carries no registers for the other).  Two waves per
// SIMD: the MASKS path fits 256 registers without spills (one wave per SIMD
// left every LDS / MFMA / memory latency exposed).
template <int LC, bool NEXT, bool DROP, bool MASKS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void dec_tail_bwd_data(Tail a, float* __restrict__ scr) {
  __shared__ Smem S;
  __shared__ float Pk[NW][2][16][64];   // parked LN1 / LN2 normalised inputs
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int chunks = (a.L + a.chunk - 1) / a.chunk;
  const int seq = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  stage_all(S, a, NEXT);
  ctx_kv(S, a, seq);
  __syncthreads();
  const uint32_t key = DROP ? key_of(a.rng, a.call_id) : 0u;
  const float scale = 0.35355339059327373f;
  const int64_t MS = (int64_t)a.M * E;   // stride between scratch vectors
  auto SV = [&](int v) { return scr + v * MS; };
  const int t0 = ch * a.chunk, t1 = min(a.L, t0 + a.chunk);
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = (int64_t)seq * a.L + (valid ? tok : t1 - 1);
    // ---------------- forward recompute -----------------
    float xh1[16], xh2[16], xh3[16], f1[16];
    float rs1, rs2, rs3;
    uint32_t km, k0 = 0xffffffffu, k1 = 0xffffffffu, k2 = 0xffffffffu;
    constexpr bool have = DROP && MASKS;   // masks stored by the forward
    if (have) {
      const uint4 mw = *reinterpret_cast<const uint4*>(a.masks + row * 4);
      const int sh = 16 * h;
      k0 = (mw.x >> sh) & 0xffffu;
      k1 = (mw.y >> sh) & 0xffffu;
      k2 = (mw.z >> sh) & 0xffffu;
      km = mw.w;
    }
    {
      float v[16], t[16], q[16], c[16], p[H][LC];
      load_row(a.O, row, h, t);
      mv16(S.Wo1, S.bo1, t, v, lane);
      load_row(a.x, row, h, t);
      if (DROP && have) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= ((k0 >> r) & 1u) ? a.inv_keep : 0.f;
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 0), row, h, a.thr, a.inv_keep, sc);
        k0 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k0 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs1, xh1);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = fmaf(xh1[r], S.g1[F(r, h)], S.be1[F(r, h)]);   // x1
      // forward values the weight gradients need go to the scratch as soon as they
      // exist, the normalised LN inputs wait in LDS (short live ranges: this kernel
      // is register-bound)
      if (valid) store_row(SV(V_X1), row, E, 0, h, t);
      park(Pk[wave][0], xh1, lane);
      mv16(S.Wq, S.bq, t, q, lane);
      if (valid) store_row(SV(V_Q), row, E, 0, h, q);
      cross_fwd<LC>(S.kv, a.Lc, q, h, site_key(key, 3), row, DROP, a.thr, a.inv_keep, p, km, c,
                    have);
      if (valid) store_row(SV(V_C), row, E, 0, h, c);
      mv16(S.Wo2, S.bo2, c, v, lane);
      if (DROP && have) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= ((k1 >> r) & 1u) ? a.inv_keep : 0.f;
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 1), row, h, a.thr, a.inv_keep, sc);
        k1 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k1 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs2, xh2);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = fmaf(xh2[r], S.g2[F(r, h)], S.be2[F(r, h)]);   // x2
      if (valid) store_row(SV(V_X2), row, E, 0, h, t);
      park(Pk[wave][1], xh2, lane);
      mv16(S.W1, S.b1, t, f1, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = gelu(f1[r]);
      if (valid) store_row(SV(V_GL), row, E, 0, h, v);
      mv16(S.W2, S.b2, v, v, lane);
      if (DROP && have) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= ((k2 >> r) & 1u) ? a.inv_keep : 0.f;
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 2), row, h, a.thr, a.inv_keep, sc);
        k2 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k2 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs3, xh3);
    }
    const float ik = DROP ? a.inv_keep : 1.f;
    // ---------------- backward -----------------
    float d[16];
    load_row(a.dy, row, h, d);
    if (NEXT) {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float g3[16];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float4 t = *reinterpret_cast<const float4*>(a.dqkv + row * 3 * E + cc * E + 8 * g4 + 4 * h);
          g3[4 * g4] = t.x; g3[4 * g4 + 1] = t.y; g3[4 * g4 + 2] = t.z; g3[4 * g4 + 3] = t.w;
        }
        mvt(S.Wn + cc * E * LP, g3, acc, lane);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];
    }
    float t[16];
    // LN3
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh3[r];
    if (valid) { store_row(SV(V_DLN3), row, E, 0, h, d); store_row(SV(V_DLN3X), row, E, 0, h, t); }
    layernorm_bwd(d, xh3, S.g3, rs3, h, d);                 // dv3 (residual into x2)
    // FFN
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k2 >> r) & 1u) ? d[r] * ik : 0.f;   // df2
    if (valid) store_row(SV(V_DF2), row, E, 0, h, t);
    {
      f16v acc = {};
      mvt(S.W2, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = acc[r] * gelu_erf_grad(f1[r]);   // df1
    }
    if (valid) store_row(SV(V_DF1), row, E, 0, h, t);
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.W1, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx2
    }
    // LN2
    unpark(Pk[wave][1], xh2, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh2[r];
    if (valid) { store_row(SV(V_DLN2), row, E, 0, h, d); store_row(SV(V_DLN2X), row, E, 0, h, t); }
    layernorm_bwd(d, xh2, S.g2, rs2, h, d);                 // dv2 (residual into x1)
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k1 >> r) & 1u) ? d[r] * ik : 0.f;   // da2
    if (valid) store_row(SV(V_DA2), row, E, 0, h, t);
    float dc[16];
    {
      f16v acc = {};
      mvt(S.Wo2, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) dc[r] = acc[r];
    }
    if (valid) store_row(SV(V_DC), row, E, 0, h, dc);
    // cross attention backward (dq -> reuse t)
    {
      // this half-wave's share of the ds / pd rows: k = 4j + hd for j in [4h, 4h + 4)
      float dsv[16], pdv[16], q[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) { dsv[k] = 0.f; pdv[k] = 0.f; }
      load_row(SV(V_Q), row, h, q);   // this lane's own store (invalid lanes: unused)
#pragma unroll
      for (int hd = 0; hd < H; ++hd) {
        float dp[LC], ph[LC];
        cross_probs<LC>(S.kv, a.Lc, q, h, hd, ph);
        float Dsum = 0.f;
#pragma unroll
        for (int j = 0; j < LC; ++j) {
          float part = 0.f;
          if (j < a.Lc) {
            const float* vj = S.kv + j * 2 * E + E + 8 * hd + 4 * h;
#pragma unroll
            for (int i = 0; i < 4; ++i) part = fmaf(dc[4 * hd + i], vj[i], part);
          }
          part = xsum32(part);
          const bool kp = (km >> (hd * LCMAX + j)) & 1u;
          dp[j] = (j < a.Lc && kp) ? part * ik : 0.f;
          if ((j >> 2) == h) pdv[4 * (j & 3) + hd] = (j < a.Lc && kp) ? ph[j] * ik : 0.f;
          Dsum = fmaf(ph[j], dp[j], Dsum);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) t[4 * hd + i] = 0.f;
#pragma unroll
        for (int j = 0; j < LC; ++j) {
          const float ds = j < a.Lc ? ph[j] * (dp[j] - Dsum) * scale : 0.f;
          if ((j >> 2) == h) dsv[4 * (j & 3) + hd] = ds;
          if (j < a.Lc) {
            const float* kj = S.kv + j * 2 * E + 8 * hd + 4 * h;
#pragma unroll
            for (int i = 0; i < 4; ++i) t[4 * hd + i] = fmaf(ds, kj[i], t[4 * hd + i]);
          }
        }
      }
      // ds / pd rows: half h writes k in [16h, 16h + 16)
      if (valid) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int k = 4 * g4;
          *reinterpret_cast<float4*>(SV(V_DS) + row * E + 16 * h + k) =
              make_float4(dsv[k], dsv[k + 1], dsv[k + 2], dsv[k + 3]);
          *reinterpret_cast<float4*>(SV(V_PD) + row * E + 16 * h + k) =
              make_float4(pdv[k], pdv[k + 1], pdv[k + 2], pdv[k + 3]);
        }
      }
    }
    if (valid) store_row(SV(V_DQ), row, E, 0, h, t);
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.Wq, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx1
    }
    // LN1
    unpark(Pk[wave][0], xh1, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh1[r];
    if (valid) { store_row(SV(V_DLN1), row, E, 0, h, d); store_row(SV(V_DLN1X), row, E, 0, h, t); }
    layernorm_bwd(d, xh1, S.g1, rs1, h, d);                 // dv1 = dx
    if (valid) store_row(a.dx, row, E, 0, h, d);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k0 >> r) & 1u) ? d[r] * ik : 0.f;   // da1
    if (valid) store_row(SV(V_DA1), row, E, 0, h, t);
    {
      f16v acc = {};
      mvt(S.Wo1, t, acc, lane);
      float dO[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) dO[r] = acc[r];
      if (valid) store_row(a.dO, row, E, 0, h, dO);
    }
  }
}

// ============================ encoder halves ================================
__device__ __forceinline__ void stage_pre(Smem& S, const Tail& a) {
  float w0[MW], w1[MW];
  load_w<E>(a.Wo1, w0); load_w<E>(a.Wq, w1);
  stage_vecs<4>({S.bo1, S.bq, S.g1, S.be1}, {a.bo1, a.bq, a.g1, a.be1}, E);
  store_w<E>(S.Wo1, w0); store_w<E>(S.Wq, w1);
}
__device__ __forceinline__ void stage_post(Smem& S, const Tail& a, bool next) {
  float w2[MW], w3[MW], w4[MW], wn[3 * MW];
  load_w<E>(a.Wo2, w2); load_w<E>(a.W1, w3); load_w<E>(a.W2, w4);
  if (next) load_w<3 * E>(a.Wn, wn);
  stage_vecs<7>({S.bo2, S.b1, S.b2, S.g2, S.be2, S.g3, S.be3},
                {a.bo2, a.b1, a.b2, a.g2, a.be2, a.g3, a.be3}, E);
  if (next) stage_vecs<1>({S.bn}, {a.bn}, 3 * E);
  store_w<E>(S.Wo2, w2); store_w<E>(S.W1, w3); store_w<E>(S.W2, w4);
  if (next) store_w<3 * E>(S.Wn, wn);
}

// residual dropout of one site: v *= keep / (1 - p); keep bits recorded in m16[slot]
template <bool DROP>
__device__ __forceinline__ void drop_site_fwd(float (&v)[16], uint32_t key, int site, int64_t row,
                                              int h, const Tail& a, uint16_t* m16, int slot,
                                              bool keep_masks) {
  if (!DROP) return;
  float sc[16];
  drop_res(site_key(key, site), row, h, a.thr, a.inv_keep, sc);
  uint32_t m = 0u;
#pragma unroll
  for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; m |= (sc[r] != 0.f ? 1u : 0u) << r; }
  if (keep_masks) m16[slot] = (uint16_t)m;
}

template <bool DROP>
__global__ __launch_bounds__(NT) void enc_pre_fwd(Tail a) {
  __shared__ Smem S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  stage_pre(S, a);
  __syncthreads();
  const uint32_t key = DROP ? key_of(a.rng, a.call_id) : 0u;
  const int t0 = blockIdx.x * a.chunk, t1 = min(a.M, t0 + a.chunk);
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = valid ? tok : t1 - 1;
    float xin[16], v[16], xh[16], rs;
    load_row(a.O, row, h, v);
    mv(S.Wo1, S.bo1, v, v, lane);                          // a1
    load_row(a.x, row, h, xin);
    uint16_t* m16 = reinterpret_cast<uint16_t*>(a.masks) + row * 8 + h;
    drop_site_fwd<DROP>(v, key, 0, row, h, a, m16, 0, DROP && a.masks != nullptr && valid);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) xin[r] = fmaf(xh[r], S.g1[F(r, h)], S.be1[F(r, h)]);  // x1
    if (valid) store_row(a.y, row, E, 0, h, xin);
    mv(S.Wq, S.bq, xin, v, lane);                           // q
    if (valid) store_row(a.qkv, row, E, 0, h, v);
  }
}

template <bool NEXT, bool DROP>
__global__ __launch_bounds__(NT) void enc_post_fwd(Tail a) {
  __shared__ Smem S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  stage_post(S, a, NEXT);
  __syncthreads();
  const uint32_t key = DROP ? key_of(a.rng, a.call_id) : 0u;
  const int t0 = blockIdx.x * a.chunk, t1 = min(a.M, t0 + a.chunk);
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = valid ? tok : t1 - 1;
    float xin[16], v[16], xh[16], rs;
    const bool km = DROP && a.masks != nullptr && valid;
    uint16_t* m16 = reinterpret_cast<uint16_t*>(a.masks) + row * 8 + h;
    load_row(a.O, row, h, v);
    mv(S.Wo2, S.bo2, v, v, lane);                           // a2
    load_row(a.x, row, h, xin);                             // x1
    drop_site_fwd<DROP>(v, key, 1, row, h, a, m16, 2, km);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) xin[r] = fmaf(xh[r], S.g2[F(r, h)], S.be2[F(r, h)]);  // x2
    mv(S.W1, S.b1, xin, v, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = gelu(v[r]);
    mv(S.W2, S.b2, v, v, lane);                             // f
    drop_site_fwd<DROP>(v, key, 2, row, h, a, m16, 4, km);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += xin[r];
    layernorm(v, rs, xh);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaf(xh[r], S.g3[F(r, h)], S.be3[F(r, h)]);    // y
    if (valid) store_row(a.y, row, E, 0, h, v);
    if (NEXT) {
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float o[16];
        mv(S.Wn + cc * E * LP, S.bn + cc * E, v, o, lane);
        if (valid) store_row(a.qkv, row, 3 * E, cc * E, h, o);
      }
    }
  }
}

// keep bits of one residual site (16 per half) from the forward's stored words
__device__ __forceinline__ uint32_t site_mask(const Tail& a, int64_t row, int word, int h) {
  return (a.masks[row * 4 + word] >> (16 * h)) & 0xffffu;
}
template <bool DROP>
__device__ __forceinline__ void drop_apply(float (&v)[16], uint32_t k, float ik) {
  if (!DROP) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] *= ((k >> r) & 1u) ? ik : 0.f;
}

// PRE backward: dy = d x1 (from POST and the residual), dqkv = d q [M, 32];
// writes dx, dO and the scratch vectors of Wo1 / Wq / LN1
template <bool DROP>
__global__ __launch_bounds__(NT) void enc_pre_bwd_data(Tail a, float* __restrict__ scr) {
  __shared__ Smem S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  stage_pre(S, a);
  __syncthreads();
  const int64_t MS = (int64_t)a.M * E;
  auto SV = [&](int v) { return scr + v * MS; };
  const float ik = DROP ? a.inv_keep : 1.f;
  const int t0 = blockIdx.x * a.chunk, t1 = min(a.M, t0 + a.chunk);
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = valid ? tok : t1 - 1;
    const uint32_t k0 = DROP ? site_mask(a, row, 0, h) : 0xffffu;
    float v[16], t[16], xh1[16], rs1;
    load_row(a.O, row, h, t);
    mv(S.Wo1, S.bo1, t, v, lane);
    drop_apply<DROP>(v, k0, a.inv_keep);
    load_row(a.x, row, h, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += t[r];
    layernorm(v, rs1, xh1);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = fmaf(xh1[r], S.g1[F(r, h)], S.be1[F(r, h)]);   // x1
    if (valid) store_row(SV(V_X1), row, E, 0, h, t);
    float d[16];
    load_row(a.dy, row, h, d);
    load_row(a.dqkv, row, h, t);                            // dq
    if (valid) store_row(SV(V_DQ), row, E, 0, h, t);
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.Wq, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx1
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh1[r];
    if (valid) { store_row(SV(V_DLN1), row, E, 0, h, d); store_row(SV(V_DLN1X), row, E, 0, h, t); }
    layernorm_bwd(d, xh1, S.g1, rs1, h, d);                 // dx
    if (valid) store_row(a.dx, row, E, 0, h, d);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k0 >> r) & 1u) ? d[r] * ik : 0.f;   // da1
    if (valid) store_row(SV(V_DA1), row, E, 0, h, t);
    f16v acc = {};
    mvt(S.Wo1, t, acc, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = acc[r];
    if (valid) store_row(a.dO, row, E, 0, h, v);
  }
}

// POST backward: dy = d y, dqkv = d qkv_next [M, 96] (NEXT); writes dx = d x1,
// dO = d c and the scratch vectors of Wo2 / W1 / W2 / LN2 / LN3
template <bool NEXT, bool DROP>
__global__ __launch_bounds__(NT) void enc_post_bwd_data(Tail a, float* __restrict__ scr) {
  __shared__ Smem S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  stage_post(S, a, NEXT);
  __syncthreads();
  const int64_t MS = (int64_t)a.M * E;
  auto SV = [&](int v) { return scr + v * MS; };
  const float ik = DROP ? a.inv_keep : 1.f;
  const int t0 = blockIdx.x * a.chunk, t1 = min(a.M, t0 + a.chunk);
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < t1;
    const int64_t row = valid ? tok : t1 - 1;
    const uint32_t k1 = DROP ? site_mask(a, row, 1, h) : 0xffffu;
    const uint32_t k2 = DROP ? site_mask(a, row, 2, h) : 0xffffu;
    float v[16], t[16], xh2[16], xh3[16], f1[16], rs2, rs3;
    load_row(a.O, row, h, t);
    mv(S.Wo2, S.bo2, t, v, lane);
    drop_apply<DROP>(v, k1, a.inv_keep);
    load_row(a.x, row, h, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += t[r];
    layernorm(v, rs2, xh2);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = fmaf(xh2[r], S.g2[F(r, h)], S.be2[F(r, h)]);   // x2
    if (valid) store_row(SV(V_X2), row, E, 0, h, t);
    mv(S.W1, S.b1, t, f1, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = gelu(f1[r]);
    if (valid) store_row(SV(V_GL), row, E, 0, h, v);
    mv(S.W2, S.b2, v, v, lane);
    drop_apply<DROP>(v, k2, a.inv_keep);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += t[r];
    layernorm(v, rs3, xh3);
    float d[16];
    load_row(a.dy, row, h, d);
    if (NEXT) {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float g3[16];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float4 q4 = *reinterpret_cast<const float4*>(a.dqkv + row * 3 * E + cc * E + 8 * g4 + 4 * h);
          g3[4 * g4] = q4.x; g3[4 * g4 + 1] = q4.y; g3[4 * g4 + 2] = q4.z; g3[4 * g4 + 3] = q4.w;
        }
        mvt(S.Wn + cc * E * LP, g3, acc, lane);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh3[r];
    if (valid) { store_row(SV(V_DLN3), row, E, 0, h, d); store_row(SV(V_DLN3X), row, E, 0, h, t); }
    layernorm_bwd(d, xh3, S.g3, rs3, h, d);                 // dv3 (residual into x2)
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k2 >> r) & 1u) ? d[r] * ik : 0.f;   // df2
    if (valid) store_row(SV(V_DF2), row, E, 0, h, t);
    {
      f16v acc = {};
      mvt(S.W2, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = acc[r] * gelu_erf_grad(f1[r]);   // df1
    }
    if (valid) store_row(SV(V_DF1), row, E, 0, h, t);
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.W1, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx2
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh2[r];
    if (valid) { store_row(SV(V_DLN2), row, E, 0, h, d); store_row(SV(V_DLN2X), row, E, 0, h, t); }
    layernorm_bwd(d, xh2, S.g2, rs2, h, d);                 // dx1
    if (valid) store_row(a.dx, row, E, 0, h, d);
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = ((k1 >> r) & 1u) ? d[r] * ik : 0.f;   // da2
    if (valid) store_row(SV(V_DA2), row, E, 0, h, t);
    f16v acc = {};
    mvt(S.Wo2, t, acc, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = acc[r];
    if (valid) store_row(a.dO, row, E, 0, h, v);               // dc
  }
}

// gradient partial layout per workgroup (floats)
// gradient layout (slabs and gflat alike).  The cross in_proj region holds all
// 3E rows [Wq; Wk; Wv] (and 3E biases): the tail writes rows [0, E), the
// context k | v projection's weight gradient writes rows [E, 3E) in place, so
// the whole in_proj gradient is one view of gflat.
constexpr int OFF_WO1 = 0, OFF_WQ = 1024, OFF_WO2 = 4096, OFF_W1 = 5120, OFF_W2 = 6144,
              OFF_WN = 7168, OFF_BO1 = 10240, OFF_BQ = 10272, OFF_BO2 = 10368, OFF_B1 = 10400,
              OFF_B2 = 10432, OFF_BN = 10464, OFF_G1 = 10560, OFF_BE1 = 10592, OFF_G2 = 10624,
              OFF_BE2 = 10656, OFF_G3 = 10688, OFF_BE3 = 10720, WPART = 10752;

// acc[o][k] += sum_t G[t][o] X[t][k] over the wave's 32 tokens (rows r0..r0+31,
// rows >= rmax contribute 0); operands read straight from L2 / HBM, all 32 loads
// issued before the MFMAs; returns this lane's share of the column sum of G
// (rows of parity h; the caller adds the other half-wave)
__device__ __forceinline__ float wg_tile(const float* G, int ldg, const float* X, int ldx,
                                         int64_t r0, int64_t rmax, f16v& acc, int lane) {
  const int c = lane & 31, h = lane >> 5;
  float g[16], x[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int64_t t = min(r0 + 2 * s + h, rmax - 1);
    g[s] = G[t * ldg + c];
    x[s] = X[t * ldx + c];
  }
  float cs = 0.f;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const bool ok = r0 + 2 * s + h < rmax;
    const float gg = ok ? g[s] : 0.f;
    cs += gg;
    acc = mfma(gg, ok ? x[s] : 0.f, acc);
  }
  return cs;
}
__device__ __forceinline__ float cs_tile(const float* G, int ldg, int64_t r0, int64_t rmax,
                                         int lane) {
  const int c = lane & 31, h = lane >> 5;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = G[min(r0 + 16 * h + i, rmax - 1) * ldg + c];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += r0 + 16 * h + i < rmax ? v[i] : 0.f;
  return s;
}

// one workgroup per (job, sequence chunk); job = which weight matrix (or the
// LayerNorm vectors, or the context k / v gradients).  A single accumulator per
// wave keeps occupancy high so the streamed operand loads overlap.
enum Job { J_WO1 = 0, J_WQ, J_WO2, J_W1, J_W2, J_WN0, J_WN1, J_WN2, J_K, J_V, J_LN, NJOB };

__global__ __launch_bounds__(NT) void dec_tail_wgrad(Tail a, const float* __restrict__ scr, int job0) {
  __shared__ float red[NW * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int job = blockIdx.y + job0;
  const bool next = a.Wn != nullptr;
  if (!next && job >= J_WN0 && job <= J_WN2) return;
  if (a.mode != MODE_FULL) {
    // encoder halves: no context gradients; the other half's matrices are not
    // computed (their gflat regions are neither summed nor written)
    if (job == J_K || job == J_V) return;
    const bool mine = a.mode == MODE_PRE ? (job == J_WO1 || job == J_WQ || job == J_LN)
                                         : !(job == J_WO1 || job == J_WQ);
    if (!mine) return;
  }
  const int chunks = (a.L + a.chunk - 1) / a.chunk;
  const int seq = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  // context (k, v) gradients are per sequence: the sequence's first workgroup
  // covers all its chunks and writes dkvc directly (no cross-workgroup sum)
  const bool ctx_job = job == J_K || job == J_V;
  if (ctx_job && ch != 0) return;
  const int64_t MS = (int64_t)a.M * E;
  const float* Gm = nullptr;
  const float* X = nullptr;
  int ldg = E;
  int boff = -1, moff = -1;
  switch (job) {
    case J_WO1: Gm = scr + V_DA1 * MS; X = a.O; moff = OFF_WO1; boff = OFF_BO1; break;
    case J_WQ: Gm = scr + V_DQ * MS; X = scr + V_X1 * MS; moff = OFF_WQ; boff = OFF_BQ; break;
    case J_WO2:   // POST reads c straight from its input (no V_C copy)
      Gm = scr + V_DA2 * MS; X = a.mode == MODE_POST ? a.O : scr + V_C * MS;
      moff = OFF_WO2; boff = OFF_BO2; break;
    case J_W1: Gm = scr + V_DF1 * MS; X = scr + V_X2 * MS; moff = OFF_W1; boff = OFF_B1; break;
    case J_W2: Gm = scr + V_DF2 * MS; X = scr + V_GL * MS; moff = OFF_W2; boff = OFF_B2; break;
    case J_WN0: case J_WN1: case J_WN2: {
      const int c = job - J_WN0;
      Gm = a.dqkv + c * E; ldg = 3 * E; X = a.y; moff = OFF_WN + 1024 * c; boff = OFF_BN + 32 * c;
      break;
    }
    case J_K: Gm = scr + V_Q * MS; X = scr + V_DS * MS; break;
    case J_V: Gm = scr + V_DC * MS; X = scr + V_PD * MS; break;
    default: break;
  }
  const int t0 = ctx_job ? 0 : ch * a.chunk, t1 = ctx_job ? a.L : min(a.L, t0 + a.chunk);
  const int64_t base = (int64_t)seq * a.L, rmax = base + t1;
  float* out = a.wpart + (int64_t)blockIdx.x * WPART;   // == gflat when the grid is one workgroup
  if (job == J_LN) {
    const int voff[6] = {V_DLN1X, V_DLN1, V_DLN2X, V_DLN2, V_DLN3X, V_DLN3};
    const int ooff[6] = {OFF_G1, OFF_BE1, OFF_G2, OFF_BE2, OFF_G3, OFF_BE3};
    float cs[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32)
#pragma unroll
      for (int i = 0; i < 6; ++i)   // PRE holds LN1 only, POST LN2 / LN3
        if (a.mode == MODE_FULL || (a.mode == MODE_PRE) == (i < 2))
          cs[i] += cs_tile(scr + voff[i] * MS, E, base + tt, rmax, lane);
#pragma unroll
    for (int i = 0; i < 6; ++i) red[i * 256 + threadIdx.x] = cs[i];
    __syncthreads();
    if (threadIdx.x < 6 * 32) {
      const int i = threadIdx.x / 32, c = threadIdx.x % 32;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[i * 256 + w * 64 + c] + red[i * 256 + w * 64 + 32 + c];
      if (a.mode == MODE_FULL || (a.mode == MODE_PRE) == (i < 2)) out[ooff[i] + c] = sum;
    }
    return;
  }
  f16v acc = {};
  float cs = 0.f;
#pragma unroll 2
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32)
    cs += wg_tile(Gm, ldg, X, E, base + tt, rmax, acc, lane);
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave * 1024 + F(r, h) * 32 + (lane & 31)] = acc[r];
  __syncthreads();
  if (ctx_job) {
    // acc[f = F(r,h)][j' = lane&31] is valid where (j' & 3) == f >> 3, j = j' >> 2 < Lc
    float* dk = a.dkvc + (int64_t)seq * a.Lc * 2 * E + (job == J_V ? E : 0);
    for (int i = threadIdx.x; i < a.Lc * E; i += NT) {
      const int j = i / E, f = i % E;
      const int idx = f * 32 + 4 * j + (f >> 3);
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w * 1024 + idx];
      dk[j * 2 * E + f] = sum;
    }
    return;
  }
  for (int i = threadIdx.x; i < 1024; i += NT)
    out[moff + i] = ((red[i] + red[1024 + i]) + red[2048 + i]) + red[3072 + i];
  __syncthreads();
  red[threadIdx.x] = cs;
  __syncthreads();
  if (threadIdx.x < 32) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += red[w * 64 + threadIdx.x] + red[w * 64 + 32 + threadIdx.x];
    out[boff + threadIdx.x] = sum;
  }
}

// The next block's in_proj gradient (dqkv^T y over the tokens: inputs only) beside the fused
// backward: the three 32-row slices of one workgroup's tokens together, so each y row is read
// once (dec_tail_wgrad's J_WN0..2 jobs read it three times); per slice the same tiles in the
// same order as those jobs (the same sums).
__global__ __launch_bounds__(NT) void dec_tail_wgrad_wn(Tail a) {
  __shared__ float red[NW * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, c = lane & 31;
  const int chunks = (a.L + a.chunk - 1) / a.chunk;
  const int seq = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const int t0 = ch * a.chunk, t1 = min(a.L, t0 + a.chunk);
  const int64_t base = (int64_t)seq * a.L, rmax = base + t1;
  float* out = a.wpart + (int64_t)blockIdx.x * WPART;
  f16v acc[3] = {{}, {}, {}};
  float cs[3] = {0.f, 0.f, 0.f};
  for (int tt = t0 + wave * 32; tt < t1; tt += NW * 32) {   // 64 loads per lane in flight a tile
    const int64_t r0 = base + tt;
    float g[3][16], x[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int64_t t = min(r0 + 2 * s + h, rmax - 1);
      x[s] = a.y[t * E + c];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) g[cc][s] = a.dqkv[t * 3 * E + cc * E + c];
    }
#pragma unroll
    for (int cc = 0; cc < 3; ++cc)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const bool ok = r0 + 2 * s + h < rmax;
        const float gg = ok ? g[cc][s] : 0.f;
        cs[cc] += gg;
        acc[cc] = mfma(gg, ok ? x[s] : 0.f, acc[cc]);
      }
  }
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave * 1024 + F(r, h) * 32 + c] = acc[cc][r];
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += NT)
      out[OFF_WN + 1024 * cc + i] = ((red[i] + red[1024 + i]) + red[2048 + i]) + red[3072 + i];
    __syncthreads();
    red[threadIdx.x] = cs[cc];
    __syncthreads();
    if (threadIdx.x < 32) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w * 64 + threadIdx.x] + red[w * 64 + 32 + threadIdx.x];
      out[OFF_BN + 32 * cc + threadIdx.x] = sum;
    }
    __syncthreads();
  }
}

// ======================= fused backward (long sequences) =====================
// One workgroup per sequence runs dec_tail_bwd_data's chain per 32-token tile and
// does every weight-gradient contraction in place, instead of writing 19
// per-token scratch vectors (~2.4 KB per token, ~0.6 GB per spectra layer) for
// dec_tail_wgrad to read back: each vector is transposed through a per-wave LDS
// tile into the MFMA operand layout (lane = feature, k = token) and contracted
// into accumulators that live for the whole sequence (7 matrices x 16 plus 11
// column sums per lane: one wave per SIMD, 512 registers).  The workgroup's
// partials go to the usual partial row / column sums; the context k | v gradient
// is complete per workgroup and written directly.  The next block's in_proj
// gradient (dqkv^T y: inputs only) stays with dec_tail_wgrad's jobs.
constexpr int LT = 33;        // LDS tile row stride (floats)
constexpr int TILE = 32 * LT;

// token-major tile: lane (t, h) stores its feature-layout values of token t
__device__ __forceinline__ void put_fl(float* tile, const float (&v)[16], int lane) {
  const int t = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) tile[t * LT + F(r, h)] = v[r];
}
// rows whose half h holds columns [16h, 16h + 16) in order (cross-attention ds / pd)
__device__ __forceinline__ void put_half(float* tile, const float (&v)[16], int lane) {
  const int t = lane & 31, h = lane >> 5;
#pragma unroll
  for (int k = 0; k < 16; ++k) tile[t * LT + 16 * h + k] = v[k];
}
// MFMA operand layout: lane (c, h) reads column c of tokens 2s + h
__device__ __forceinline__ void get_op(const float* tile, float (&o)[16], int lane) {
  const int c = lane & 31, h = lane >> 5;
  asm volatile("" ::: "memory");
#pragma unroll
  for (int s = 0; s < 16; ++s) o[s] = tile[(2 * s + h) * LT + c];
}
__device__ __forceinline__ void contract(f16v& acc, const float (&g)[16], const float (&x)[16],
                                         float& cs) {
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    cs += g[s];
    acc = mfma(g[s], x[s], acc);
  }
}
__device__ __forceinline__ void colsum_tile(float* tile, const float (&v)[16], int lane, float& cs) {
  put_fl(tile, v, lane);
  float o[16];
  get_op(tile, o, lane);
#pragma unroll
  for (int s = 0; s < 16; ++s) cs += o[s];
  asm volatile("" ::: "memory");
}
template <int LC, bool NEXT, bool DROP, bool MASKS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) void dec_tail_bwd_fused(Tail a) {
  __shared__ Smem S;
  __shared__ float Lt[NW][7 * TILE];   // per wave: X1, C / dC, X2, GL, Q, transient, O
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  const int seq = blockIdx.x;
  stage_all(S, a, NEXT);
  ctx_kv(S, a, seq);
  __syncthreads();
  float* tX1 = Lt[wave];
  float* tC = tX1 + TILE;
  float* tX2 = tC + TILE;
  float* tGL = tX2 + TILE;
  float* tQ = tGL + TILE;
  float* tT = tQ + TILE;
  float* tO = tT + TILE;      // the attention output rows, for the out-projection's dW
  const uint32_t key = DROP ? key_of(a.rng, a.call_id) : 0u;
  const float scale = 0.35355339059327373f;
  const float ik = DROP ? a.inv_keep : 1.f;
  f16v aWO1 = {}, aWQ = {}, aWO2 = {}, aW1 = {}, aW2 = {}, aK = {}, aV = {};
  float cBO1 = 0.f, cBQ = 0.f, cBO2 = 0.f, cB1 = 0.f, cB2 = 0.f;
  float cG1 = 0.f, cBE1 = 0.f, cG2 = 0.f, cBE2 = 0.f, cG3 = 0.f, cBE3 = 0.f;
  const int64_t base = (int64_t)seq * a.L;
  for (int tt = wave * 32; tt < a.L; tt += NW * 32) {
    const int tok = tt + (lane & 31);
    const bool valid = tok < a.L;
    const int64_t row = base + (valid ? tok : a.L - 1);
    // ---------------- forward recompute -----------------
    float xh1[16], xh2[16], xh3[16], f1[16], q[16];
    float rs1, rs2, rs3;
    uint32_t km, k0 = 0xffffffffu, k1 = 0xffffffffu, k2 = 0xffffffffu;
    constexpr bool have = DROP && MASKS;
    if (have) {
      const uint4 mw = *reinterpret_cast<const uint4*>(a.masks + row * 4);
      const int sh = 16 * h;
      k0 = (mw.x >> sh) & 0xffffu;
      k1 = (mw.y >> sh) & 0xffffu;
      k2 = (mw.z >> sh) & 0xffffu;
      km = mw.w;
    }
    {
      float v[16], t[16], c[16], p[H][LC], xr[16];
      load_row(a.O, row, h, t);
      load_row(a.x, row, h, xr);   // in flight with O's row (one HBM round trip)
      put_fl(tO, t, lane);    // read back at the tile's end (the dW_o1 operand): LDS, not HBM
      mv16(S.Wo1, S.bo1, t, v, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = xr[r];
      if (DROP && have) {
        const uint32_t kk = opaque(k0);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= keep_sc(kk, r, a.inv_keep);
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 0), row, h, a.thr, a.inv_keep, sc);
        k0 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k0 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs1, xh1);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = fmaf(xh1[r], S.g1[F(r, h)], S.be1[F(r, h)]);   // x1
      put_fl(tX1, t, lane);
      mv16(S.Wq, S.bq, t, q, lane);
      put_fl(tQ, q, lane);
      cross_fwd<LC>(S.kv, a.Lc, q, h, site_key(key, 3), row, DROP, a.thr, a.inv_keep, p, km, c,
                    have);
      put_fl(tC, c, lane);
      mv16(S.Wo2, S.bo2, c, v, lane);
      if (DROP && have) {
        const uint32_t kk = opaque(k1);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= keep_sc(kk, r, a.inv_keep);
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 1), row, h, a.thr, a.inv_keep, sc);
        k1 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k1 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs2, xh2);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = fmaf(xh2[r], S.g2[F(r, h)], S.be2[F(r, h)]);   // x2
      put_fl(tX2, t, lane);
      mv16(S.W1, S.b1, t, f1, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = gelu(f1[r]);
      put_fl(tGL, v, lane);
      mv16(S.W2, S.b2, v, v, lane);
      if (DROP && have) {
        const uint32_t kk = opaque(k2);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] *= keep_sc(kk, r, a.inv_keep);
      } else if (DROP) {
        float sc[16];
        drop_res_pairs(site_key(key, 2), row, h, a.thr, a.inv_keep, sc);
        k2 = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) { v[r] *= sc[r]; k2 |= (sc[r] != 0.f ? 1u : 0u) << r; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += t[r];
      layernorm(v, rs3, xh3);
    }
    float go[16], xo[16];
    // ---------------- backward -----------------
    // tokens past the sequence end (last tile only) get a zero incoming gradient:
    // every backward value of theirs is then zero, and each contraction / column-sum
    // term (a backward value times a finite forward one) adds exactly nothing, so
    // the tile stores need no per-element masks
    float d[16];
    load_row(a.dy, row, h, d);
#pragma unroll
    for (int r = 0; r < 16; ++r) d[r] = valid ? d[r] : 0.f;
    if (NEXT) {   // (the next block's in_proj gradient reads only inputs: dec_tail_wgrad)
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      // the three q | k | v gradient rows in flight together (one HBM round trip, not three)
      float4 gq[3][4];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          gq[cc][g4] = *reinterpret_cast<const float4*>(a.dqkv + row * 3 * E + cc * E + 8 * g4 + 4 * h);
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float g3[16];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 t = gq[cc][g4];
          g3[4 * g4] = t.x; g3[4 * g4 + 1] = t.y; g3[4 * g4 + 2] = t.z; g3[4 * g4 + 3] = t.w;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) g3[r] = valid ? g3[r] : 0.f;
        mvt(S.Wn + cc * E * LP, g3, acc, lane);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];
    }
    float t[16];
    // LN3
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh3[r];
    colsum_tile(tT, d, lane, cBE3);
    colsum_tile(tT, t, lane, cG3);
    layernorm_bwd(d, xh3, S.g3, rs3, h, d);                 // dv3 (residual into x2)
    // FFN
    {   // df2
      const uint32_t kk = opaque(k2);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = d[r] * keep_sc(kk, r, ik);
    }
    put_fl(tT, t, lane);
    get_op(tT, go, lane);
    get_op(tGL, xo, lane);
    contract(aW2, go, xo, cB2);
    asm volatile("" ::: "memory");
    {
      f16v acc = {};
      mvt(S.W2, t, acc, lane);
      // GELU'(x) = 0.5 (1 + erf(x / sqrt2)) + x phi(x) = gelu(x) / x + x phi(x): the
      // recompute's gelu(x), parked in tGL, instead of a second erf (~28 VALU ops each);
      // the ratio is well conditioned (0.5 (1 + erf) up to the two roundings), x = 0 -> 1/2
      const int tl = lane & 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float x = f1[r];
        const float gx = tGL[tl * LT + F(r, h)];
        const float ratio = x != 0.f ? gx / x : 0.5f;
        t[r] = acc[r] * fmaf(x * 0.39894228040143268f, __expf(-0.5f * x * x), ratio);   // df1
      }
    }
    put_fl(tT, t, lane);
    get_op(tT, go, lane);
    get_op(tX2, xo, lane);
    contract(aW1, go, xo, cB1);
    asm volatile("" ::: "memory");
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.W1, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx2
    }
    // LN2
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh2[r];
    colsum_tile(tT, d, lane, cBE2);
    colsum_tile(tT, t, lane, cG2);
    layernorm_bwd(d, xh2, S.g2, rs2, h, d);                 // dv2 (residual into x1)
    {   // da2
      const uint32_t kk = opaque(k1);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = d[r] * keep_sc(kk, r, ik);
    }
    put_fl(tT, t, lane);
    get_op(tT, go, lane);
    get_op(tC, xo, lane);
    contract(aWO2, go, xo, cBO2);
    asm volatile("" ::: "memory");
    float dc[16];
    {
      f16v acc = {};
      mvt(S.Wo2, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) dc[r] = acc[r];
    }
    put_fl(tC, dc, lane);        // C is consumed: the slot now holds dC
    // cross attention backward (dq -> t)
    {
      float dsv[16], pdv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) { dsv[k] = 0.f; pdv[k] = 0.f; }
#pragma unroll
      for (int hd = 0; hd < H; ++hd) {
        float dp[LC], ph[LC];
        cross_probs<LC>(S.kv, a.Lc, q, h, hd, ph);
        float Dsum = 0.f;
#pragma unroll
        for (int j = 0; j < LC; ++j) {
          float part = 0.f;
          if (j < a.Lc) {
            const float* vj = S.kv + j * 2 * E + E + 8 * hd + 4 * h;
#pragma unroll
            for (int i = 0; i < 4; ++i) part = fmaf(dc[4 * hd + i], vj[i], part);
          }
          part = xsum32(part);
          const bool kp = (km >> (hd * LCMAX + j)) & 1u;
          dp[j] = (j < a.Lc && kp) ? part * ik : 0.f;
          if ((j >> 2) == h) pdv[4 * (j & 3) + hd] = (j < a.Lc && kp) ? ph[j] * ik : 0.f;
          Dsum = fmaf(ph[j], dp[j], Dsum);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) t[4 * hd + i] = 0.f;
#pragma unroll
        for (int j = 0; j < LC; ++j) {
          const float ds = j < a.Lc ? ph[j] * (dp[j] - Dsum) * scale : 0.f;
          if ((j >> 2) == h) dsv[4 * (j & 3) + hd] = ds;
          if (j < a.Lc) {
            const float* kj = S.kv + j * 2 * E + 8 * hd + 4 * h;
#pragma unroll
            for (int i = 0; i < 4; ++i) t[4 * hd + i] = fmaf(ds, kj[i], t[4 * hd + i]);
          }
        }
      }
      float unused = 0.f;
      // dk part: acc[f][j'] += q[t][f] ds[t][j'];  dv part: dC[t][f] pd[t][j']
      put_half(tT, dsv, lane);
      get_op(tQ, go, lane);
      get_op(tT, xo, lane);
      contract(aK, go, xo, unused);
      asm volatile("" ::: "memory");
      put_half(tT, pdv, lane);
      get_op(tC, go, lane);
      get_op(tT, xo, lane);
      contract(aV, go, xo, unused);
      asm volatile("" ::: "memory");
    }
    put_fl(tT, t, lane);         // dq
    get_op(tT, go, lane);
    get_op(tX1, xo, lane);
    contract(aWQ, go, xo, cBQ);
    asm volatile("" ::: "memory");
    {
      f16v acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = d[r];
      mvt(S.Wq, t, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = acc[r];                        // dx1
    }
    // LN1
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = d[r] * xh1[r];
    colsum_tile(tT, d, lane, cBE1);
    colsum_tile(tT, t, lane, cG1);
    layernorm_bwd(d, xh1, S.g1, rs1, h, d);                 // dv1 = dx
    if (valid) store_row(a.dx, row, E, 0, h, d);
    {   // da1
      const uint32_t kk = opaque(k0);
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = d[r] * keep_sc(kk, r, ik);
    }
    put_fl(tT, t, lane);
    get_op(tT, go, lane);
    get_op(tO, xo, lane);
    contract(aWO1, go, xo, cBO1);
    asm volatile("" ::: "memory");
    {
      f16v acc = {};
      mvt(S.Wo1, t, acc, lane);
      float dO[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) dO[r] = acc[r];
      if (valid) store_row(a.dO, row, E, 0, h, dO);
    }
  }
  // ---------------- workgroup sums -----------------
  __syncthreads();
  constexpr int RS = 1024 + 64;                  // per-wave stride of the reduction rows
  float* red = &Lt[0][0];                         // [NW][RS] (reuses the tiles)
  float* out = a.wpart + (int64_t)seq * WPART;
  auto flush_job = [&](const f16v& acc, float cs, int moff, int boff) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave * RS + F(r, h) * 32 + (lane & 31)] = acc[r];
    red[wave * RS + 1024 + lane] = cs;             // lanes 32..63: the other half's rows
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += NT)
      out[moff + i] = ((red[i] + red[RS + i]) + red[2 * RS + i]) + red[3 * RS + i];
    if (threadIdx.x < 32) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w)
        sum += red[w * RS + 1024 + threadIdx.x] + red[w * RS + 1024 + 32 + threadIdx.x];
      out[boff + threadIdx.x] = sum;
    }
    __syncthreads();
  };
  flush_job(aWO1, cBO1, OFF_WO1, OFF_BO1);
  flush_job(aWQ, cBQ, OFF_WQ, OFF_BQ);
  flush_job(aWO2, cBO2, OFF_WO2, OFF_BO2);
  flush_job(aW1, cB1, OFF_W1, OFF_B1);
  flush_job(aW2, cB2, OFF_W2, OFF_B2);
  {   // LayerNorm vectors: [g1 b1 | g2 b2 | g3 b3]
    const float cl[6] = {cG1, cBE1, cG2, cBE2, cG3, cBE3};
#pragma unroll
    for (int i = 0; i < 6; ++i) red[wave * RS + i * 64 + lane] = cl[i];
    __syncthreads();
    if (threadIdx.x < 6 * 32) {
      const int i = threadIdx.x / 32, c = threadIdx.x % 32;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w * RS + i * 64 + c] + red[w * RS + i * 64 + 32 + c];
      out[OFF_G1 + i * 32 + c] = sum;
    }
    __syncthreads();
  }
  // context k | v gradients of this sequence: acc[f = F(r,h)][j' = lane&31] is valid
  // where (j' & 3) == f >> 3, j = j' >> 2 < Lc.  Summed into S.kv (no longer read),
  // then this sequence's share of the k | v projection backward: d context and the
  // partials of the in_proj rows [E, 3E) (weights and biases).
  for (int kv = 0; kv < 2; ++kv) {
    const f16v& acc = kv ? aV : aK;
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave * RS + F(r, h) * 32 + (lane & 31)] = acc[r];
    __syncthreads();
    for (int i = threadIdx.x; i < a.Lc * E; i += NT) {
      const int j = i / E, f = i % E;
      const int idx = f * 32 + 4 * j + (f >> 3);
      S.kv[j * 2 * E + (kv ? E : 0) + f] =
          ((red[idx] + red[RS + idx]) + red[2 * RS + idx]) + red[3 * RS + idx];
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < a.Lc * E; i += NT) {          // d context
    const int j = i / E, k = i % E;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < 2 * E; ++c) acc = fmaf(S.kv[j * 2 * E + c], a.Wq[(int64_t)(E + c) * E + k], acc);
    a.dctx[((int64_t)seq * a.Lc + j) * E + k] = acc;
  }
  for (int i = threadIdx.x; i < 2 * E * E; i += NT) {         // dW rows [E, 3E)
    const int c = i / E, k = i % E;
    float acc = 0.f;
    for (int j = 0; j < a.Lc; ++j) acc = fmaf(S.kv[j * 2 * E + c], S.ctxs[j * E + k], acc);
    out[OFF_WQ + E * E + i] = acc;
  }
  if (threadIdx.x < 2 * E) {                                   // db rows [E, 3E)
    float acc = 0.f;
    for (int j = 0; j < a.Lc; ++j) acc += S.kv[j * 2 * E + threadIdx.x];
    out[OFF_BQ + E + threadIdx.x] = acc;
  }
}

// column ranges of the gradient layout a mode produces (the k | v rows of the
// cross in_proj are excluded: the caller's projection gradient owns them)
int tail_ranges(int mode, int (&r)[3][2]) {
  if (mode == MODE_PRE) {
    r[0][0] = OFF_WO1; r[0][1] = OFF_WQ + 1024;
    r[1][0] = OFF_BO1; r[1][1] = OFF_BQ + 32;
    r[2][0] = OFF_G1;  r[2][1] = OFF_G1 + 64;
  } else if (mode == MODE_POST) {
    r[0][0] = OFF_WO2; r[0][1] = OFF_BO1;
    r[1][0] = OFF_BO2; r[1][1] = OFF_G1;
    r[2][0] = OFF_G2;  r[2][1] = WPART;
  } else {
    r[0][0] = 0;       r[0][1] = OFF_WQ + 1024;
    r[1][0] = OFF_WO2; r[1][1] = OFF_BQ + 32;
    r[2][0] = OFF_BO2; r[2][1] = WPART;
  }
  return 3;
}

int sum_tail(int mode, const float* wpart, int G, float* gflat, vaesne_colsum_list* defer,
             hipStream_t s) {
  int r[3][2];
  const int n = tail_ranges(mode, r);
  for (int k = 0; k < n; ++k) {
    const int rc = colsum_or_defer(defer, wpart + r[k][0], WPART, G, r[k][1] - r[k][0],
                                   gflat + r[k][0], 0, s);
    if (rc) return rc;
  }
  return 0;
}

template <int LC, bool NEXT, bool DROP>
int launch_fwd(const Tail& a, int grid, float*, hipStream_t s) {
  hipLaunchKernelGGL((dec_tail_fwd<LC, NEXT, DROP>), dim3(grid), dim3(NT), 0, s, a);
  VAESNE_CHECK_LAUNCH();
  return 0;
}
// the weight-gradient jobs' token chunk of the two-kernel backward: up to 4 data chunks (the
// data kernel's chunk fills the CUs with one job; the eleven jobs need fewer, longer
// workgroups: fewer partial rows and loads in flight per wave)
int wgrad_chunk(int L, int chunk) { return std::min((L + 127) / 128 * 128, 4 * chunk); }
int wgrad_grid(int M, int L, int chunk) {
  const int wc = wgrad_chunk(L, chunk);
  return (M / L) * ((L + wc - 1) / wc);
}
template <int LC, bool NEXT, bool DROP>
int launch_bwd(const Tail& a, int grid, float* scr, hipStream_t s) {
  if (DROP && !a.masks)
    hipLaunchKernelGGL((dec_tail_bwd_data<LC, NEXT, DROP, false>), dim3(grid), dim3(NT), 0, s, a,
                       scr);
  else
    hipLaunchKernelGGL((dec_tail_bwd_data<LC, NEXT, DROP, true>), dim3(grid), dim3(NT), 0, s, a,
                       scr);
  VAESNE_CHECK_LAUNCH();
  Tail b = a;
  b.chunk = wgrad_chunk(a.L, a.chunk);
  const int gw = wgrad_grid(a.M, a.L, a.chunk);
  hipLaunchKernelGGL(dec_tail_wgrad, dim3(gw, NJOB), dim3(NT), 0, s, b, (const float*)scr, 0);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

template <int LC, bool NEXT, bool DROP>
int launch_fused(const Tail& a, int grid, hipStream_t s) {
  if (DROP && !a.masks)
    hipLaunchKernelGGL((dec_tail_bwd_fused<LC, NEXT, DROP, false>), dim3(grid), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((dec_tail_bwd_fused<LC, NEXT, DROP, true>), dim3(grid), dim3(NT), 0, s, a);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int dispatch_fused(const Tail& a, int grid, hipStream_t s) {
  const bool next = a.Wn != nullptr, drop = a.p_drop > 0.f;
#define VAESNE_FUSED_CASE(LCV)                                                  \
  if (next && drop) return launch_fused<LCV, true, true>(a, grid, s);           \
  if (next) return launch_fused<LCV, true, false>(a, grid, s);                  \
  if (drop) return launch_fused<LCV, false, true>(a, grid, s);                  \
  return launch_fused<LCV, false, false>(a, grid, s);
  // LC: the compile-time context-token bound (4: photometry decoder, latent_len tokens;
  // 5: spectra decoder, latent_len + the phase token; 8: anything else up to LCMAX)
  if (a.Lc <= 4) { VAESNE_FUSED_CASE(4) }
  if (a.Lc == 5) { VAESNE_FUSED_CASE(5) }
  VAESNE_FUSED_CASE(8)
#undef VAESNE_FUSED_CASE
}

// long sequences take the fused backward (vaesne_dec_tail_force_path(2): the two-kernel
// path; force_path(1): fused always)
int g_tail_path = 0;
bool use_fused(int L, int nseq) {
  if (g_tail_path == 1) return true;
  if (g_tail_path == 2) return false;
  // one workgroup per sequence: only when the sequences alone fill half the chip (the
  // fused kernel runs a whole 982-token sequence serially: 0.22 ms at any batch); small
  // batches take the two-kernel path over chunks (tail_chunk)
  return L >= 256 && nseq >= 128;
}

// tokens per workgroup of the two-kernel path and the forward: short sequences whole
// (rounded to 128); long ones in 512-token chunks, halved down to 128 while the grid
// would stay under one workgroup per CU (small batches: B = 2 -> 32 sequences x 8 chunks)
int tail_chunk(int M, int L) {
  if (L <= 256) return ((L + 127) / 128) * 128;
  const int64_t nseq = M / L;
  for (int c = 512; c > 128; c >>= 1)
    if (nseq * ((L + c - 1) / c) >= 256) return c;
  return 128;
}

template <bool FWD>
int dispatch(const Tail& a, int grid, float* scr, hipStream_t s) {
  const bool next = a.Wn != nullptr, drop = a.p_drop > 0.f;
#define VAESNE_TAIL_CASE(LCV)                                                                   \
  if (next && drop) return FWD ? launch_fwd<LCV, true, true>(a, grid, scr, s) : launch_bwd<LCV, true, true>(a, grid, scr, s); \
  if (next) return FWD ? launch_fwd<LCV, true, false>(a, grid, scr, s) : launch_bwd<LCV, true, false>(a, grid, scr, s);       \
  if (drop) return FWD ? launch_fwd<LCV, false, true>(a, grid, scr, s) : launch_bwd<LCV, false, true>(a, grid, scr, s);       \
  return FWD ? launch_fwd<LCV, false, false>(a, grid, scr, s) : launch_bwd<LCV, false, false>(a, grid, scr, s);
  if (a.Lc <= 4) { VAESNE_TAIL_CASE(4) }
  if (a.Lc == 5) { VAESNE_TAIL_CASE(5) }
  VAESNE_TAIL_CASE(8)
#undef VAESNE_TAIL_CASE
}

Tail make(const float* x, const float* O, const float* ctx, int M, int L, int Lc,
          const float* const* w, float p_drop, const int64_t* rng, uint32_t call_id) {
  Tail a{};
  a.x = x; a.O = O; a.ctx = ctx; a.M = M; a.L = L; a.Lc = Lc;
  a.Wo1 = w[0]; a.bo1 = w[1]; a.g1 = w[2]; a.be1 = w[3]; a.Wq = w[4]; a.bq = w[5];
  a.Wo2 = w[6]; a.bo2 = w[7]; a.g2 = w[8]; a.be2 = w[9]; a.W1 = w[10]; a.b1 = w[11];
  a.W2 = w[12]; a.b2 = w[13]; a.g3 = w[14]; a.be3 = w[15]; a.Wn = w[16]; a.bn = w[17];
  a.p_drop = p_drop; a.thr = drop_thr16(p_drop);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.rng = rng; a.call_id = call_id;
  a.chunk = tail_chunk(M, L);
  return a;
}

bool shapes_ok(int M, int L, int Lc) {
  return M > 0 && L > 0 && M % L == 0 && Lc >= 1 && Lc <= LCMAX;
}

}  // namespace

// two-kernel path: [G][WPART] slabs | scratch vectors | d k|v [Nseq, Lc, 64] | the
// k | v projection's weight-gradient workspace
int64_t ctx_grad_floats(int M, int L, int Lc) {
  const int64_t rows = (int64_t)(M / L) * Lc;
  return rows * 2 * E + (vaesne_linear_bwd_weight_workspace(rows, 2 * E, E) + 3) / 4;
}

VAESNE_API int64_t vaesne_dec_tail_workspace(int M, int L, int Lc) {
  if (!shapes_ok(M, L, Lc)) return 0;
  const int chunk = tail_chunk(M, L);
  const int chunks = (L + chunk - 1) / chunk;
  const int64_t G = (int64_t)(M / L) * chunks;
  return (G * WPART + (int64_t)NVEC * M * E + ctx_grad_floats(M, L, Lc)) * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_dec_tail_fwd(const float* x, const float* O, const float* ctx, int M, int L,
                                   int Lc, const float* const* w, float p_drop,
                                   const int64_t* rng, uint32_t call_id, float* y, float* qkv,
                                   uint32_t* drop_masks, void* stream) {
  if (!shapes_ok(M, L, Lc)) return (int)hipErrorInvalidValue;
  Tail a = make(x, O, ctx, M, L, Lc, w, p_drop, rng, call_id);
  a.masks = p_drop > 0.f ? drop_masks : nullptr;
  a.y = y; a.qkv = qkv;
  if (a.Wn && !qkv) return (int)hipErrorInvalidValue;
  const int grid = (M / L) * ((L + a.chunk - 1) / a.chunk);
  return dispatch<true>(a, grid, nullptr, (hipStream_t)stream);
}

// gflat [WPART]: every parameter gradient of the block in the layout of the
// per-workgroup slabs (see include/vaesne_hip.h), the whole cross in_proj included;
// dctx [Nseq, Lc, 32] the context tokens' gradient.
VAESNE_API int vaesne_dec_tail_bwd(const float* x, const float* O, const float* ctx, int M, int L,
                                   int Lc, const float* const* w, float p_drop,
                                   const int64_t* rng, uint32_t call_id, const float* y,
                                   const float* dy, const float* dqkv, const uint32_t* drop_masks,
                                   float* dx, float* dO, float* dctx, float* gflat,
                                   float* workspace, vaesne_colsum_list* defer, void* stream) {
  if (!shapes_ok(M, L, Lc)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  Tail a = make(x, O, ctx, M, L, Lc, w, p_drop, rng, call_id);
  a.masks = p_drop > 0.f ? const_cast<uint32_t*>(drop_masks) : nullptr;
  a.dy = dy; a.dqkv = dqkv; a.dx = dx; a.dO = dO;
  if (a.Wn && !dqkv) return (int)hipErrorInvalidValue;
  a.y = const_cast<float*>(y);
  a.dctx = dctx;
  if (use_fused(L, M / L)) {   // one workgroup per sequence, no scratch
    const int nseq = M / L;
    a.wpart = workspace;
    int rc = dispatch_fused(a, nseq, s);
    if (rc) return rc;
    // the next block's in_proj gradient: dec_tail_wgrad's WN jobs (inputs only) into
    // a second partial area, one row per (sequence, chunk)
    const int chunks = (L + a.chunk - 1) / a.chunk;
    float* wn = workspace + (int64_t)nseq * WPART;
    if (a.Wn) {
      Tail b = a;
      b.wpart = wn;
      hipLaunchKernelGGL(dec_tail_wgrad_wn, dim3(nseq * chunks), dim3(NT), 0, s, b);
      VAESNE_CHECK_LAUNCH();
    }
    // fused rows: everything but the in_proj-of-next regions
    const int fr[3][2] = {{0, OFF_WN}, {OFF_BO1, OFF_BN}, {OFF_G1, WPART}};
    for (int k = 0; k < 3; ++k) {
      rc = colsum_or_defer(defer, workspace + fr[k][0], WPART, nseq, fr[k][1] - fr[k][0],
                           gflat + fr[k][0], 0, s);
      if (rc) return rc;
    }
    if (!a.Wn) return 0;
    rc = colsum_or_defer(defer, wn + OFF_WN, WPART, nseq * chunks, 3 * 1024, gflat + OFF_WN, 0, s);
    return rc ? rc : colsum_or_defer(defer, wn + OFF_BN, WPART, nseq * chunks, 96, gflat + OFF_BN,
                                     0, s);
  }
  const int chunks = (L + a.chunk - 1) / a.chunk;
  const int grid = (M / L) * chunks;
  // one workgroup: its slab IS the gradient (no column sum)
  a.wpart = grid == 1 ? gflat : workspace;
  float* scr = workspace + (int64_t)grid * WPART;
  float* dkv = scr + (int64_t)NVEC * M * E;           // per-sequence d k|v (wgrad J_K / J_V jobs)
  a.dkvc = dkv;
  int rc = dispatch<false>(a, grid, scr, s);
  if (rc) return rc;
  if (grid > 1) {
    rc = sum_tail(MODE_FULL, workspace, wgrad_grid(M, L, a.chunk), gflat, defer, s);
    if (rc) return rc;
  }
  // the context k | v projection backward over the Nseq * Lc context tokens
  const int64_t rows = (int64_t)(M / L) * Lc;
  float* lws = dkv + rows * 2 * E;
  rc = vaesne_linear_bwd_weight(dkv, 2 * E, nullptr, 0, 0, ctx, E, nullptr, 0, rows, 2 * E, E,
                                gflat + OFF_WQ + E * E, gflat + OFF_BQ + E, 0, lws, defer, s);
  if (rc) return rc;
  return vaesne_linear_bwd_data(dkv, 2 * E, nullptr, 0, 0, rows, 2 * E, a.Wq + E * E, E, dctx, E,
                                0, s);
}

VAESNE_API int64_t vaesne_enc_block_workspace(int M) {
  return M > 0 ? vaesne_dec_tail_workspace(M, M, 1) : 0;
}

VAESNE_API int vaesne_enc_block_fwd(int mode, const float* x, const float* O, int M,
                                    const float* const* w, float p_drop, const int64_t* rng,
                                    uint32_t call_id, float* y, float* q_or_qkv,
                                    uint32_t* drop_masks, void* stream) {
  if (M <= 0 || (mode != MODE_PRE && mode != MODE_POST)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && (!drop_masks || !rng)) return (int)hipErrorInvalidValue;
  Tail a = make(x, O, nullptr, M, M, 1, w, p_drop, rng, call_id);
  a.mode = mode;
  a.masks = p_drop > 0.f ? drop_masks : nullptr;
  a.y = y; a.qkv = q_or_qkv;
  if (!q_or_qkv && (mode == MODE_PRE || a.Wn)) return (int)hipErrorInvalidValue;
  const int grid = (M + a.chunk - 1) / a.chunk;
  hipStream_t s = (hipStream_t)stream;
  const bool drop = p_drop > 0.f, next = a.Wn != nullptr;
  if (mode == MODE_PRE) {
    if (drop) hipLaunchKernelGGL((enc_pre_fwd<true>), dim3(grid), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((enc_pre_fwd<false>), dim3(grid), dim3(NT), 0, s, a);
  } else if (next) {
    if (drop) hipLaunchKernelGGL((enc_post_fwd<true, true>), dim3(grid), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((enc_post_fwd<true, false>), dim3(grid), dim3(NT), 0, s, a);
  } else {
    if (drop) hipLaunchKernelGGL((enc_post_fwd<false, true>), dim3(grid), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((enc_post_fwd<false, false>), dim3(grid), dim3(NT), 0, s, a);
  }
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_enc_block_bwd(int mode, const float* x, const float* O, int M,
                                    const float* const* w, float p_drop, const int64_t* rng,
                                    uint32_t call_id, const float* y, const float* dy,
                                    const float* dq_or_dqkv, const uint32_t* drop_masks,
                                    float* dx, float* dO, float* gflat, float* workspace,
                                    vaesne_colsum_list* defer, void* stream) {
  if (M <= 0 || (mode != MODE_PRE && mode != MODE_POST)) return (int)hipErrorInvalidValue;
  if (p_drop > 0.f && !drop_masks) return (int)hipErrorInvalidValue;
  Tail a = make(x, O, nullptr, M, M, 1, w, p_drop, rng, call_id);
  a.mode = mode;
  a.masks = p_drop > 0.f ? const_cast<uint32_t*>(drop_masks) : nullptr;
  a.dy = dy; a.dqkv = dq_or_dqkv; a.dx = dx; a.dO = dO;
  a.y = const_cast<float*>(y);
  if (!dq_or_dqkv && (mode == MODE_PRE || a.Wn)) return (int)hipErrorInvalidValue;
  const int grid = (M + a.chunk - 1) / a.chunk;
  a.wpart = grid == 1 ? gflat : workspace;
  float* scr = workspace + (int64_t)grid * WPART;   // vaesne_dec_tail_workspace(M, M, 1) layout
  hipStream_t s = (hipStream_t)stream;
  const bool drop = p_drop > 0.f, next = a.Wn != nullptr;
  if (mode == MODE_PRE) {
    if (drop) hipLaunchKernelGGL((enc_pre_bwd_data<true>), dim3(grid), dim3(NT), 0, s, a, scr);
    else hipLaunchKernelGGL((enc_pre_bwd_data<false>), dim3(grid), dim3(NT), 0, s, a, scr);
  } else if (next) {
    if (drop) hipLaunchKernelGGL((enc_post_bwd_data<true, true>), dim3(grid), dim3(NT), 0, s, a, scr);
    else hipLaunchKernelGGL((enc_post_bwd_data<true, false>), dim3(grid), dim3(NT), 0, s, a, scr);
  } else {
    if (drop) hipLaunchKernelGGL((enc_post_bwd_data<false, true>), dim3(grid), dim3(NT), 0, s, a, scr);
    else hipLaunchKernelGGL((enc_post_bwd_data<false, false>), dim3(grid), dim3(NT), 0, s, a, scr);
  }
  VAESNE_CHECK_LAUNCH();
  hipLaunchKernelGGL(dec_tail_wgrad, dim3(grid, NJOB), dim3(NT), 0, s, a, (const float*)scr, 0);
  VAESNE_CHECK_LAUNCH();
  if (grid == 1) return 0;
  return sum_tail(mode, workspace, grid, gflat, defer, s);
}

VAESNE_API int vaesne_dec_tail_force_path(int path) {
  if (path < 0 || path > 2) return (int)hipErrorInvalidValue;
  g_tail_path = path;
  return 0;
}

VAESNE_API int vaesne_dec_tail_grad_layout(int* offsets) {
  const int off[18] = {OFF_WO1, OFF_BO1, OFF_G1, OFF_BE1, OFF_WQ, OFF_BQ, OFF_WO2, OFF_BO2,
                       OFF_G2, OFF_BE2, OFF_W1, OFF_B1, OFF_W2, OFF_B2, OFF_G3, OFF_BE3,
                       OFF_WN, OFF_BN};
  for (int i = 0; i < 18; ++i) offsets[i] = off[i];
  return WPART;
}
