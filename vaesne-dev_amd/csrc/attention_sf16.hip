// Masked multi-head attention of head_dim 8 on the f16 matrix cores, at fp32 accuracy.
//
// The arithmetic is attention.hip's (util_layers.py:289 -> torch/nn/functional.py:6559-6594:
// S = q k^T / sqrt(dh) + key bias, P = softmax(S), A = Dropout_p(P), O = A v, and the
// backward of each), flash-style in the log2 domain.  What changes is where the products
// run: every one of them (S, P V in the forward; S, dP, dV, dK, dQ in the backward) is a
// v_mfma_f32_16x16x32_f16 on SPLIT operands.  An fp32 value x is carried as two f16,
// hi = f16(x) and lo = f16(x - hi) (the difference is exact in fp32, rounded once), so
// x = hi + lo to 2^-22 relative; a product x y is taken as hi_x hi_y + hi_x lo_y + lo_x hi_y
// (the dropped lo_x lo_y is 2^-22 of it) with fp32 accumulation.  f16 MFMA issue is 16x the
// fp32 rate (MI355X_MICROARCH.md, Matrix cores), so the three terms cost far less than the
// packed-fp32 VALU FMAs they replace, and the VALU keeps only what is not a product: the
// exponentials, the dropout hash and keep decisions, dS and the hi / lo conversions.
//
// Operand terms.  With head_dim 8, one 32-deep MFMA holds a whole dot product in its four
// 8-element slots: lane group g (lanes 16g .. 16g + 15) carries term g.  Scores:
//   A = Q:  [q_hi | q_hi | q_lo | 1, 1, 0..]    B = K: [k_hi | k_lo | k_hi | bias_hi, bias_lo, 0..]
// (the fourth slot adds the key bias: 0 / -inf key padding), value products likewise.  The
// contraction sums over slots, and A's slot (g, j) meets B's slot (g, j) whichever k the
// hardware gives it, so the term layout needs only that A and B share one slot map.
// Contractions over the 16 rows of an accumulator tile (P V, dV = P^T dO, dK = dS^T Q,
// dQ = dS K) carry the values as hi pair words and lo pair words (f16x2 of two values of the
// same precision); the other operand supplies the matching y_hi in the slots of both for its
// hi rows and y_lo / 0 for its lo rows (rows f and f + 8 of the result summed at the end: the
// same three terms).  A dword of either operand never mixes a hi and a lo part: the matrix
// core adds a dword's two products first, and a (hi, lo) dword of one value measurably loses
// the lo product ("Split-f16 operand pairing").
//
// Range.  Softmax probabilities enter scaled, P' = 2^c P (c = 7 forward with the lazy
// running max, 14 backward), so they sit in f16's normal range; the gradient operands of the
// backward are scaled by per-(sequence, head) powers of two chosen from their maxima (a
// prologue over dO and O), so dS stays below 2^15.  q, k and v enter unscaled: an element
// beyond f16's range (65504) becomes inf and the output NaN (loud), and elements below 2^-3
// keep an absolute error of 2^-25 instead of a relative one -- for the softmax only the
// absolute score error matters, and it is then 2^-25 per feature product, fp32's own scale.
//
// Dropout.  The forward hashes each (query, key pair) exactly as attn_fwd_kernel does
// (attn_pair_bits_mixed: the same keep decisions for the same (seed, counter, call id,
// row, key)) and writes the keep bits in this path's own layout, which the backward reads:
// word ((bh * NT8 + key / 128) * 4 + (key % 16) / 4) * Lqp + query, bit
// 4 ((key % 128) / 16) + key % 4  (NT8 = ceil(Lk / 128), Lqp = Lq rounded up to 16).
#include <algorithm>

#include "attn_common.h"

namespace vaesne {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mma(u4 a, u4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b),
                                                c, 0, 0, 0);
}
// f16x2 (round to nearest even) of (a, b): the hi halves
__device__ __forceinline__ uint32_t pk_hi(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, h2v));
}
// f16x2 of (a - hi.x, b - hi.y): the differences are exact in fp32, rounded once.  Plain
// code, no inline asm: the compiler's hazard recognizer pads every producer / consumer of
// these registers (exp results read here, MFMA operands written here), which an asm
// statement hides from it
__device__ __forceinline__ uint32_t pk_lo(float a, float b, uint32_t hi) {
  const f2v h = __builtin_convertvector(__builtin_bit_cast(h2v, hi), f2v);
  return pk_hi(a - h.x, b - h.y);
}
// pk_lo through v_fma_mix_f32 (a * one - f16 hi half, one rounding: the same bits as a - hi,
// which is exact): one instruction per value instead of a conversion and a subtract.  `one`
// is 1.0 from opaque_one(), which the compiler cannot fold (a * 1 would become the plain
// subtract again)
__device__ __forceinline__ uint32_t pk_lo1(float a, float b, uint32_t hi, float one) {
  const h2v h = __builtin_bit_cast(h2v, hi);
  return pk_hi(fmaf(a, one, -(float)h.x), fmaf(b, one, -(float)h.y));
}
__device__ __forceinline__ float opaque_one() {
  float x;
  asm volatile("v_mov_b32 %0, 1.0" : "=v"(x));
  return x;
}
__device__ __forceinline__ _Float16 f16_hi(float x) { return (_Float16)x; }
__device__ __forceinline__ _Float16 f16_lo(float x) {
  return isfinite(x) ? (_Float16)(x - (float)(_Float16)x) : (_Float16)0.f;
}
__device__ __forceinline__ uint32_t pack2(_Float16 a, _Float16 b) {
  return __builtin_bit_cast(uint32_t, (h2v){a, b});
}
__device__ __forceinline__ float max4(f4 v) { return fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])); }
__device__ __forceinline__ int imax8(f4 a, f4 b) {
  const int m0 = max(max(__float_as_int(a[0]), __float_as_int(a[1])), __float_as_int(a[2]));
  const int m1 = max(max(__float_as_int(a[3]), __float_as_int(b[0])), __float_as_int(b[1]));
  return max(max(m0, m1), max(__float_as_int(b[2]), __float_as_int(b[3])));
}
__device__ __forceinline__ f4 splat(float x) { return (f4){x, x, x, x}; }
__device__ __forceinline__ u4 ldu4(const uint32_t* p) { return *reinterpret_cast<const u4*>(p); }
__device__ __forceinline__ uint32_t as_u(float x) { return __float_as_uint(x); }

constexpr uint32_t ONES_F16X2 = 0x3C003C00u;   // (1.0h, 1.0h): the bias slot's multipliers

// =================================== forward ===================================
// Workgroup: NW waves (NW = 1, 2, 4), wave w owns NQT query tiles of 16 (queries
// qb*16NQT*NW + 16(NQT w + n) + c, n < NQT, c = lane & 15) and RC copies of them, all keys of
// one (distinct sequence, head) in chunks of 32 NW (one (key, half-row) staging item per
// thread).  Scores as S^T tiles: A = the staged K image (16 keys), B = the wave's resident Q
// operand, C = (7 - m) per query column, so the MFMA leaves S - m + 7 and p' = exp2 of it
// directly.  Lane (g, c) holds keys 4g..4g+3 of each 16-key tile for query c: its (m, l)
// partial state covers its own keys, the origin m is shared by the column's four lane groups
// (moved only together, in the rare rescale, decided per query tile so a tile's arithmetic
// never depends on the other tiles of its wave).
// P' V: per 32 keys (two tiles), B = the lane's eight p' as hi / lo pair words (f16x2 of two
// keys each, RNE hi and lo = f16(p' - hi)), A = the staged V^T image (16 rows: v_hi features
// 0..7, v_lo features 0..7), accumulating O^T (two MFMAs: hi pairs, lo pairs).  The pairs keep
// like magnitudes in each dword of the operands: the matrix core sums a dword's two products
// before accumulating, and a pair mixing a hi and a lo product (a (hi, lo) word of ONE value)
// loses that value's lo part to ~2^-15 of the pair (measured: tools/dbg).
// Copies (the decoders' first block, SpectraLayers.py:54-62 / PhotometricLayers.py:59-67: the
// R = K x 2 copies of each distinct sequence see the same q, k, v): the scores, exponentials,
// running sums and splits are computed once per distinct query tile, the keep decisions and
// P' V per copy (copy r of distinct sequence b is sequence r Bd + b of the output, its keep
// decisions those of the plain kernel on that sequence, its bitmap words that sequence's).
// One copy (RC = 1, R = 1) is the plain attention.
constexpr int FNW_MAX = 4;
constexpr int FKC_MAX = 32 * FNW_MAX;

constexpr int fwd_occ(int NQT, int RC) { return NQT * RC >= 16 ? 2 : 3; }

template <int NQT, int RC, bool DROP>
__global__ __launch_bounds__(256, fwd_occ(NQT, RC)) void attn_fwd_sf16_kernel(AttnArgs a, int NT8, int Lqp,
                                                                            int R, int qb0, int nqbs) {
  // per staged key: [hi 4 u32 | lo 4 | bias (hi, lo), 0 ...]; V^T per 32-key pair: 16 rows
  // x 32 f16 at a 24-word row stride (conflict-free staging stores and operand reads);
  // key-pair mixes for the dropout hash
  __shared__ __attribute__((aligned(16))) uint32_t Ki[2][FKC_MAX * 12];
  __shared__ __attribute__((aligned(16))) uint32_t Vi[2][FKC_MAX * 12];
  __shared__ __attribute__((aligned(16))) uint32_t Kp[2][FKC_MAX / 2];
  __shared__ uint32_t Red[3][FNW_MAX];
  const int NW = blockDim.x >> 6, KC = 32 * NW, QB = 16 * NQT * NW;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, c = l & 15;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qb = qb0 + wg % nqbs, bh = wg / nqbs;
  const int b = bh / a.H, h = bh - b * a.H;
  const int Bd = a.B;
  const int r0 = blockIdx.y * RC;                  // first copy of this workgroup
  const float* kg = a.k + (int64_t)b * a.k_bs + h * 8;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * 8;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  const uint32_t skey = DROP ? key_of(a.rng_state, a.call_id) : 0u;
  const float one = opaque_one();
  // the output sequence of copy rc: copies past R (R % RC != 0) run as copy R - 1, not stored
  auto seq_of = [&](int rc) { return (int64_t)min(r0 + rc, R - 1) * Bd + b; };

  // operand ranges: powers of two for the f16 splits.  v' = v 2^ev with max |v'| over the
  // (sequence, head) in [2^14, 2^15) (o unscaled once at the end: relative precision for any
  // |v|); q' = q 2^-ek, k' = k 2^ek balanced around sqrt(max|q| max|k|), max |q| over the
  // aligned group of 256 queries holding this workgroup's (whatever the kernel's query block:
  // the plain and the copies' kernels agree bit for bit), max |k| over the keys (the product,
  // hence S, unchanged; f16 range for |q|, |k| up to ~2^15 either side of the balance).
  // Maxima on bit patterns (an unsigned max of |x| is the float max)
  // staging items: K of key kk_i of the chunk, features 4 hf .. 4 hf + 3; V of keys
  // 32 w + 2 vp + {0, 1}, features 2 vf, 2 vf + 1 (one pair word per V^T row written).  The
  // raw rows are loaded here (the first chunk's in flight with the range pass's loads) and
  // scaled by 2^ek / 2^ev when committed
  const int kk_i = t >> 1, hf = t & 1, vp = l & 15, vf = l >> 4;
  float4 rK = make_float4(0.f, 0.f, 0.f, 0.f);
  float2 rV0 = make_float2(0.f, 0.f), rV1 = rV0;
  float rB = 0.f;
  auto issue = [&](int ks) {
    const int key = ks + kk_i;
    const bool ok = key < a.Lk;
    const int64_t kc = min(key, a.Lk - 1);
    rK = ok ? *reinterpret_cast<const float4*>(kg + kc * a.k_ls + 4 * hf) : make_float4(0.f, 0.f, 0.f, 0.f);
    rB = ok ? (kbg ? kbg[key] : 0.f) : -INFINITY;
    const int v0 = ks + 32 * w + 2 * vp;
    const int64_t vc0 = min(v0, a.Lk - 1), vc1 = min(v0 + 1, a.Lk - 1);
    rV0 = v0 < a.Lk ? *reinterpret_cast<const float2*>(vg + vc0 * a.v_ls + 2 * vf) : make_float2(0.f, 0.f);
    rV1 = v0 + 1 < a.Lk ? *reinterpret_cast<const float2*>(vg + vc1 * a.v_ls + 2 * vf) : make_float2(0.f, 0.f);
  };
  float fk = 1.f, fv = 1.f;
  float xq[NQT][8];
  uint32_t mq_ = 0u, mk_ = 0u, mv_ = 0u;
  const uint32_t am = 0x7fffffffu;
#pragma unroll
  for (int n = 0; n < NQT; ++n) {
    const int qc = min(qb * QB + 16 * (NQT * w + n) + c, a.Lq - 1);
    const float* qp = a.q + (int64_t)b * a.q_bs + (int64_t)qc * a.q_ls + h * 8;
    const float4 x0 = *reinterpret_cast<const float4*>(qp);
    const float4 x1 = *reinterpret_cast<const float4*>(qp + 4);
    const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int f = 0; f < 8; ++f) xq[n][f] = x[f];
  }
  issue(0);
  for (int i = (qb * QB & ~255) + t; i < min((qb * QB & ~255) + 256, a.Lq); i += blockDim.x) {
    const float* qp = a.q + (int64_t)b * a.q_bs + (int64_t)i * a.q_ls + h * 8;
    const float4 x0 = *reinterpret_cast<const float4*>(qp), x1 = *reinterpret_cast<const float4*>(qp + 4);
    mq_ = max(mq_, max(max(max(as_u(x0.x) & am, as_u(x0.y) & am), max(as_u(x0.z) & am, as_u(x0.w) & am)),
                       max(max(as_u(x1.x) & am, as_u(x1.y) & am), max(as_u(x1.z) & am, as_u(x1.w) & am))));
  }
  for (int i0 = 0; i0 < a.Lk; i0 += 4 * (int)blockDim.x) {   // four rows a thread: one round trip
    float4 kx[4][2], vx[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = min(i0 + j * (int)blockDim.x + t, a.Lk - 1);   // (repeats: max unchanged)
      kx[j][0] = *reinterpret_cast<const float4*>(kg + i * a.k_ls);
      kx[j][1] = *reinterpret_cast<const float4*>(kg + i * a.k_ls + 4);
      vx[j][0] = *reinterpret_cast<const float4*>(vg + i * a.v_ls);
      vx[j][1] = *reinterpret_cast<const float4*>(vg + i * a.v_ls + 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        mk_ = max(mk_, max(max(as_u(kx[j][u].x) & am, as_u(kx[j][u].y) & am),
                           max(as_u(kx[j][u].z) & am, as_u(kx[j][u].w) & am)));
        mv_ = max(mv_, max(max(as_u(vx[j][u].x) & am, as_u(vx[j][u].y) & am),
                           max(as_u(vx[j][u].z) & am, as_u(vx[j][u].w) & am)));
      }
  }
  {
    const float mq0 = wave_max(__uint_as_float(mq_)), mk0 = wave_max(__uint_as_float(mk_)),
                mv0 = wave_max(__uint_as_float(mv_));
    if (l == 0) {
      Red[0][w] = as_u(mq0);
      Red[1][w] = as_u(mk0);
      Red[2][w] = as_u(mv0);
    }
  }
  __syncthreads();
  int ev = 0, ek = 0;
  {
    float mq = 0.f, mk = 0.f, mv = 0.f;
    for (int i = 0; i < NW; ++i) {
      mq = fmaxf(mq, __uint_as_float(Red[0][i]));
      mk = fmaxf(mk, __uint_as_float(Red[1][i]));
      mv = fmaxf(mv, __uint_as_float(Red[2][i]));
    }
    int e;
    if (mv > 0.f && isfinite(mv)) {
      frexpf(mv, &e);                                   // mv = m 2^e, m in [0.5, 1)
      ev = max(-100, min(100, 15 - e));
    }
    mq *= fabsf(a.scale_log2);
    if (mq > 0.f && mk > 0.f && isfinite(mq) && isfinite(mk)) {
      int eq;
      frexpf(mq, &eq);
      frexpf(mk, &e);
      ek = max(-60, min(60, (eq - e) / 2));
    }
  }
  fk = ldexpf(1.f, ek);
  fv = ldexpf(1.f, ev);

  // resident Q operands (term g of lane group g), running state
  u4 Qop[NQT];
  f4 Cm[NQT], O[NQT][RC];
  float m[NQT], lsum[NQT];
  uint32_t rk[NQT][RC], wb[NQT][RC];
#pragma unroll
  for (int n = 0; n < NQT; ++n) {
    const int q = qb * QB + 16 * (NQT * w + n) + c;
    const int qc = min(q, a.Lq - 1);
    const float s = ldexpf(a.scale_log2, -ek);
    float x[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) x[f] = xq[n][f] * s;
    u4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hi[j] = pk_hi(x[2 * j], x[2 * j + 1]);
      lo[j] = pk_lo(x[2 * j], x[2 * j + 1], hi[j]);
    }
    const u4 ones = {ONES_F16X2, 0u, 0u, 0u};
    Qop[n] = g == 3 ? ones : (g == 1 ? lo : hi);
    m[n] = M_INIT;
    Cm[n] = splat(7.f - M_INIT);
    lsum[n] = 0.f;
#pragma unroll
    for (int rc = 0; rc < RC; ++rc) {
      O[n][rc] = splat(0.f);
      wb[n][rc] = 0u;
      rk[n][rc] = DROP ? attn_row_key(skey, (uint32_t)((seq_of(rc) * a.H + h) * a.Lq + qc)) : 0u;
    }
  }
  // K image term of lane group g: hi, hi, lo, bias (lo / bias swapped for keys 4..11 of a
  // tile: the upper lane groups' reads conflict-free)
  const int ksw = ((c + 4) >> 3) & 1;
  const int toff = g == 2 ? 4 + 4 * ksw : (g == 3 ? 8 - 4 * ksw : 0);

  auto commit = [&](int ks, int buf) {
    uint32_t* K_ = Ki[buf] + kk_i * 12;
    const float4 k4 = make_float4(rK.x * fk, rK.y * fk, rK.z * fk, rK.w * fk);
    const float2 va = make_float2(rV0.x * fv, rV0.y * fv), vb = make_float2(rV1.x * fv, rV1.y * fv);
    const uint32_t h0 = pk_hi(k4.x, k4.y), h1 = pk_hi(k4.z, k4.w);
    *reinterpret_cast<uint2*>(K_ + 2 * hf) = make_uint2(h0, h1);
    const int kx = 4 * (((kk_i + 4) >> 3) & 1);
    *reinterpret_cast<uint2*>(K_ + 4 + kx + 2 * hf) = make_uint2(pk_lo(k4.x, k4.y, h0), pk_lo(k4.z, k4.w, h1));
    *reinterpret_cast<uint2*>(K_ + 8 - kx + 2 * hf) = make_uint2(hf == 0 ? pack2(f16_hi(rB), f16_lo(rB)) : 0u, 0u);
    // V^T of pair w: slot of key kq in it 8 gg + 4 tt + jj (kq = 16 tt + 4 gg + jj); keys
    // 2 vp, 2 vp + 1 are neighbouring slots: one word per row (hi rows 2 vf, 2 vf + 1, lo + 8)
    const int kq = 2 * vp;
    uint32_t* V_ = Vi[buf] + w * 384 + (8 * ((kq & 15) >> 2) + 4 * (kq >> 4) + (kq & 3)) / 2;
    const uint32_t v0 = pk_hi(va.x, vb.x), v1 = pk_hi(va.y, vb.y);
    V_[(2 * vf) * 24] = v0;
    V_[(2 * vf + 1) * 24] = v1;
    V_[(8 + 2 * vf) * 24] = pk_lo(va.x, vb.x, v0);
    V_[(9 + 2 * vf) * 24] = pk_lo(va.y, vb.y, v1);
    if (DROP && hf == 0 && (kk_i & 1) == 0)
      Kp[buf][kk_i >> 1] = attn_keypair_mix(skey, (uint32_t)((ks + kk_i) >> 1));
  };

  const int nch = (a.Lk + KC - 1) / KC;
  const int Tlast = 2 * ((a.Lk + 31) / 32) - 1;     // last 16-key tile processed (pairs)
  commit(0, 0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int ks = ch * KC, buf = ch & 1;
    if (ch + 1 < nch) issue(ks + KC);
    const uint32_t* K_ = Ki[buf];
    const uint32_t* V_ = Vi[buf];
    for (int p = 0; p < NW; ++p) {
      if (ks + 32 * p >= a.Lk) break;
      const u4 A0 = ldu4(K_ + (32 * p + c) * 12 + toff);
      const u4 A1 = ldu4(K_ + (32 * p + 16 + c) * 12 + toff);
      const u4 VT = ldu4(V_ + p * 384 + c * 24 + g * 4);
      f4 S0[NQT], S1[NQT];
#pragma unroll
      for (int n = 0; n < NQT; ++n) {
        S0[n] = mma(A0, Qop[n], Cm[n]);
        S1[n] = mma(A1, Qop[n], Cm[n]);
      }
      uint32_t kpm[4] = {0u, 0u, 0u, 0u};
      if (DROP) {   // key pairs of this lane: tile 2p keys 32p + 4g + {0,1}, {2,3}; tile 2p+1 + 16
        const uint32_t* kp = Kp[buf] + 16 * p + 2 * g;
        kpm[0] = kp[0]; kpm[1] = kp[1]; kpm[2] = kp[8]; kpm[3] = kp[9];
      }
      const int T0 = ks / 16 + 2 * p;
#pragma unroll
      for (int n = 0; n < NQT; ++n) {
        // lazy origin: p' <= 2^15 while no score passes m by more than 8.  Tested on the bit
        // patterns (scores are never NaN; a negative one is a negative integer): an integer
        // max needs no NaN canonicalisation (v_max3_i32)
        if (__builtin_amdgcn_ballot_w64(imax8(S0[n], S1[n]) > (int)0x41700000)) {   // > 15.f
          const f4 z = splat(0.f);
          const f4 R0 = mma(A0, Qop[n], z), R1 = mma(A1, Qop[n], z);
          float x = fmaxf(max4(R0), max4(R1));
          x = xmax32(x);
          x = xmax16(x);                     // the column's max over its four lane groups
          const float mn = fmaxf(m[n], x);
          const float al = ex2(m[n] - mn);
          lsum[n] *= al;
#pragma unroll
          for (int rc = 0; rc < RC; ++rc) O[n][rc] *= al;
          m[n] = mn;
          const float cc = 7.f - mn;
          Cm[n] = splat(cc);
          S0[n] = R0 + cc;
          S1[n] = R1 + cc;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          S0[n][r] = ex2(S0[n][r]);
          S1[n][r] = ex2(S1[n][r]);
        }
        lsum[n] += ((S0[n][0] + S0[n][1]) + (S0[n][2] + S0[n][3])) +
                   ((S1[n][0] + S1[n][1]) + (S1[n][2] + S1[n][3]));
        if (DROP && RC == 1) {   // one copy: the keep mask on p', then its split (as before r06)
          const int q = qb * QB + 16 * (NQT * w + n) + c;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            f4& P = u ? S1[n] : S0[n];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const uint32_t bits = attn_pair_bits_mixed(rk[n][0], kpm[2 * u + j]);
              const bool klo = (bits & 0xffffu) >= a.thr, khi = (bits >> 16) >= a.thr;
              wb[n][0] = push_bit(push_bit(wb[n][0], __builtin_amdgcn_ballot_w64(klo)),
                                  __builtin_amdgcn_ballot_w64(khi));
              P[2 * j] = klo ? P[2 * j] : 0.f;
              P[2 * j + 1] = khi ? P[2 * j + 1] : 0.f;
            }
            const int Tg = T0 + u;
            if ((Tg & 7) == 7 || Tg == Tlast) {
              if (q < a.Lq)
                a.bits[(((seq_of(0) * a.H + h) * NT8 + (Tg >> 3)) * 4 + g) * Lqp + q] =
                    keep_word(wb[n][0], 4 * ((Tg & 7) + 1));
              wb[n][0] = 0u;
            }
          }
        }
        // p' as hi / lo pair words: [t0 keys 0,1 | t0 keys 2,3 | t1 keys 0,1 | t1 keys 2,3]
        u4 Bh, Bl;
        Bh[0] = pk_hi(S0[n][0], S0[n][1]);
        Bh[1] = pk_hi(S0[n][2], S0[n][3]);
        Bh[2] = pk_hi(S1[n][0], S1[n][1]);
        Bh[3] = pk_hi(S1[n][2], S1[n][3]);
        Bl[0] = pk_lo1(S0[n][0], S0[n][1], Bh[0], one);
        Bl[1] = pk_lo1(S0[n][2], S0[n][3], Bh[1], one);
        Bl[2] = pk_lo1(S1[n][0], S1[n][1], Bh[2], one);
        Bl[3] = pk_lo1(S1[n][2], S1[n][3], Bh[3], one);
        if (DROP && RC > 1) {    // copies: the split is shared, each copy masks the words
          const int q = qb * QB + 16 * (NQT * w + n) + c;
#pragma unroll
          for (int rc = 0; rc < RC; ++rc) {
            u4 Mh, Ml;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const uint32_t bits = attn_pair_bits_mixed(rk[n][rc], kpm[2 * u + j]);
                const bool klo = (bits & 0xffffu) >= a.thr, khi = (bits >> 16) >= a.thr;
                wb[n][rc] = push_bit(push_bit(wb[n][rc], __builtin_amdgcn_ballot_w64(klo)),
                                     __builtin_amdgcn_ballot_w64(khi));
                const uint32_t m = (klo ? 0x0000FFFFu : 0u) | (khi ? 0xFFFF0000u : 0u);
                Mh[2 * u + j] = Bh[2 * u + j] & m;
                Ml[2 * u + j] = Bl[2 * u + j] & m;
              }
              const int Tg = T0 + u;
              if ((Tg & 7) == 7 || Tg == Tlast) {
                if (q < a.Lq && r0 + rc < R)
                  a.bits[(((seq_of(rc) * a.H + h) * NT8 + (Tg >> 3)) * 4 + g) * Lqp + q] =
                      keep_word(wb[n][rc], 4 * ((Tg & 7) + 1));
                wb[n][rc] = 0u;
              }
            }
            O[n][rc] = mma(VT, Mh, O[n][rc]);
            O[n][rc] = mma(VT, Ml, O[n][rc]);
          }
        } else {
          O[n][0] = mma(VT, Bh, O[n][0]);
          O[n][0] = mma(VT, Bl, O[n][0]);
        }
      }
    }
    if (ch + 1 < nch) commit(ks + KC, buf ^ 1);
    __syncthreads();
  }
  // rows f (lane groups 0, 1) + rows f + 8 (groups 2, 3); l over the column's four groups
  const float ik = ldexpf(DROP ? a.inv_keep : 1.f, -ev);     // and v' = v 2^ev back
#pragma unroll
  for (int n = 0; n < NQT; ++n) {
    const float lt = xsum16(xsum32(lsum[n]));
    const float sc = ik / lt;        // l == 0 (every key masked) -> NaN, as the reference
    const int q = qb * QB + 16 * (NQT * w + n) + c;
#pragma unroll
    for (int rc = 0; rc < RC; ++rc) {
      f4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = xsum32(O[n][rc][r]) * sc;
      if (q < a.Lq && g < 2) {
        // without dropout every copy is the same: copy 0's accumulator goes to all R of them
        const int nst = DROP ? (r0 + rc < R ? 1 : 0) : R;
        for (int i = 0; i < nst; ++i) {
          const int64_t sq = DROP ? seq_of(rc) : (int64_t)i * Bd + b;
          *reinterpret_cast<float4*>(a.o_out + sq * a.o_bs + (int64_t)q * a.o_ls + h * 8 + 4 * g) =
              make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    if (blockIdx.y == 0 && q < a.Lq && g == 0) a.lse[(int64_t)bh * a.Lq + q] = m[n] + __log2f(lt) - 7.f;
  }
}

// =================================== backward ===================================
// Workgroup: NW waves (<= 8), wave w owns the 128 keys kb*128NW + 128w + 16t + c
// (t = 0..7 key tiles), the lane holding key c of each tile; queries stream in tiles of 16.
// Per (key tile, query tile), with the key on the lane and 4 queries per lane group:
//   S' = Q K^T + bias + (14 - lse)        (C: the row constant)  -> p' = exp2(S') = 2^14 P
//   dP' = dO' V'^T - D'                    (C: -D' = -2^s D)
//   t = keep ? dP' : -D',  dS'' = p' t     (= 2^(14+s) dS)
//   dV^T += dO'^T [keep p']   dK^T += Q^T dS''   (B: the lane's four values as hi / lo pairs)
//   dQ^T += K^T dS''^T: dS'' crosses a wave-private LDS image once (8-byte row writes,
//   ds_read_b64_tr_b16 column reads), K^T from a per-wave image built in the prologue.
// dQ of a query tile is summed over the waves in LDS and stored (or, with several key blocks
// per sequence, stored as a partial and summed after the launch).  Prologue: D = rowsum(dO O)
// per query and the maxima of |dO|, |D|, |v| choose the powers of two 2^s (|t| <= 2, so
// |dS''| <= 2^15) and 2^cs (dO' = dO sd 2^(s+cs), v' = v 2^-cs: balanced magnitudes).
constexpr int BNW_MAX = 8;
constexpr int BKT = 8;             // key tiles per wave
constexpr int BLQ_MAX = 2048;      // queries of the prologue arrays
// dS'' transpose image: 32 rows of 4 eight-byte chunks (16 queries as f16); chunk j of row r
// at dword sc_at(r, j).  Rows padded 16 dwords per 4 and chunks XOR-swizzled per 8 rows:
// the writes (ds_write_b64, 16-lane groups, 32 banks) and the transposed reads
// (ds_read_b64_tr_b16, 32-lane halves, 64 banks) are both conflict-free (plain 8-dword rows
// were 8-way / 2-way: SQ_LDS_BANK_CONFLICT 27 % of the wave cycles)
constexpr int SC_WORDS = 368;
__device__ __forceinline__ int sc_at(int r, int j) {
  return r * 8 + 2 * (j ^ ((r >> 3) & 3)) + 16 * (r >> 2);
}

// Transposed A-operand images (K^T, Q^T, dO'^T: 16 rows of 32 f16, 16 dwords): the 4-dword
// chunk g of row r sits at chunk g ^ tsw(r), so the operand reads (ds_read_b128, 16-lane
// groups over 64 banks: rows c, c + 4 of one chunk collide at the plain 16-dword stride) are
// conflict-free
__device__ __forceinline__ int tsw(int r) { return (r >> 1) & 2; }

template <bool DROP>
__global__ __launch_bounds__(512, 2) void attn_bwd_sf16_kernel(AttnArgs a, int nkb, int NT8, int Lqp) {
  __shared__ __attribute__((aligned(16))) float Cs_l[BLQ_MAX];     // 14 - lse (-inf past Lq)
  __shared__ __attribute__((aligned(16))) float Cd_l[BLQ_MAX];     // D, then -2^s D
  // sized by the launch's wave count (bwd_lds_bytes): K^T A operands [NW][BKT][256], the
  // dS'' transpose images [NW][2][SC_WORDS], the dQ partials [2][NW * 128] -- a key-split
  // launch of 2 or 4 waves then leaves room for more workgroups per CU
  extern __shared__ __attribute__((aligned(16))) uint32_t bwd_dyn[];
  // staged query tile: Q A operand [16][hi | lo | ones], dO' [16][hi | lo | 0], Q^T and
  // dO'^T A operands [16 rows][32 slots]
  __shared__ __attribute__((aligned(16))) uint32_t Qa[2][16 * 12];
  __shared__ __attribute__((aligned(16))) uint32_t Da[2][16 * 12];
  __shared__ __attribute__((aligned(16))) uint32_t QT[2][256];
  __shared__ __attribute__((aligned(16))) uint32_t DT[2][256];
  __shared__ float Red[3][BNW_MAX];
  const int NW = blockDim.x >> 6, KB = 128 * NW;
  uint32_t* const KTi = bwd_dyn;
  uint32_t* const Sc = bwd_dyn + NW * BKT * 256;
  float* const Qp = reinterpret_cast<float*>(Sc + NW * 2 * SC_WORDS);
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, c = l & 15;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int kb = wg % nkb, bh = wg / nkb;
  const float one = opaque_one();
  const int b = bh / a.H, h = bh - b * a.H;
  const int key0 = kb * KB + 128 * w;
  const int ntile = key0 < a.Lk ? min(BKT, (a.Lk - key0 + 15) / 16) : 0;   // wave-uniform
  // query chunk blockIdx.y (a.qchunk > 0: few (sequence, head) pairs; dK / dV partials at
  // + blockIdx.y * a.dk_ss, summed after the launch): query tiles [it0, it1)
  const int qc0 = a.qchunk > 0 ? (int)blockIdx.y * a.qchunk : 0;
  const int it0 = qc0 / 16;
  const int it1 = a.qchunk > 0 ? min((a.Lq + 15) / 16, (qc0 + a.qchunk) / 16) : (a.Lq + 15) / 16;
  const int Lq16 = 16 * it1;
  const float* qg = a.q + (int64_t)b * a.q_bs + h * 8;
  const float* dg = a.dout + (int64_t)b * a.do_bs + h * 8;
  const float* og = a.o + (int64_t)b * a.o_bs + h * 8;

  // ---- prologue: D, row constants, maxima ----
  float mdo = 0.f, md = 0.f, mv = 0.f;
  for (int q = 16 * it0 + t; q < Lq16; q += blockDim.x) {
    float D = 0.f, cs = -INFINITY;
    if (q < a.Lq) {
      const float* dp = dg + (int64_t)q * a.do_ls;
      const float* op = og + (int64_t)q * a.o_ls;
      const float4 d0 = *reinterpret_cast<const float4*>(dp), d1 = *reinterpret_cast<const float4*>(dp + 4);
      const float4 o0 = *reinterpret_cast<const float4*>(op), o1 = *reinterpret_cast<const float4*>(op + 4);
      const float dd[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
      const float oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        D = fmaf(dd[f], oo[f], D);
        mdo = fmaxf(mdo, fabsf(dd[f]));
      }
      md = fmaxf(md, fabsf(D));
      cs = 14.f - a.lse[(int64_t)bh * a.Lq + q];
    }
    Cd_l[q] = D;
    Cs_l[q] = cs;
  }
  // resident K operands, K^T image, max |v|
  u4 Kop[BKT], Vop[BKT];
  const float* kg = a.k + (int64_t)b * a.k_bs + h * 8;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * 8;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  _Float16* KT_ = reinterpret_cast<_Float16*>(KTi + (w * BKT) * 256);
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    Kop[tt] = (u4){0u, 0u, 0u, 0u};
    {   // every tile, past-Lk keys too (zero K / V, bias -inf): no per-tile branch
      const int key = key0 + 16 * tt + c;
      const bool ok = key < a.Lk;
      const int64_t kc = min(key, a.Lk - 1);
      float kr[8], vr[8];
      {
        const float4 k0 = *reinterpret_cast<const float4*>(kg + kc * a.k_ls);
        const float4 k1 = *reinterpret_cast<const float4*>(kg + kc * a.k_ls + 4);
        const float4 v0 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls);
        const float4 v1 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls + 4);
        const float kk[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
        const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          kr[f] = ok ? kk[f] : 0.f;
          vr[f] = ok ? vv[f] : 0.f;
          mv = fmaxf(mv, fabsf(vr[f]));
        }
      }
      const float bias = ok ? (kbg ? kbg[key] : 0.f) : -INFINITY;
      u4 hi, lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hi[j] = pk_hi(kr[2 * j], kr[2 * j + 1]);
        lo[j] = pk_lo(kr[2 * j], kr[2 * j + 1], hi[j]);
      }
      const u4 bs = {pack2(f16_hi(bias), f16_lo(bias)), 0u, 0u, 0u};
      Kop[tt] = g == 3 ? bs : (g == 1 ? lo : hi);
      // K^T image of tile tt: row f (hi) / f + 8 (lo), slot 8 gs + j <-> (key 4 gs + 2 (j/4) +
      // j%2, precision (j/2)%2); this lane (key c) writes features 2g, 2g + 1
      const int gs = c >> 2, jb = 4 * ((c & 3) >> 1) + (c & 1);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int f = 2 * g + e;
        const _Float16 kh = f16_hi(kr[f]), kl = f16_lo(kr[f]);
        _Float16* row = KT_ + tt * 512 + f * 32 + 8 * (gs ^ tsw(f)) + jb;
        row[0] = kh;                 // (hi row, prec 0)
        row[2] = kh;                 // (hi row, prec 1)
        row[8 * 32] = kl;            // (lo row, prec 0)
        row[8 * 32 + 2] = (_Float16)0.f;
      }
    }
  }
  // maxima over the workgroup
  mdo = wave_max(mdo);
  md = wave_max(md);
  mv = wave_max(mv);
  if (l == 0) {
    Red[0][w] = mdo;
    Red[1][w] = md;
    Red[2][w] = mv;
  }
  __syncthreads();
  float Mdo = 0.f, Md = 0.f, Mv = 0.f;
  for (int i = 0; i < NW; ++i) {
    Mdo = fmaxf(Mdo, Red[0][i]);
    Md = fmaxf(Md, Red[1][i]);
    Mv = fmaxf(Mv, Red[2][i]);
  }
  const float sd = DROP ? a.inv_keep : 1.f;
  const float bnd = 8.f * Mdo * sd * Mv + Md;       // >= |keep sd dP - D|
  int s = 0;
  if (bnd > 0.f && isfinite(bnd)) {
    int e;
    frexpf(bnd, &e);                                  // bnd = m 2^e, m in [0.5, 1)
    s = max(-100, min(100, 1 - e));                   // 2^s bnd < 2
  }
  int cs = 0;
  if (Mdo > 0.f && Mv > 0.f && isfinite(Mdo) && isfinite(Mv))
    cs = max(-30, min(30, (int)rintf(0.5f * (log2f(Mv) - log2f(Mdo * sd) - (float)s))));
  const float fdo = ldexpf(sd, s + cs), fv = ldexpf(1.f, -cs), fd = ldexpf(1.f, s);
  for (int q = 16 * it0 + t; q < Lq16; q += blockDim.x) Cd_l[q] *= -fd;
  // resident V' operands
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    Vop[tt] = (u4){0u, 0u, 0u, 0u};
    {   // every tile, past-Lk keys too (zero K / V, bias -inf): no per-tile branch
      const int key = key0 + 16 * tt + c;
      const bool ok = key < a.Lk;
      const int64_t kc = min(key, a.Lk - 1);
      const float4 v0 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls);
      const float4 v1 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls + 4);
      const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      float vr[8];
#pragma unroll
      for (int f = 0; f < 8; ++f) vr[f] = ok ? vv[f] * fv : 0.f;
      u4 hi, lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hi[j] = pk_hi(vr[2 * j], vr[2 * j + 1]);
        lo[j] = pk_lo(vr[2 * j], vr[2 * j + 1], hi[j]);
      }
      Vop[tt] = g == 3 ? (u4){0u, 0u, 0u, 0u} : (g == 1 ? lo : hi);
    }
  }
  f4 dV[BKT], dK[BKT];
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    dV[tt] = splat(0.f);
    dK[tt] = splat(0.f);
  }

  // ---- query tiles ----
  // staging item (threads 0..63): query qi = t >> 2 of the tile, part 0/1: q features
  // 4 part.., part 2/3: dO features
  const int qi = t >> 2, part = t & 3;
  float4 rX = make_float4(0.f, 0.f, 0.f, 0.f);
  auto issue = [&](int q0) {
    if (t >= 64) return;
    const int q = q0 + qi;
    if (q >= a.Lq) {
      rX = make_float4(0.f, 0.f, 0.f, 0.f);
      return;
    }
    const float* src = part < 2 ? qg + (int64_t)q * a.q_ls + 4 * part
                                : dg + (int64_t)q * a.do_ls + 4 * (part - 2);
    rX = *reinterpret_cast<const float4*>(src);
  };
  auto commit = [&](int buf) {
    if (t >= 64) return;
    const bool isq = part < 2;
    const int f0 = 4 * (part & 1);
    const float m_ = isq ? a.scale_log2 : fdo;
    const float x[4] = {rX.x * m_, rX.y * m_, rX.z * m_, rX.w * m_};
    uint32_t* A_ = (isq ? Qa[buf] : Da[buf]) + qi * 12;
    const uint32_t h0 = pk_hi(x[0], x[1]), h1 = pk_hi(x[2], x[3]);
    A_[(f0 >> 1)] = h0;
    A_[(f0 >> 1) + 1] = h1;
    A_[4 + (f0 >> 1)] = pk_lo(x[0], x[1], h0);
    A_[5 + (f0 >> 1)] = pk_lo(x[2], x[3], h1);
    if (f0 == 0) {
      A_[8] = isq ? ONES_F16X2 : 0u;
      A_[9] = 0u;
    } else {
      A_[10] = 0u;
      A_[11] = 0u;
    }
    // transposed A operand: rows f / f + 8, slots 8 gs + i (precision 0) and 8 gs + 4 + i
    // (precision 1) of query qi = 4 gs + i (B: [hi(q0, q1) | hi(q2, q3) | lo(q0, q1) | lo(q2, q3)])
    _Float16* T_ = reinterpret_cast<_Float16*>(isq ? QT[buf] : DT[buf]);
    const int gs = qi >> 2, j0 = qi & 3;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = f0 + e;
      const _Float16 xh = f16_hi(x[e]), xl = f16_lo(x[e]);
      _Float16* row = T_ + f * 32 + 8 * (gs ^ tsw(f)) + j0;
      row[0] = xh;
      row[4] = xh;
      row[8 * 32] = xl;
      row[8 * 32 + 4] = (_Float16)0.f;
    }
  };
  // keep words of this lane: 4 queries (q0 + 4g + r), key residue c, the wave's 128 keys
  const uint32_t* bitw = DROP && ntile > 0
                             ? a.bits + (((int64_t)bh * NT8 + (kb * NW + w)) * 4 + (c >> 2)) * Lqp + 4 * g
                             : nullptr;
  auto words = [&](int q0) -> u4 {
    if (!DROP || ntile == 0 || q0 >= a.Lq) return (u4){0u, 0u, 0u, 0u};
    return *reinterpret_cast<const u4*>(bitw + q0);
  };
  // dQ unscale: 2^-(14+s) * scale; dK: 2^-(14+s) * scale / scale_log2; dV: 2^-(14+s+cs)
  const float uq = ldexpf(a.scale, -14 - s);
  float* dqb = a.dq + (nkb > 1 ? (int64_t)kb * a.dq_ss : 0) + (int64_t)b * a.dq_bs + h * 8;
  auto dq_reduce = [&](int q0, int buf) {
    for (int i0 = t; i0 < 128; i0 += blockDim.x) {
      const int qq = i0 >> 3, f = i0 & 7;
      float acc = 0.f;
      for (int i = 0; i < NW; ++i) acc += Qp[buf * NW * 128 + i * 128 + qq * 8 + f];
      if (q0 + qq < a.Lq) dqb[(int64_t)(q0 + qq) * a.dq_ls + f] = acc * uq;
    }
  };

  issue(16 * it0);
  u4 kw = words(16 * it0);
  commit(0);
  __syncthreads();
  for (int it = it0; it < it1; ++it) {
    const int q0 = 16 * it, buf = (it - it0) & 1;
    if (it > it0) dq_reduce(q0 - 16, buf ^ 1);
    if (it + 1 < it1) issue(q0 + 16);
    const u4 kwn = it + 1 < it1 ? words(q0 + 16) : (u4){0u, 0u, 0u, 0u};
    f4 dQa = splat(0.f);
    if (ntile > 0) {
      const u4 QA = ldu4(Qa[buf] + c * 12 + (g == 2 ? 4 : (g == 3 ? 8 : 0)));
      const u4 DA = ldu4(Da[buf] + c * 12 + (g == 2 ? 4 : (g == 3 ? 8 : 0)));
      const u4 QTA = ldu4(QT[buf] + c * 16 + 4 * (g ^ tsw(c)));
      const u4 DTA = ldu4(DT[buf] + c * 16 + 4 * (g ^ tsw(c)));
      const f4 CS = *reinterpret_cast<const f4*>(Cs_l + q0 + 4 * g);
      const f4 CD = *reinterpret_cast<const f4*>(Cd_l + q0 + 4 * g);
#pragma unroll
      for (int tt = 0; tt < BKT; ++tt) {
        {   // every tile, past-Lk keys too (zero K / V, bias -inf): no per-tile branch
          const f4 S = mma(QA, Kop[tt], CS);
          // with dropout dP' without the row constant: dS'' = p' keep dP' + p' (-D') = fma(Pd,
          // dP', p' C) (the keep select folded into the masked p' the dV product needs anyway)
          const f4 dP = mma(DA, Vop[tt], DROP ? splat(0.f) : CD);
          float P[4], Pd[4], dS[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            P[r] = ex2(S[r]);
            if (DROP) {
              const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int)kw[r], 4 * tt + (c & 3), 1);
              Pd[r] = __uint_as_float(as_u(P[r]) & mk);
              dS[r] = fmaf(Pd[r], dP[r], P[r] * CD[r]);
            } else {
              Pd[r] = P[r];
              dS[r] = P[r] * dP[r];
            }
          }
          u4 Bv, Bk;
          Bv[0] = pk_hi(Pd[0], Pd[1]);
          Bv[1] = pk_hi(Pd[2], Pd[3]);
          Bv[2] = pk_lo1(Pd[0], Pd[1], Bv[0], one);
          Bv[3] = pk_lo1(Pd[2], Pd[3], Bv[1], one);
          Bk[0] = pk_hi(dS[0], dS[1]);
          Bk[1] = pk_hi(dS[2], dS[3]);
          Bk[2] = pk_lo1(dS[0], dS[1], Bk[0], one);
          Bk[3] = pk_lo1(dS[2], dS[3], Bk[1], one);
          dV[tt] = mma(DTA, Bv, dV[tt]);
          dK[tt] = mma(QTA, Bk, dK[tt]);
          // dS'' through LDS: row R = 4 (c/2) + 2 prec + c%2 holds queries 0..15 (32 B)
          uint32_t* sc = Sc + (w * 2 + (tt & 1)) * SC_WORDS;
          const int R = 4 * (c >> 1) + (c & 1);
          *reinterpret_cast<uint2*>(sc + sc_at(R, g)) = make_uint2(Bk[0], Bk[1]);
          *reinterpret_cast<uint2*>(sc + sc_at(R + 2, g)) = make_uint2(Bk[2], Bk[3]);
          // (the wave's LDS operations complete in order: the transposed reads see these rows)
          // B[slot 8g + j][query c] = row 8g + j: two 4-row transposed reads
          const int rq = (c >> 2), cp = (c & 3);
          const s4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(sc + sc_at(8 * g + rq, cp)));
          const s4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(sc + sc_at(8 * g + 4 + rq, cp)));
          const u4 Bq = {__builtin_bit_cast(uint2, r0).x, __builtin_bit_cast(uint2, r0).y,
                         __builtin_bit_cast(uint2, r1).x, __builtin_bit_cast(uint2, r1).y};
          const u4 KA = ldu4(KTi + (w * BKT + tt) * 256 + c * 16 + 4 * (g ^ tsw(c)));
          dQa = mma(KA, Bq, dQa);
        }
      }
    }
    // this wave's dQ partial: rows f (groups 0, 1) + f + 8 (groups 2, 3)
    f4 dq;
#pragma unroll
    for (int r = 0; r < 4; ++r) dq[r] = xsum32(dQa[r]);
    if (g < 2) *reinterpret_cast<f4*>(Qp + buf * NW * 128 + w * 128 + c * 8 + 4 * g) = dq;
    if (it + 1 < it1) commit(buf ^ 1);
    kw = kwn;
    __syncthreads();
  }
  dq_reduce(16 * (it1 - 1), (it1 - 1 - it0) & 1);
  // dK, dV: rows f + rows f + 8
  const float uk = ldexpf(a.scale / a.scale_log2, -14 - s), uv = ldexpf(1.f, -14 - s - cs);
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    if (tt < ntile) {
      f4 v, k_;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = xsum32(dV[tt][r]) * uv;
        k_[r] = xsum32(dK[tt][r]) * uk;
      }
      const int key = key0 + 16 * tt + c;
      if (g < 2 && key < a.Lk) {
        const int64_t part = (int64_t)blockIdx.y * a.dk_ss;
        *reinterpret_cast<float4*>(a.dv + part + (int64_t)b * a.dv_bs + (int64_t)key * a.dv_ls + h * 8 + 4 * g) =
            make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(a.dk + part + (int64_t)b * a.dk_bs + (int64_t)key * a.dk_ls + h * 8 + 4 * g) =
            make_float4(k_[0], k_[1], k_[2], k_[3]);
      }
    }
  }
}

// ============================ backward, repeated sequences ============================
// The decoders' first block (SpectraLayers.py:54-62, PhotometricLayers.py:59-67): q, k, v of
// Bd distinct sequences, R copies each with their own dO, O and keep bits (copy r of distinct
// sequence b is sequence r Bd + b).  Q, K and V are shared, so their gradients are sums over
// the copies; per (key tile, query tile) the scores and P are computed once and
//   acc = sum_c keep_c dP''_c         (dP''_c = dO''_c V''^T on MFMA, C = acc, keep by v_bfi)
//   dV^T += dO''_c^T [keep_c p']      (per copy; B = p' as hi / lo pair words, halves masked)
//   dS'' = p' (fm acc - sum_c D'_c)   (once; dK^T += Q^T dS'', dQ^T += K^T dS''^T as the
//                                      plain kernel, dS'' through the LDS transpose image)
// Workgroup: NW waves x 8 key tiles of 16 (the whole key axis: L <= 1024), a chunk of qchunk
// queries (grid.y = query chunks; dK / dV of each chunk a partial, summed after the launch,
// dQ complete).  Query tiles of 16 stream through LDS with every copy's dO'_c operands (copies
// staged RG at a time); each wave walks its key tiles in two halves of four (P, its words and
// acc of four tiles live across the copy loop).  Prologue: D_c = rowsum(dO_c O_c) summed over
// the copies per query, the maxima of |dO|, |sum D|, |v| choose the powers of two: 2^s so that
// |dS''| <= 2^15 with R copies summed (bound R (8 |dO| sd |v|) + |sum D|), and the operand scales
// of dO'' and v'' (maxima in [2^6, 2^7): normal f16 lo parts).
constexpr int RB_NW_MAX = 8;
constexpr int RB_RG = 16;            // copies per staged group
constexpr int RB_QCH_MAX = 512;      // queries of a chunk (prologue arrays)
constexpr int RB_LMAX = 1024;        // sequence length of the path (8 waves x 128 keys)
// dS'' transpose image: ONE per wave (a wave's LDS operations complete in order, so the next
// tile's writes never overtake this tile's transposed reads)
size_t rep_bwd_lds_bytes(int nw) {
  return (size_t)nw * (BKT * 256 + SC_WORDS + 2 * 128) * sizeof(uint32_t);
}

template <bool DROP>
__global__ __launch_bounds__(512, 2) void attn_rep_bwd_sf16_kernel(AttnArgs a, int R, int QS, int NT8, int Lqp) {
  __shared__ __attribute__((aligned(16))) float Cs_l[RB_QCH_MAX];     // 14 - lse (-inf past Lq)
  __shared__ __attribute__((aligned(16))) float Cd_l[RB_QCH_MAX];     // sum_c D_c, then -2^s of it
  // copy operands of the staged query tile: dO'_c A operand [RG][16][hi | lo | 0] and the dO'^T
  // image [RG][256]; during the prologue the per-copy D_c [RG][chunk] scratch
  __shared__ __attribute__((aligned(16))) uint32_t Ca[RB_RG * 16 * 12];
  __shared__ __attribute__((aligned(16))) uint32_t Ct[RB_RG * 256];
  // K^T A operands [NW][BKT][256], dS'' transpose images [NW][SC_WORDS], dQ partials [2][NW * 128]
  extern __shared__ __attribute__((aligned(16))) uint32_t bwd_dyn[];
  __shared__ __attribute__((aligned(16))) uint32_t Qa[16 * 12];
  __shared__ __attribute__((aligned(16))) uint32_t QT[256];
  // the staged step's keep words: [wave][copy][key group (key % 16) / 4][16 queries]
  __shared__ __attribute__((aligned(16))) uint32_t Kw[RB_NW_MAX * RB_RG * 64];
  __shared__ float Red[3][RB_NW_MAX];
  const int NW = blockDim.x >> 6;
  uint32_t* const KTi = bwd_dyn;
  uint32_t* const Sc = bwd_dyn + NW * BKT * 256;
  float* const Qp = reinterpret_cast<float*>(Sc + NW * SC_WORDS);
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, c = l & 15;
  const int wg = xcd_swizzle(blockIdx.x, gridDim.x);
  const int qs = wg % QS, bh = wg / QS;
  const float one = opaque_one();
  const int b = bh / a.H, h = bh - b * a.H;
  const int Bd = a.B;
  const int key0 = 128 * w;
  const int ntile = key0 < a.Lk ? min(BKT, (a.Lk - key0 + 15) / 16) : 0;   // wave-uniform
  const int qbeg = qs * a.qchunk, qend = min(a.Lq, qbeg + a.qchunk);
  const int nq = qend - qbeg, nqt = (nq + 15) / 16;
  const float* qg = a.q + (int64_t)b * a.q_bs + h * 8;
  auto seq = [&](int r) { return (int64_t)r * Bd + b; };
  auto dorow = [&](int r, int q) { return a.dout + seq(r) * a.do_bs + (int64_t)q * a.do_ls + h * 8; };

  // ---- prologue: sum_c D_c, row constants, maxima ----
  float mdo = 0.f, md = 0.f, mv = 0.f;
  float* const Dc = reinterpret_cast<float*>(Ca);      // scratch [RG][nq] before the first tile
  const int qcap = (RB_RG * 16 * 12) / RB_RG;            // queries of the scratch per pass (192)
  for (int q = t; q < 16 * nqt; q += blockDim.x) {
    Cd_l[q] = 0.f;
    Cs_l[q] = qbeg + q < qend ? 14.f - a.lse[(int64_t)bh * a.Lq + qbeg + q] : -INFINITY;
  }
  for (int r0 = 0; r0 < R; r0 += RB_RG) {
    const int ng = min(RB_RG, R - r0);
    for (int q0 = 0; q0 < nq; q0 += qcap) {
      const int nqq = min(qcap, nq - q0);
      __syncthreads();
      for (int i = t; i < ng * nqq; i += blockDim.x) {
        const int rc = i / nqq, qq = i - rc * nqq, q = qbeg + q0 + qq;
        const float* dp = dorow(r0 + rc, q);
        const float* op = a.o + seq(r0 + rc) * a.o_bs + (int64_t)q * a.o_ls + h * 8;
        const float4 d0 = *reinterpret_cast<const float4*>(dp), d1 = *reinterpret_cast<const float4*>(dp + 4);
        const float4 o0 = *reinterpret_cast<const float4*>(op), o1 = *reinterpret_cast<const float4*>(op + 4);
        const float dd[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        const float oo[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
        float D = 0.f;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          D = fmaf(dd[f], oo[f], D);
          mdo = fmaxf(mdo, fabsf(dd[f]));
        }
        Dc[rc * nqq + qq] = D;
      }
      __syncthreads();
      for (int qq = t; qq < nqq; qq += blockDim.x) {   // fixed copy order
        float D = Cd_l[q0 + qq];
        for (int rc = 0; rc < ng; ++rc) D += Dc[rc * nqq + qq];
        Cd_l[q0 + qq] = D;
      }
    }
  }
  __syncthreads();
  for (int q = t; q < nq; q += blockDim.x) md = fmaxf(md, fabsf(Cd_l[q]));

  // resident K operands, K^T image, max |v| (as attn_bwd_sf16_kernel)
  u4 Kop[BKT], Vop[BKT];
  const float* kg = a.k + (int64_t)b * a.k_bs + h * 8;
  const float* vg = a.v + (int64_t)b * a.v_bs + h * 8;
  const float* kbg = a.kbias ? a.kbias + (int64_t)b * a.kb_bs : nullptr;
  _Float16* KT_ = reinterpret_cast<_Float16*>(KTi + (w * BKT) * 256);
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    const int key = key0 + 16 * tt + c;
    const bool ok = key < a.Lk;
    const int64_t kc = min(key, a.Lk - 1);
    float kr[8];
    {
      const float4 k0 = *reinterpret_cast<const float4*>(kg + kc * a.k_ls);
      const float4 k1 = *reinterpret_cast<const float4*>(kg + kc * a.k_ls + 4);
      const float4 v0 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls);
      const float4 v1 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls + 4);
      const float kk[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        kr[f] = ok ? kk[f] : 0.f;
        mv = fmaxf(mv, ok ? fabsf(vv[f]) : 0.f);
      }
    }
    const float bias = ok ? (kbg ? kbg[key] : 0.f) : -INFINITY;
    u4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hi[j] = pk_hi(kr[2 * j], kr[2 * j + 1]);
      lo[j] = pk_lo(kr[2 * j], kr[2 * j + 1], hi[j]);
    }
    const u4 bs = {pack2(f16_hi(bias), f16_lo(bias)), 0u, 0u, 0u};
    Kop[tt] = g == 3 ? bs : (g == 1 ? lo : hi);
    const int gs = c >> 2, jb = 4 * ((c & 3) >> 1) + (c & 1);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int f = 2 * g + e;
      const _Float16 kh = f16_hi(kr[f]), kl = f16_lo(kr[f]);
      _Float16* row = KT_ + tt * 512 + f * 32 + 8 * (gs ^ tsw(f)) + jb;
      row[0] = kh;
      row[2] = kh;
      row[8 * 32] = kl;
      row[8 * 32 + 2] = (_Float16)0.f;
    }
  }
  mdo = wave_max(mdo);
  md = wave_max(md);
  mv = wave_max(mv);
  if (l == 0) {
    Red[0][w] = mdo;
    Red[1][w] = md;
    Red[2][w] = mv;
  }
  __syncthreads();
  float Mdo = 0.f, Md = 0.f, Mv = 0.f;
  for (int i = 0; i < NW; ++i) {
    Mdo = fmaxf(Mdo, Red[0][i]);
    Md = fmaxf(Md, Red[1][i]);
    Mv = fmaxf(Mv, Red[2][i]);
  }
  const float sd = DROP ? a.inv_keep : 1.f;
  const float bnd = (float)R * 8.f * Mdo * sd * Mv + Md;     // >= |sum_c keep_c sd dP_c - sum_c D_c|
  int s = 0;
  if (bnd > 0.f && isfinite(bnd)) {
    int e;
    frexpf(bnd, &e);
    s = max(-100, min(100, 1 - e));                          // 2^s bnd < 2
  }
  // the f16 operands dO'' = sd dO 2^ea and v'' = v 2^eb sit at a maximum of [2^6, 2^7) each,
  // so their lo parts stay normal f16 (2^s of the R-copy bound alone would push them into the
  // subnormals); dP'' = dO'' v''^T is brought to the dS scale 2^s by one multiply (fm)
  int ea = 0, eb = 0;
  if (Mdo * sd > 0.f && isfinite(Mdo * sd)) {
    frexpf(Mdo * sd, &ea);
    ea = max(-100, min(100, 7 - ea));
  }
  if (Mv > 0.f && isfinite(Mv)) {
    frexpf(Mv, &eb);
    eb = max(-100, min(100, 7 - eb));
  }
  const float fdo = ldexpf(sd, ea), fv = ldexpf(1.f, eb), fd = ldexpf(1.f, s);
  const float fm = ldexpf(1.f, s - ea - eb);
  for (int q = t; q < 16 * nqt; q += blockDim.x) Cd_l[q] = q < nq ? Cd_l[q] * -fd : 0.f;
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    const int key = key0 + 16 * tt + c;
    const bool ok = key < a.Lk;
    const int64_t kc = min(key, a.Lk - 1);
    const float4 v0 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls);
    const float4 v1 = *reinterpret_cast<const float4*>(vg + kc * a.v_ls + 4);
    const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    float vr[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) vr[f] = ok ? vv[f] * fv : 0.f;
    u4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hi[j] = pk_hi(vr[2 * j], vr[2 * j + 1]);
      lo[j] = pk_lo(vr[2 * j], vr[2 * j + 1], hi[j]);
    }
    Vop[tt] = g == 3 ? (u4){0u, 0u, 0u, 0u} : (g == 1 ? lo : hi);
  }
  f4 dV[BKT], dK[BKT];
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    dV[tt] = splat(0.f);
    dK[tt] = splat(0.f);
  }

  // ---- query tiles x copy groups ----
  // staging: threads 0..31 the Q tile (query t >> 1, features 4 (t & 1)..), every thread one
  // (copy, query, feature half) of the group's dO
  const int ngrp = (R + RB_RG - 1) / RB_RG;
  const int sq_i = (t >> 1) & 15, shf = t & 1, src = t >> 5;
  float4 rQ = make_float4(0.f, 0.f, 0.f, 0.f), rD = rQ;
  // this wave's keep words of step (it, gi) straight into its own LDS region (LDS-DMA: no
  // registers; a wave reads only its own region, so it may refill it once its copy loops are
  // done): 4 loads of 1 KB, lane l of load j = copy 4j + l / 16, key group (l / 4) % 4, queries
  // 4 (l % 4) .. + 3 of the tile
  auto keep_dma = [&](int it, int gi) {
    if (!DROP || ntile == 0) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int rc = 4 * j + (l >> 4), G = (l >> 2) & 3, r = gi * RB_RG + rc;
      if (r < R) {
        const int64_t nh = seq(r) * a.H + h;
        const uint32_t* src = a.bits + ((nh * NT8 + w) * 4 + G) * Lqp + qbeg + 16 * it + 4 * (l & 3);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(Kw + (w * RB_RG * 64 + j * 256)),
                                         16, 0, 0);
      }
    }
  };
  auto issue = [&](int it, int gi) {
    const int q = qbeg + 16 * it + sq_i;
    if (t < 32 && gi == 0)
      rQ = q < qend ? *reinterpret_cast<const float4*>(qg + (int64_t)q * a.q_ls + 4 * shf)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    const int r = gi * RB_RG + src;
    rD = (src < RB_RG && r < R && q < qend) ? *reinterpret_cast<const float4*>(dorow(r, q) + 4 * shf)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto commit = [&](int gi) {
    if (t < 32 && gi == 0) {   // Q: A operand [hi | lo | ones] and the transposed A operand
      const float m_ = a.scale_log2;
      const float x[4] = {rQ.x * m_, rQ.y * m_, rQ.z * m_, rQ.w * m_};
      uint32_t* A_ = Qa + sq_i * 12;
      const uint32_t h0 = pk_hi(x[0], x[1]), h1 = pk_hi(x[2], x[3]);
      *reinterpret_cast<uint2*>(A_ + 2 * shf) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(A_ + 4 + 2 * shf) = make_uint2(pk_lo(x[0], x[1], h0), pk_lo(x[2], x[3], h1));
      *reinterpret_cast<uint2*>(A_ + 8 + 2 * shf) = make_uint2(shf == 0 ? ONES_F16X2 : 0u, 0u);
      _Float16* T_ = reinterpret_cast<_Float16*>(QT);
      const int gs = sq_i >> 2, j0 = sq_i & 3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int f = 4 * shf + e;
        const _Float16 xh = f16_hi(x[e]), xl = f16_lo(x[e]);
        _Float16* row = T_ + f * 32 + 8 * (gs ^ tsw(f)) + j0;
        row[0] = xh;
        row[4] = xh;
        row[8 * 32] = xl;
        row[8 * 32 + 4] = (_Float16)0.f;
      }
    }
    if (src < RB_RG) {   // dO'_c: A operand [hi | lo | 0] (the dP' product) and the dO'^T image
      const float x[4] = {rD.x * fdo, rD.y * fdo, rD.z * fdo, rD.w * fdo};
      uint32_t* A_ = Ca + (src * 16 + sq_i) * 12;
      const uint32_t h0 = pk_hi(x[0], x[1]), h1 = pk_hi(x[2], x[3]);
      *reinterpret_cast<uint2*>(A_ + 2 * shf) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(A_ + 4 + 2 * shf) = make_uint2(pk_lo(x[0], x[1], h0), pk_lo(x[2], x[3], h1));
      *reinterpret_cast<uint2*>(A_ + 8 + 2 * shf) = make_uint2(0u, 0u);
      {   // the transposed A operand, rows f / f + 8, as the Q^T image
        _Float16* T_ = reinterpret_cast<_Float16*>(Ct + src * 256);
        const int gs = sq_i >> 2, j0 = sq_i & 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int f = 4 * shf + e;
          const _Float16 xh = f16_hi(x[e]), xl = f16_lo(x[e]);
          _Float16* row = T_ + f * 32 + 8 * (gs ^ tsw(f)) + j0;
          row[0] = xh;
          row[4] = xh;
          row[8 * 32] = xl;
          row[8 * 32 + 4] = (_Float16)0.f;
        }
      }
    }
  };
  // keep words of staged copy rc for this lane: 4 queries (q0 + 4g + i), key group c / 4, the
  // wave's 128 keys
  auto words = [&](int rc) -> u4 { return ldu4(Kw + ((w * RB_RG + rc) * 4 + (c >> 2)) * 16 + 4 * g); };
  const float uq = ldexpf(a.scale, -14 - s);
  float* dqb = a.dq + (int64_t)b * a.dq_bs + h * 8;
  auto dq_reduce = [&](int q0, int buf) {
    for (int i0 = t; i0 < 128; i0 += blockDim.x) {
      const int qq = i0 >> 3, f = i0 & 7;
      float acc = 0.f;
      for (int i = 0; i < NW; ++i) acc += Qp[buf * NW * 128 + i * 128 + qq * 8 + f];
      if (q0 + qq < qend) dqb[(int64_t)(q0 + qq) * a.dq_ls + f] = acc * uq;
    }
  };

  const int nsteps = nqt * ngrp;
  keep_dma(0, 0);
  issue(0, 0);
  __syncthreads();      // the prologue's scratch (Ca) is free
  commit(0);
  __syncthreads();
  f4 dQa = splat(0.f);
  int pend = -1;        // query tile whose dQ partials await the reduction (buffer pend & 1)
  for (int st = 0; st < nsteps; ++st) {
    const int it = st / ngrp, gi = st - it * ngrp;
    const int q0 = qbeg + 16 * it, ql = 16 * it, buf = it & 1;
    const int rg0 = gi * RB_RG, ng = min(RB_RG, R - rg0);
    if (gi == 0 && pend >= 0) {
      dq_reduce(qbeg + 16 * pend, pend & 1);
      pend = -1;
    }
    if (gi == 0) dQa = splat(0.f);
    // the next step's staging loads go out after the copy loops (fewer live registers there)
    bool issued = false;
    if (ntile > 0) {
      const int dtoff = g == 2 ? 4 : (g == 3 ? 8 : 0);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (4 * hh >= ntile) break;
        f4 acc[4];
        u4 Pw[4];     // p' as hi / lo pair words [hi(0,1) | hi(2,3) | lo(0,1) | lo(2,3)]
        const u4 QA = ldu4(Qa + c * 12 + dtoff);
        const f4 CS = *reinterpret_cast<const f4*>(Cs_l + ql + 4 * g);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f4 S = mma(QA, Kop[4 * hh + u], CS);
          float P[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) P[r] = ex2(S[r]);
          Pw[u][0] = pk_hi(P[0], P[1]);
          Pw[u][1] = pk_hi(P[2], P[3]);
          Pw[u][2] = pk_lo1(P[0], P[1], Pw[u][0], one);
          Pw[u][3] = pk_lo1(P[2], P[3], Pw[u][1], one);
          acc[u] = splat(0.f);
        }
        if (DROP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's keep-word DMA
        for (int rc = 0; rc < ng; ++rc) {
          const u4 kw = words(rc);
          const u4 DA = ldu4(Ca + (rc * 16 + c) * 12 + dtoff);
          const u4 DT = ldu4(Ct + rc * 256 + c * 16 + 4 * (g ^ tsw(c)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int tt = 4 * hh + u;
            const f4 x = mma(DA, Vop[tt], acc[u]);     // acc + dP''_c
            // keep masks per query; the pair words' halves masked per query: (q0, q1), (q2, q3)
            u4 Bv;
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
              uint32_t mk[2];
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                const int r = 2 * r2 + i;
                mk[i] = DROP ? (uint32_t)__builtin_amdgcn_sbfe((int)kw[r], 4 * tt + (c & 3), 1) : ~0u;
                acc[u][r] = __uint_as_float((as_u(x[r]) & mk[i]) | (as_u(acc[u][r]) & ~mk[i]));
              }
              const uint32_t mm = (mk[0] & 0xFFFFu) | (mk[1] & 0xFFFF0000u);
              Bv[r2] = Pw[u][r2] & mm;
              Bv[2 + r2] = Pw[u][2 + r2] & mm;
            }
            dV[tt] = mma(DT, Bv, dV[tt]);
          }
        }
        if (!issued && (hh == 1 || 4 >= ntile) && st + 1 < nsteps) {
          keep_dma((st + 1) / ngrp, (st + 1) % ngrp);
          issue((st + 1) / ngrp, (st + 1) % ngrp);
          issued = true;
        }
        const u4 QTA = ldu4(QT + c * 16 + 4 * (g ^ tsw(c)));
        const f4 CD = gi == 0 ? *reinterpret_cast<const f4*>(Cd_l + ql + 4 * g) : splat(0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int tt = 4 * hh + u;
          float dS[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // p' = hi + lo again, each half converted on its own (hipcc 7.2 miscompiled the
            // vector conversion of a u4 element here, converting element 0's word for all r)
            const uint32_t wh = Pw[u][r >> 1], wl = Pw[u][2 + (r >> 1)];
            const int sh = 16 * (r & 1);
            const float ph = (float)__builtin_bit_cast(_Float16, (uint16_t)((wh >> sh) & 0xffffu));
            const float pl = (float)__builtin_bit_cast(_Float16, (uint16_t)((wl >> sh) & 0xffffu));
            dS[r] = (ph + pl) * fmaf(acc[u][r], fm, CD[r]);
          }
          u4 Bk;
          Bk[0] = pk_hi(dS[0], dS[1]);
          Bk[1] = pk_hi(dS[2], dS[3]);
          Bk[2] = pk_lo1(dS[0], dS[1], Bk[0], one);
          Bk[3] = pk_lo1(dS[2], dS[3], Bk[1], one);
          dK[tt] = mma(QTA, Bk, dK[tt]);
          uint32_t* sc = Sc + w * SC_WORDS;
          const int Rw = 4 * (c >> 1) + (c & 1);
          *reinterpret_cast<uint2*>(sc + sc_at(Rw, g)) = make_uint2(Bk[0], Bk[1]);
          *reinterpret_cast<uint2*>(sc + sc_at(Rw + 2, g)) = make_uint2(Bk[2], Bk[3]);
          const int rq = (c >> 2), cp = (c & 3);
          const s4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(sc + sc_at(8 * g + rq, cp)));
          const s4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(sc + sc_at(8 * g + 4 + rq, cp)));
          const u4 Bq = {__builtin_bit_cast(uint2, x0).x, __builtin_bit_cast(uint2, x0).y,
                         __builtin_bit_cast(uint2, x1).x, __builtin_bit_cast(uint2, x1).y};
          const u4 KA = ldu4(KTi + (w * BKT + tt) * 256 + c * 16 + 4 * (g ^ tsw(c)));
          dQa = mma(KA, Bq, dQa);
        }
      }
    }
    if (!issued && st + 1 < nsteps) issue((st + 1) / ngrp, (st + 1) % ngrp);
    if (gi == ngrp - 1) {   // this wave's dQ partial of the tile: rows f + rows f + 8
      f4 dq;
#pragma unroll
      for (int r = 0; r < 4; ++r) dq[r] = xsum32(dQa[r]);
      if (g < 2) *reinterpret_cast<f4*>(Qp + buf * NW * 128 + w * 128 + c * 8 + 4 * g) = dq;
      pend = it;
    }
    __syncthreads();
    if (st + 1 < nsteps) {
      commit((st + 1) % ngrp);
      __syncthreads();
    }
  }
  if (pend >= 0) dq_reduce(qbeg + 16 * pend, pend & 1);
  // dK, dV partials of this query chunk: rows f + rows f + 8
  const float uk = ldexpf(a.scale / a.scale_log2, -14 - s), uvs = ldexpf(1.f, -14 - ea);
  float* dkb = a.dk + (int64_t)qs * a.dk_ss + (int64_t)b * a.dk_bs + h * 8;
  float* dvb = a.dv + (int64_t)qs * a.dk_ss + (int64_t)b * a.dv_bs + h * 8;
#pragma unroll
  for (int tt = 0; tt < BKT; ++tt) {
    if (tt < ntile) {
      f4 v, k_;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = xsum32(dV[tt][r]) * uvs;
        k_[r] = xsum32(dK[tt][r]) * uk;
      }
      const int key = key0 + 16 * tt + c;
      if (g < 2 && key < a.Lk) {
        *reinterpret_cast<float4*>(dvb + (int64_t)key * a.dv_ls + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(dkb + (int64_t)key * a.dk_ls + 4 * g) = make_float4(k_[0], k_[1], k_[2], k_[3]);
      }
    }
  }
}

// out[b, q, h*8 + f] = sum over the nkb key blocks' partials (fixed order)
__global__ void sf16_dq_sum_kernel(const float* __restrict__ ws, int64_t ss, int n, int B, int Lq,
                                   int E, float* __restrict__ dq, int64_t bs, int64_t ls) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * Lq * E) return;
  const int e = (int)(t % E);
  const int64_t bl = t / E;
  const int q = (int)(bl % Lq), b = (int)(bl / Lq);
  float v = 0.f;
  for (int i = 0; i < n; ++i) v += ws[i * ss + t];
  dq[(int64_t)b * bs + (int64_t)q * ls + e] = v;
}

int fwd_waves(int Lq) { return Lq <= 64 ? 1 : (Lq <= 128 ? 2 : 4); }
// waves of a repeated-sequence forward workgroup (one query tile per wave)
int rep_fwd_waves(int Lq) { return Lq <= 16 ? 1 : (Lq <= 32 ? 2 : 4); }
// waves (128 keys each) per backward workgroup: the whole key axis in one workgroup of up
// to 8 waves, unless (sequence, head) pairs are too few to give every CU a workgroup -- small
// batches (B = 2: 128 decoder pairs) and the encoders' context attention (64 pairs) -- then
// halved (down to 2) until they do, the key blocks' dQ partials summed after the launch
int bwd_waves(int Lk, int64_t bh) {
  int nw = std::min(BNW_MAX, (Lk + 127) / 128);
  while (nw > 2 && bh * ((Lk + 128 * nw - 1) / (128 * nw)) < 256) nw = (nw + 1) / 2;
  return nw;
}
int bwd_blocks(int Lk, int64_t bh) {
  const int nw = bwd_waves(Lk, bh);
  return (Lk + 128 * nw - 1) / (128 * nw);
}
int lq_pad(int Lq) { return (Lq + 15) & ~15; }
// query chunks of a backward launch: while the workgroups' waves would leave SIMDs empty
// (fewer than 2 per SIMD: 2048), the query axis is cut into chunks of >= 64 queries, each
// chunk's dK / dV a partial summed after the launch (the encoders' context attention, 64
// pairs; small batches).  Returns the chunk length (0: one chunk)
int bwd_qchunk(int Lq, int Lk, int64_t bh) {
  const int64_t waves = bh * bwd_blocks(Lk, bh) * bwd_waves(Lk, bh);
  const int tiles = (Lq + 15) / 16;
  int nqc = (int)std::min<int64_t>((2048 + waves - 1) / waves, tiles / 4);
  if (nqc <= 1) return 0;
  return (tiles + nqc - 1) / nqc * 16;
}
size_t bwd_lds_bytes(int nw) {
  return (size_t)nw * (BKT * 256 + 2 * SC_WORDS + 2 * 128) * sizeof(uint32_t);
}
int nt8(int Lk) { return (Lk + 127) / 128; }

// repeated-sequence kernels' configuration: copies per forward workgroup (0: by R), backward
// workgroups targeted (query chunks = target / (Bd H)); vaesne_attn_rep_sf16_config (tests, A/B)
struct RepSf16Cfg { int frc, bwgs; };
const RepSf16Cfg kRepSf16Default{0, 256};
RepSf16Cfg g_rs = kRepSf16Default;
int rep_fwd_rc(int R) {
  if (g_rs.frc > 0) return g_rs.frc;
  return R <= 4 ? 4 : (R <= 8 ? 8 : 16);
}
struct RepBwdPlan { int QS, qchunk; };
RepBwdPlan rep_bwd_plan_sf16(int Bd, int H, int L) {
  const int tiles = (L + 15) / 16;
  const int64_t bh = (int64_t)Bd * H;
  int qs = (int)std::max<int64_t>(1, (g_rs.bwgs + bh / 2) / bh);
  qs = std::min(qs, tiles);
  qs = std::max(qs, (tiles + RB_QCH_MAX / 16 - 1) / (RB_QCH_MAX / 16));   // chunk <= RB_QCH_MAX
  RepBwdPlan pl;
  pl.qchunk = (tiles + qs - 1) / qs * 16;
  pl.QS = (L + pl.qchunk - 1) / pl.qchunk;
  return pl;
}

template <int NQT, int RC, bool DROP>
void launch_fwd_k(const AttnArgs& a, int R, int nw, int qb0, int nqbs, int cy, hipStream_t s) {
  const dim3 grid((unsigned)((int64_t)a.B * a.H * nqbs), (unsigned)cy);
  hipLaunchKernelGGL((attn_fwd_sf16_kernel<NQT, RC, DROP>), grid, dim3(64 * nw), 0, s, a, nt8(a.Lk),
                     lq_pad(a.Lq), R, qb0, nqbs);
}

}  // namespace

bool sf16_path(int dh, int64_t bh, int Lq, int Lk) {
  return dh == 8 && bh > 0 && Lq > 16 && Lq <= BLQ_MAX && Lk >= 1;
}
bool sf16_rep_path(int L, int R) { return L > 16 && L <= RB_LMAX && R >= 1; }

int64_t sf16_bits_bytes(int B, int H, int Lq, int Lk) {
  return (int64_t)B * H * nt8(Lk) * 4 * lq_pad(Lq) * (int64_t)sizeof(uint32_t);
}

int64_t sf16_bwd_ws_floats(int B, int H, int Lq, int Lk) {
  const int64_t bh = (int64_t)B * H;
  const int nkb = bwd_blocks(Lk, bh), qch = bwd_qchunk(Lq, Lk, bh);
  const int nqc = qch > 0 ? (Lq + qch - 1) / qch : 1;
  return (nkb > 1 ? (int64_t)nkb * B * Lq * H * 8 : 0) +
         (nqc > 1 ? 2 * (int64_t)nqc * B * Lk * H * 8 : 0);
}

int64_t sf16_rep_bwd_ws_floats(int Bd, int H, int L) {
  const RepBwdPlan pl = rep_bwd_plan_sf16(Bd, H, L);
  return pl.QS > 1 ? 2 * (int64_t)pl.QS * Bd * L * H * 8 : 0;
}

int sf16_fwd(const AttnArgs& a, float p_drop, hipStream_t s) {
  const int nw = fwd_waves(a.Lq);
  const int nqb = (a.Lq + 64 * nw - 1) / (64 * nw);
  if (p_drop > 0.f) launch_fwd_k<4, 1, true>(a, 1, nw, 0, nqb, 1, s);
  else launch_fwd_k<4, 1, false>(a, 1, nw, 0, nqb, 1, s);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

// R copies of a.B distinct sequences (o, bits over the R a.B copy sequences); query blocks
// [p0 nqb / np, p1 nqb / np) of the launch geometry
int sf16_rep_fwd(const AttnArgs& a, int R, float p_drop, int p0, int p1, int np, hipStream_t s) {
  if (p_drop > 0.f) {
    const int nw = rep_fwd_waves(a.Lq), rc = rep_fwd_rc(R);
    const int nqb = (a.Lq + 16 * nw - 1) / (16 * nw);
    const int qb0 = (int)((int64_t)p0 * nqb / np), qb1 = (int)((int64_t)p1 * nqb / np);
    if (qb1 <= qb0) return 0;
    const int cy = (R + rc - 1) / rc;
    if (rc == 4) launch_fwd_k<1, 4, true>(a, R, nw, qb0, qb1 - qb0, cy, s);
    else if (rc == 8) launch_fwd_k<1, 8, true>(a, R, nw, qb0, qb1 - qb0, cy, s);
    else launch_fwd_k<1, 16, true>(a, R, nw, qb0, qb1 - qb0, cy, s);
  } else {   // every copy the same: the plain kernel, its output stored to all R
    const int nw = fwd_waves(a.Lq);
    const int nqb = (a.Lq + 64 * nw - 1) / (64 * nw);
    const int qb0 = (int)((int64_t)p0 * nqb / np), qb1 = (int)((int64_t)p1 * nqb / np);
    if (qb1 <= qb0) return 0;
    launch_fwd_k<4, 1, false>(a, R, nw, qb0, qb1 - qb0, 1, s);
  }
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int sf16_bwd(const AttnArgs& a, float p_drop, float* ws, hipStream_t s) {
  const int64_t bh = (int64_t)a.B * a.H;
  const int nw = bwd_waves(a.Lk, bh), nkb = bwd_blocks(a.Lk, bh);
  const int E = a.H * 8;
  const int qch = bwd_qchunk(a.Lq, a.Lk, bh), nqc = qch > 0 ? (a.Lq + qch - 1) / qch : 1;
  AttnArgs c = a;
  c.qchunk = qch;
  c.dk_ss = 0;
  float* wsk = ws;
  if (nkb > 1) {
    if (!ws) return (int)hipErrorInvalidValue;
    c.dq = ws;
    c.dq_bs = (int64_t)a.Lq * E;
    c.dq_ls = E;
    c.dq_ss = (int64_t)a.B * a.Lq * E;
    wsk = ws + (int64_t)nkb * c.dq_ss;
  }
  if (nqc > 1) {   // dK / dV partials per query chunk: [nqc][B][Lk][E] each
    if (!ws) return (int)hipErrorInvalidValue;
    c.dk_ss = (int64_t)a.B * a.Lk * E;
    c.dk = wsk; c.dk_bs = (int64_t)a.Lk * E; c.dk_ls = E;
    c.dv = wsk + (int64_t)nqc * c.dk_ss; c.dv_bs = c.dk_bs; c.dv_ls = E;
  }
  const dim3 grid((unsigned)(bh * nkb), (unsigned)nqc);
  static const bool lds_ok = [] {     // dynamic LDS beyond 64 KB (8 waves: 95 KB)
    const int mx = (int)bwd_lds_bytes(BNW_MAX);
    return hipFuncSetAttribute((const void*)attn_bwd_sf16_kernel<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, mx) == hipSuccess &&
           hipFuncSetAttribute((const void*)attn_bwd_sf16_kernel<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, mx) == hipSuccess;
  }();
  if (!lds_ok) return (int)hipErrorInvalidConfiguration;
  if (p_drop > 0.f)
    hipLaunchKernelGGL(attn_bwd_sf16_kernel<true>, grid, dim3(64 * nw), bwd_lds_bytes(nw), s, c, nkb,
                       nt8(a.Lk), lq_pad(a.Lq));
  else
    hipLaunchKernelGGL(attn_bwd_sf16_kernel<false>, grid, dim3(64 * nw), bwd_lds_bytes(nw), s, c, nkb,
                       nt8(a.Lk), lq_pad(a.Lq));
  VAESNE_CHECK_LAUNCH();
  if (nkb > 1) {
    const int64_t n = (int64_t)a.B * a.Lq * E;
    hipLaunchKernelGGL(sf16_dq_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ws,
                       c.dq_ss, nkb, a.B, a.Lq, E, a.dq, a.dq_bs, a.dq_ls);
    VAESNE_CHECK_LAUNCH();
  }
  if (nqc > 1) {
    const int64_t n = (int64_t)a.B * a.Lk * E;
    const dim3 sg((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(sf16_dq_sum_kernel, sg, dim3(256), 0, s, c.dk, c.dk_ss, nqc, a.B, a.Lk, E,
                       a.dk, a.dk_bs, a.dk_ls);
    VAESNE_CHECK_LAUNCH();
    hipLaunchKernelGGL(sf16_dq_sum_kernel, sg, dim3(256), 0, s, c.dv, c.dk_ss, nqc, a.B, a.Lk, E,
                       a.dv, a.dv_bs, a.dv_ls);
    VAESNE_CHECK_LAUNCH();
  }
  return 0;
}

// dropout only (without it every copy is the same: the plain backward of sum_r dO_r)
int sf16_rep_bwd(const AttnArgs& a, int R, float* ws, hipStream_t s) {
  const RepBwdPlan pl = rep_bwd_plan_sf16(a.B, a.H, a.Lq);
  const int E = a.H * 8;
  AttnArgs c = a;
  c.qchunk = pl.qchunk;
  c.dk_ss = 0;
  if (pl.QS > 1) {
    if (!ws) return (int)hipErrorInvalidValue;
    c.dk = ws; c.dk_bs = (int64_t)a.Lk * E; c.dk_ls = E;
    c.dv = ws + (int64_t)pl.QS * a.B * a.Lk * E; c.dv_bs = c.dk_bs; c.dv_ls = E;
    c.dk_ss = (int64_t)a.B * a.Lk * E;
  }
  static const bool lds_ok = hipFuncSetAttribute((const void*)attn_rep_bwd_sf16_kernel<true>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)rep_bwd_lds_bytes(RB_NW_MAX)) == hipSuccess;
  if (!lds_ok) return (int)hipErrorInvalidConfiguration;
  const dim3 grid((unsigned)((int64_t)a.B * a.H * pl.QS));
  hipLaunchKernelGGL(attn_rep_bwd_sf16_kernel<true>, grid, dim3(64 * RB_NW_MAX), rep_bwd_lds_bytes(RB_NW_MAX),
                     s, c, R, pl.QS, nt8(a.Lk), lq_pad(a.Lq));
  VAESNE_CHECK_LAUNCH();
  if (pl.QS > 1) {
    const int64_t n = (int64_t)a.B * a.Lk * E;
    const dim3 sg((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(sf16_dq_sum_kernel, sg, dim3(256), 0, s, c.dk, c.dk_ss, pl.QS, a.B, a.Lk, E,
                       a.dk, a.dk_bs, a.dk_ls);
    VAESNE_CHECK_LAUNCH();
    hipLaunchKernelGGL(sf16_dq_sum_kernel, sg, dim3(256), 0, s, c.dv, c.dk_ss, pl.QS, a.B, a.Lk, E,
                       a.dv, a.dv_bs, a.dv_ls);
    VAESNE_CHECK_LAUNCH();
  }
  return 0;
}

int sf16_rep_config(int frc, int bwgs) {
  if (frc < 0) { g_rs = kRepSf16Default; return 0; }
  if ((frc != 0 && frc != 4 && frc != 8 && frc != 16) || bwgs <= 0) return (int)hipErrorInvalidValue;
  g_rs = {frc, bwgs};
  return 0;
}

}  // namespace vaesne
