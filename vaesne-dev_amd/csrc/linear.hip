// Token-wise linear layers (nn.Linear on [*, K] -> [*, N]) for the VAESNe
// transformer stacks: in-projections (32->96), out-projections and FFN
// (32->32), the MLP heads (32->32->1 / Dz) and the embedding MLPs (64->32,
// 96->32).  Reference: torch.nn.Linear as used throughout
// package/VAESNe/util_layers.py:9-34,131-149,257-309.
//
// Forward / backward-data kernel (one kernel, two weight orientations):
//   out[r, n] = (accum ? out[r, n] : 0) + bias[n] + sum_k in[r, k] * Wt[n, k]
//   in[r, k]  = (a[r, k] + a2[r, k]) * (act_in_grad ? act'(zin[r, k]) : 1)
//   optional activation on the way out (relu / exact-erf gelu), pre-activation
//   optionally stored for the backward.
// Geometry: MFMA v_mfma_f32_32x32x2_f32 (exact f32) in the feature layout of
// decoder_block.hip: a wave owns 32 rows (lane = row, 16 features per lane and
// 32-block as 4 float4s), y^T = W x^T is 16 MFMAs per 32x32 block with the
// weight in LDS (staged once per workgroup, odd row stride).
//
// Backward-weight kernel: dW[o, i] = sum_r dz[r, o] x[r, i], db[o] = sum_r dz[r, o]
// with dz = dy * act'(z) recomputed on the fly, as MFMAs contracting over rows
// (both operands coalesced row segments); per-workgroup partial sums in a
// workspace, then a fixed-order reduction (bitwise reproducible).
#include "common.h"

using namespace vaesne;

namespace {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

struct LinArgs {
  const float* a; int64_t lda;
  const float* a2; int64_t lda2;
  const float* zin; int64_t ldzin; int act_in_grad;
  const float* W; int w_trans; const float* bias;
  int K; int N; int64_t M;
  float* out; int64_t ldo; int accum; int act_out;
  float* zout; int64_t ldzo;
};

__device__ __forceinline__ float act_fwd(int act, float v) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_GELU) return gelu_erf(v);
  return v;
}
__device__ __forceinline__ float act_grad(int act, float z) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_GELU) return gelu_erf_grad(z);
  return 1.f;
}

constexpr int NT = 256;
constexpr int MAXK = 128;
constexpr int MAXN = 128;
constexpr int MAXB = MAXK / 32;   // 32-feature blocks

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// feature layout of v_mfma_f32_32x32x2_f32 (as decoder_block.hip): lane l holds
// row t = l & 31 and, per 32-feature block, features F(s, h), h = l >> 5
__device__ __forceinline__ int F(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// x[s] = (a + a2)[row][kb*32 + F(s,h)] * (act_in_grad ? act'(zin) : 1), 0 past K
template <bool VIN>
__device__ __forceinline__ void load_feat(const LinArgs& p, int64_t row, int kb, int h,
                                          float (&x)[16]) {
  const float* ar = p.a + row * p.lda;
  const float* a2r = p.a2 ? p.a2 + row * p.lda2 : nullptr;
  const float* zr = p.act_in_grad ? p.zin + row * p.ldzin : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k0 = kb * 32 + 8 * j + 4 * h;
    if (VIN) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k0 < p.K) {
        v = *reinterpret_cast<const float4*>(ar + k0);
        if (a2r) {
          const float4 w = *reinterpret_cast<const float4*>(a2r + k0);
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
        if (zr) {
          const float4 z = *reinterpret_cast<const float4*>(zr + k0);
          v.x *= act_grad(p.act_in_grad, z.x); v.y *= act_grad(p.act_in_grad, z.y);
          v.z *= act_grad(p.act_in_grad, z.z); v.w *= act_grad(p.act_in_grad, z.w);
        }
      }
      x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + i;
        float v = 0.f;
        if (k < p.K) {
          v = ar[k];
          if (a2r) v += a2r[k];
          if (zr) v *= act_grad(p.act_in_grad, zr[k]);
        }
        x[4 * j + i] = v;
      }
    }
  }
}

// out[row][nb*32 + F(i,h)] = act((accum ? out : 0) + acc[i]), pre-activation to zout
template <bool VOUT>
__device__ __forceinline__ void store_feat(const LinArgs& p, int64_t row, int nb, int h,
                                           const f16v& acc) {
  float* orow = p.out + row * p.ldo;
  float* zrow = p.zout ? p.zout + row * p.ldzo : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n0 = nb * 32 + 8 * j + 4 * h;
    if (VOUT) {
      if (n0 < p.N) {
        float4 v = make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
        if (p.accum) {
          const float4 o = *reinterpret_cast<const float4*>(orow + n0);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        if (zrow) *reinterpret_cast<float4*>(zrow + n0) = v;
        v.x = act_fwd(p.act_out, v.x); v.y = act_fwd(p.act_out, v.y);
        v.z = act_fwd(p.act_out, v.z); v.w = act_fwd(p.act_out, v.w);
        *reinterpret_cast<float4*>(orow + n0) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + i;
        if (n < p.N) {
          float v = acc[4 * j + i];
          if (p.accum) v += orow[n];
          if (zrow) zrow[n] = v;
          orow[n] = act_fwd(p.act_out, v);
        }
      }
    }
  }
}

// y^T = W x^T on v_mfma_f32_32x32x2_f32: a wave owns 32 rows; A = W from LDS
// (row n = lane & 31, k = F(s, h)), B = the row's own features: 16 MFMAs per
// 32x32 block, output straight in the feature layout (no shuffles).  The
// weight (zero padded to kbn x nbn blocks of 32) is staged once per workgroup.
template <bool VIN, bool VOUT>
__device__ __forceinline__ void linear_body(const LinArgs& p, int kbn, int nbn) {
  extern __shared__ float smem[];
  const int LDW = kbn * 32 + 1;             // odd row stride: conflict-free A reads
  float* Ws = smem;                         // [nbn*32][LDW]: Ws[n][k] = W(n, k)
  float* bs = smem + nbn * 32 * LDW;        // [nbn*32]
  // 8 loads in flight per thread before their LDS stores (the one-element loop waited on
  // each L2 round trip in turn at the start of every launch)
  const int wtotal = nbn * 32 * kbn * 32;
  for (int base = 0; base < wtotal; base += 8 * NT) {
    float w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      const int n = idx / (kbn * 32), k = idx - n * (kbn * 32);
      w[u] = 0.f;
      if (idx < wtotal && n < p.N && k < p.K)
        w[u] = p.w_trans ? p.W[(int64_t)k * p.N + n] : p.W[(int64_t)n * p.K + k];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      const int n = idx / (kbn * 32), k = idx - n * (kbn * 32);
      if (idx < wtotal) Ws[n * LDW + k] = w[u];
    }
  }
  for (int n = threadIdx.x; n < nbn * 32; n += NT) bs[n] = (p.bias && n < p.N) ? p.bias[n] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane & 31, h = lane >> 5;
  const int64_t tiles = (p.M + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * (NT / 64) + wave; tile < tiles;
       tile += (int64_t)gridDim.x * (NT / 64)) {
    const int64_t r = tile * 32 + t;
    const bool valid = r < p.M;
    const int64_t rr = valid ? r : p.M - 1;
    float x[MAXB][16];
#pragma unroll
    for (int kb = 0; kb < MAXB; ++kb)
      if (kb < kbn) load_feat<VIN>(p, rr, kb, h, x[kb]);
    for (int nb = 0; nb < nbn; ++nb) {
      f16v acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = bs[nb * 32 + F(i, h)];
      const float* wr = Ws + (nb * 32 + t) * LDW;
#pragma unroll
      for (int kb = 0; kb < MAXB; ++kb) {
        if (kb < kbn) {
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) acc = mfma(wr[kb * 32 + F(s2, h)], x[kb][s2], acc);
        }
      }
      if (valid) store_feat<VOUT>(p, r, nb, h, acc);
    }
  }
}

template <bool VIN, bool VOUT>
__global__ __launch_bounds__(NT) void linear_kernel(LinArgs p, int kbn, int nbn) {
  linear_body<VIN, VOUT>(p, kbn, nbn);
}

// up to LGMAX independent linears with the same (K, N) in one launch: blockIdx.z
// selects the group (the encoder blocks' context projections, G = 4)
constexpr int LGMAX = 8;
struct LinGroup {
  LinArgs p[LGMAX];
};
template <bool VIN, bool VOUT>
__global__ __launch_bounds__(NT) void linear_group_kernel(LinGroup g, int kbn, int nbn) {
  linear_body<VIN, VOUT>(g.p[blockIdx.z], kbn, nbn);
}

bool al16(const void* q, int64_t ld) { return ((uintptr_t)q % 16 == 0) && (ld % 4 == 0); }

// G == 0: one linear (p[0]); G >= 1: a grouped launch over p[0..G) (same K, N)
int launch_linear_n(const LinArgs* pp, int G, hipStream_t s) {
  const LinArgs& p = pp[0];
  if (p.K < 1 || p.K > MAXK || p.N < 1 || p.N > MAXN || G > LGMAX) return (int)hipErrorInvalidValue;
  int64_t Mmax = p.M;
  for (int g = 1; g < G; ++g) {
    if (pp[g].K != p.K || pp[g].N != p.N) return (int)hipErrorInvalidValue;
    Mmax = pp[g].M > Mmax ? pp[g].M : Mmax;
  }
  if (Mmax <= 0) return 0;
  const int kbn = (p.K + 31) / 32, nbn = (p.N + 31) / 32;
  const int64_t tiles = (Mmax + 31) / 32;
  const int64_t wg = (tiles + NT / 64 - 1) / (NT / 64);
  const int grid = (int)(wg < 2048 ? wg : 2048);
  const size_t shmem = sizeof(float) * ((size_t)nbn * 32 * (kbn * 32 + 1) + nbn * 32);
  bool vin = true, vout = true;
  for (int g = 0; g < (G ? G : 1); ++g) {
    const LinArgs& q = pp[g];
    vin = vin && (q.K % 4 == 0) && al16(q.a, q.lda) && (!q.a2 || al16(q.a2, q.lda2)) &&
          (!q.act_in_grad || al16(q.zin, q.ldzin));
    vout = vout && (q.N % 4 == 0) && al16(q.out, q.ldo) && (!q.zout || al16(q.zout, q.ldzo));
  }
  if (shmem > 65536) {   // > 64 KB of LDS (K, N up to 128): opt in once per instantiation
    static bool opted = false;
    if (!opted) {
      const void* fns[8] = {(const void*)linear_kernel<true, true>,
                            (const void*)linear_kernel<true, false>,
                            (const void*)linear_kernel<false, true>,
                            (const void*)linear_kernel<false, false>,
                            (const void*)linear_group_kernel<true, true>,
                            (const void*)linear_group_kernel<true, false>,
                            (const void*)linear_group_kernel<false, true>,
                            (const void*)linear_group_kernel<false, false>};
      for (const void* f : fns) {
        hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return (int)e;
      }
      opted = true;
    }
  }
  if (G == 0) {
    if (vin && vout)
      hipLaunchKernelGGL((linear_kernel<true, true>), dim3(grid), dim3(NT), shmem, s, p, kbn, nbn);
    else if (vin)
      hipLaunchKernelGGL((linear_kernel<true, false>), dim3(grid), dim3(NT), shmem, s, p, kbn, nbn);
    else if (vout)
      hipLaunchKernelGGL((linear_kernel<false, true>), dim3(grid), dim3(NT), shmem, s, p, kbn, nbn);
    else
      hipLaunchKernelGGL((linear_kernel<false, false>), dim3(grid), dim3(NT), shmem, s, p, kbn, nbn);
  } else {
    LinGroup lg{};
    for (int g = 0; g < G; ++g) lg.p[g] = pp[g];
    const dim3 gd(grid, 1, G);
    if (vin && vout)
      hipLaunchKernelGGL((linear_group_kernel<true, true>), gd, dim3(NT), shmem, s, lg, kbn, nbn);
    else if (vin)
      hipLaunchKernelGGL((linear_group_kernel<true, false>), gd, dim3(NT), shmem, s, lg, kbn, nbn);
    else if (vout)
      hipLaunchKernelGGL((linear_group_kernel<false, true>), gd, dim3(NT), shmem, s, lg, kbn, nbn);
    else
      hipLaunchKernelGGL((linear_group_kernel<false, false>), gd, dim3(NT), shmem, s, lg, kbn, nbn);
  }
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int launch_linear(const LinArgs& p, hipStream_t s) { return launch_linear_n(&p, 0, s); }

// ---------------------------------------------------------------------------
// backward weight
// ---------------------------------------------------------------------------
struct WgtArgs {
  const float* dy; int64_t lddy;
  const float* z; int64_t ldz; int act;  // dz = dy * act'(z)
  const float* x; int64_t ldx;
  const float* x2; int64_t ldx2;         // x := x + x2
  int64_t M; int O; int I;
  float* partial;                        // [gridDim.x][O*I + O]
};

// One workgroup per (row range, 32 x 32 block of dW).  dW^T is never formed:
// v_mfma_f32_32x32x2_f32 with A[o][kk] = dz[r + kk][o] and B[kk][i] = x[r + kk][i]
// (lane l: column l & 31 of row r + (l >> 5)) contracts over rows, so both
// operands are plain coalesced 128-byte row segments straight from HBM / L2.
// db rides along as the column sum of the dz values the o-block lanes load.
constexpr int WG_MAX = 256;

int64_t wgrad_groups(int64_t M) {
  const int64_t chunks = (M + 31) / 32;                 // 32 rows per wave iteration
  int64_t g = (chunks + NT / 64 - 1) / (NT / 64);
  if (g > WG_MAX) g = WG_MAX;
  return g < 1 ? 1 : g;
}

// ACT: activation whose derivative scales dy (0 none, 1 relu, 2 gelu); X2: x := x + x2.
// Loads are unconditional (rows / columns clamped) so all 16 x 2 of a chunk are
// in flight at once; out-of-range terms are zeroed afterwards.  With G == 1
// (gridDim.x) the workgroup writes dW / db directly (no column-sum pass).
template <int ACT, bool X2>
__device__ __forceinline__ void wgrad_body(const WgtArgs& p, int nib, float* dW, float* db,
                                           int accum) {
  __shared__ float red[NT / 64][1024 + 32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 31, hh = lane >> 5;
  const int ob = blockIdx.y / nib, ib = blockIdx.y - ob * nib;
  const int o = ob * 32 + col, i = ib * 32 + col;
  const bool oin = o < p.O, iin = i < p.I;
  const int oc = min(o, p.O - 1), ic = min(i, p.I - 1);
  f16v acc = {};
  float cs = 0.f;
  const int64_t chunks = (p.M + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * (NT / 64);
  // WD chunks' loads in flight per trip (a wave waited one HBM round trip per 32 rows); the
  // chunks still enter the accumulator in the one-chunk order, and a chunk past the end
  // (wave-uniform test) is neither loaded nor multiplied
  constexpr int WD = 4;
  for (int64_t ch = (int64_t)blockIdx.x * (NT / 64) + wave; ch < chunks; ch += WD * stride) {
    float gv[WD][16], zv[WD][16], xv[WD][16], x2v[WD][16];
#pragma unroll
    for (int c = 0; c < WD; ++c) {
      if (ch + c * stride < chunks) {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const int64_t r = min((ch + c * stride) * 32 + 2 * s2 + hh, p.M - 1);
          gv[c][s2] = p.dy[r * p.lddy + oc];
          if (ACT) zv[c][s2] = p.z[r * p.ldz + oc];
          xv[c][s2] = p.x[r * p.ldx + ic];
          if (X2) x2v[c][s2] = p.x2[r * p.ldx2 + ic];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < WD; ++c) {
      if (ch + c * stride < chunks) {
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const bool ok = (ch + c * stride) * 32 + 2 * s2 + hh < p.M;
          float gg = gv[c][s2], xx = xv[c][s2];
          if (ACT) gg *= act_grad(ACT, zv[c][s2]);
          if (X2) xx += x2v[c][s2];
          gg = (ok && oin) ? gg : 0.f;
          xx = (ok && iin) ? xx : 0.f;
          cs += gg;
          acc = mfma(gg, xx, acc);
        }
      }
    }
  }
  cs = xsum32(cs);
#pragma unroll
  for (int rg = 0; rg < 16; ++rg) red[wave][F(rg, hh) * 32 + col] = acc[rg];
  if (hh == 0) red[wave][1024 + col] = cs;
  __syncthreads();
  // partial layout [G][O*I (dW) | O (db)] so one column-sum splits at O*I
  const bool direct = gridDim.x == 1;
  float* out = p.partial + (int64_t)blockIdx.x * ((int64_t)p.O * p.I + p.O);
  for (int e = threadIdx.x; e < 1024 + 32; e += NT) {
    float v = red[0][e];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) v += red[w][e];
    if (e < 1024) {
      const int oo = ob * 32 + (e >> 5), ii = ib * 32 + (e & 31);
      if (oo < p.O && ii < p.I) {
        const int64_t f = (int64_t)oo * p.I + ii;
        if (!direct) out[f] = v;
        else if (dW) dW[f] = accum ? dW[f] + v : v;
      }
    } else if (ib == 0) {
      const int oo = ob * 32 + (e - 1024);
      if (oo < p.O) {
        if (!direct) out[(int64_t)p.O * p.I + oo] = v;
        else if (db) db[oo] = accum ? db[oo] + v : v;
      }
    }
  }
}

template <int ACT, bool X2>
__global__ __launch_bounds__(NT) void linear_wgrad_kernel(WgtArgs p, int nib, float* dW, float* db,
                                                          int accum) {
  wgrad_body<ACT, X2>(p, nib, dW, db, accum);
}

struct WgtGroup {
  WgtArgs p[LGMAX];
  float* dW[LGMAX];
  float* db[LGMAX];
};
template <int ACT, bool X2>
__global__ __launch_bounds__(NT) void linear_wgrad_group_kernel(WgtGroup g, int nib, int accum) {
  const int z = blockIdx.z;
  wgrad_body<ACT, X2>(g.p[z], nib, g.dW[z], g.db[z], accum);
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
VAESNE_API int vaesne_linear_fwd(const float* x, int64_t ldx, const float* x2, int64_t ldx2,
                                 int64_t M, int K, const float* W, const float* b, int N,
                                 float* y, int64_t ldy, float* z, int64_t ldz, int act,
                                 int accum, void* stream) {
  LinArgs p{};
  p.a = x; p.lda = ldx; p.a2 = x2; p.lda2 = ldx2;
  p.zin = nullptr; p.ldzin = 0; p.act_in_grad = 0;
  p.W = W; p.w_trans = 0; p.bias = b;
  p.K = K; p.N = N; p.M = M;
  p.out = y; p.ldo = ldy; p.accum = accum; p.act_out = act;
  p.zout = z; p.ldzo = ldz;
  return launch_linear(p, (hipStream_t)stream);
}

VAESNE_API int vaesne_linear_bwd_data(const float* dy, int64_t lddy, const float* z, int64_t ldz,
                                      int act, int64_t M, int N, const float* W, int K,
                                      float* dx, int64_t lddx, int accum, void* stream) {
  // dx[M, K] (+)= (dy * act'(z))[M, N] @ W[N, K]
  LinArgs p{};
  p.a = dy; p.lda = lddy; p.a2 = nullptr; p.lda2 = 0;
  p.zin = act ? z : nullptr; p.ldzin = ldz; p.act_in_grad = act;
  p.W = W; p.w_trans = 1; p.bias = nullptr;
  p.K = N; p.N = K; p.M = M;
  p.out = dx; p.ldo = lddx; p.accum = accum; p.act_out = ACT_NONE;
  p.zout = nullptr; p.ldzo = 0;
  return launch_linear(p, (hipStream_t)stream);
}

VAESNE_API int64_t vaesne_linear_bwd_weight_workspace(int64_t M, int O, int I) {
  return wgrad_groups(M) * ((int64_t)O * I + O) * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_linear_bwd_weight(const float* dy, int64_t lddy, const float* z, int64_t ldz,
                                        int act, const float* x, int64_t ldx, const float* x2,
                                        int64_t ldx2, int64_t M, int O, int I, float* dW,
                                        float* db, int accum, float* workspace,
                                        vaesne_colsum_list* defer, void* stream) {
  if (O < 1 || O > MAXN || I < 1 || I > MAXK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int F = O * I + O;
  int G = 1;
  if (M <= 0) {
    // empty batch: gradient is zero
    hipError_t me = hipMemsetAsync(workspace, 0, sizeof(float) * F, s);
    if (me != hipSuccess) return (int)me;
  } else {
    G = (int)wgrad_groups(M);
    WgtArgs p{dy, lddy, z, ldz, act, x, ldx, x2, ldx2, M, O, I, workspace};
    const int nob = (O + 31) / 32, nib = (I + 31) / 32;
    const dim3 grid(G, nob * nib);
#define VAESNE_WG(A, X)                                                                           \
  hipLaunchKernelGGL((linear_wgrad_kernel<A, X>), grid, dim3(NT), 0, s, p, nib, dW, db, accum)
    if (act == ACT_RELU) { if (x2) VAESNE_WG(ACT_RELU, true); else VAESNE_WG(ACT_RELU, false); }
    else if (act == ACT_GELU) { if (x2) VAESNE_WG(ACT_GELU, true); else VAESNE_WG(ACT_GELU, false); }
    else { if (x2) VAESNE_WG(ACT_NONE, true); else VAESNE_WG(ACT_NONE, false); }
#undef VAESNE_WG
    VAESNE_CHECK_LAUNCH();
    if (G == 1) return 0;   // written directly
  }
  if (!defer) return launch_colsum(workspace, G, F, dW, db, O * I, accum, s);
  const int rc = colsum_or_defer(defer, workspace, F, G, O * I, dW, accum, s);
  return rc ? rc : colsum_or_defer(defer, workspace + (int64_t)O * I, F, G, O, db, accum, s);
}

// ---------------------------------------------------------------------------
// grouped launches (one kernel for G independent linears of one shape)
// ---------------------------------------------------------------------------
VAESNE_API int vaesne_linear_fwd_group(int G, const vaesne_linear_group* g, int K, int N,
                                       void* stream) {
  if (G < 1 || G > LGMAX || !g) return (int)hipErrorInvalidValue;
  LinArgs pp[LGMAX];
  for (int i = 0; i < G; ++i) {
    LinArgs& p = pp[i];
    p = LinArgs{};
    p.a = g[i].x; p.lda = g[i].ldx; p.W = g[i].W; p.w_trans = 0; p.bias = g[i].b;
    p.K = K; p.N = N; p.M = g[i].M;
    p.out = g[i].y; p.ldo = g[i].ldy; p.accum = g[i].accum; p.act_out = ACT_NONE;
  }
  return launch_linear_n(pp, G, (hipStream_t)stream);
}

VAESNE_API int vaesne_linear_bwd_data_group(int G, const vaesne_linear_group* g, int K, int N,
                                            void* stream) {
  // per group: y[M, K] (+)= x[M, N] @ W[N, K]   (x = dy, y = dx)
  if (G < 1 || G > LGMAX || !g) return (int)hipErrorInvalidValue;
  LinArgs pp[LGMAX];
  for (int i = 0; i < G; ++i) {
    LinArgs& p = pp[i];
    p = LinArgs{};
    p.a = g[i].x; p.lda = g[i].ldx; p.W = g[i].W; p.w_trans = 1; p.bias = nullptr;
    p.K = N; p.N = K; p.M = g[i].M;
    p.out = g[i].y; p.ldo = g[i].ldy; p.accum = g[i].accum; p.act_out = ACT_NONE;
  }
  return launch_linear_n(pp, G, (hipStream_t)stream);
}

VAESNE_API int64_t vaesne_linear_bwd_weight_group_workspace(int G, int64_t M, int O, int I) {
  return (int64_t)G * vaesne_linear_bwd_weight_workspace(M, O, I);
}

// per group: dW[O, I] = dy^T x, db[O] = colsum(dy) over M rows (every group the same M)
VAESNE_API int vaesne_linear_bwd_weight_group(int G, const vaesne_wgrad_group* g, int64_t M, int O,
                                              int I, float* workspace, vaesne_colsum_list* defer,
                                              void* stream) {
  if (G < 1 || G > LGMAX || !g || O < 1 || O > MAXN || I < 1 || I > MAXK || M <= 0)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int F = O * I + O;
  const int Gr = (int)wgrad_groups(M);
  WgtGroup wg{};
  for (int i = 0; i < G; ++i) {
    wg.p[i] = WgtArgs{g[i].dy, g[i].lddy, nullptr, 0, 0, g[i].x, g[i].ldx, nullptr, 0, M, O, I,
                      workspace + (int64_t)i * Gr * F};
    wg.dW[i] = g[i].dW;
    wg.db[i] = g[i].db;
  }
  const int nob = (O + 31) / 32, nib = (I + 31) / 32;
  hipLaunchKernelGGL((linear_wgrad_group_kernel<ACT_NONE, false>), dim3(Gr, nob * nib, G), dim3(NT),
                     0, s, wg, nib, 0);
  VAESNE_CHECK_LAUNCH();
  if (Gr == 1) return 0;   // written directly
  for (int i = 0; i < G; ++i) {
    const float* ws = workspace + (int64_t)i * Gr * F;
    int rc;
    if (!defer) rc = launch_colsum(ws, Gr, F, g[i].dW, g[i].db, O * I, 0, s);
    else {
      rc = colsum_or_defer(defer, ws, F, Gr, O * I, g[i].dW, 0, s);
      if (!rc) rc = colsum_or_defer(defer, ws + (int64_t)O * I, F, Gr, O, g[i].db, 0, s);
    }
    if (rc) return rc;
  }
  return 0;
}
