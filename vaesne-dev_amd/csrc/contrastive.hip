// Contrastive objective of the photometry/spectra pretraining (§8(f) row 4):
//
//   negInfoNCE (losses.py:98-110):
//     n1 = F.normalize(z1), n2 = F.normalize(z2)      x / max(||x||_2, 1e-12)
//     logits[i, j] = (n1_i . n2_j) / T                (z1 @ z2.T / temperature)
//     out = -(CE(logits, arange) + CE(logits^T, arange)) / 2,
//     CE(l, arange) = mean_i (lse_j l[i, :] - l[i, i])  (cross_entropy, mean reduction)
//
// B (batch) is tens to a few thousand and D (proj_dim) is 8 in the scripts, so
// the B x B logits are never materialised in HBM: one workgroup per row i (and
// per side: rows of logits for n1, rows of logits^T = columns for n2) recomputes
// its row into LDS.  Both sides form n1_i . n2_j with the same summation order,
// so logits[i, j] and logits^T[j, i] are the same float (the diagonal too).
// Backward, per side s and row i (A = n_s, C = n_{1-s}):
//   dl_ij = -g / (2B) * (exp(l_ij - lse_s[i]) + exp(l_ij - lse_{1-s}[j]) - 2 delta_ij)
//   dn_i  = sum_j dl_ij C_j / T          (threads over (d, j-group), fixed-order sum)
//   dz_i  = (dn_i - n_i (n_i . dn_i)) / r_i   (r_i > eps)   or   dn_i / eps
// Every reduction has a fixed order: results are bitwise reproducible.
#include "common.h"

using namespace vaesne;

namespace {
constexpr int NT = 256;
constexpr float NORM_EPS = 1e-12f;   // F.normalize default eps

__device__ float blk_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < NT / 64; ++w) s += red[w];
  return s;
}

__device__ float blk_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = red[0];
  for (int w = 1; w < NT / 64; ++w) s = fmaxf(s, red[w]);
  return s;
}

struct NceArgs {
  const float* z[2];   // [B, D] each
  float* n;            // [2, B, D] normalised rows
  float* nrm;          // [2, B]    ||z_i||
  float* lse;          // [2, B]    row lse of logits (side 0) / of logits^T (side 1)
  float* diag;         // [B]       logits[i, i]
  int B, D;
  float T;
};

// one wave per row; grid (ceil(B / 4), 2)
__global__ __launch_bounds__(NT) void nce_normalize_kernel(NceArgs a) {
  const int s = blockIdx.y;
  const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.B) return;   // wave-uniform
  const float* z = a.z[s] + (int64_t)row * a.D;
  float ss = 0.f;
  for (int d = lane; d < a.D; d += 64) ss += z[d] * z[d];
  const float r = sqrtf(wave_sum(ss));
  const float den = fmaxf(r, NORM_EPS);
  float* n = a.n + ((int64_t)s * a.B + row) * a.D;
  for (int d = lane; d < a.D; d += 64) n[d] = z[d] / den;
  if (lane == 0) a.nrm[s * a.B + row] = r;
}

__device__ __forceinline__ float row_dot(const float* __restrict__ ai, const float* __restrict__ c,
                                         int D) {
  float acc = 0.f;
  for (int d = 0; d < D; ++d) acc = fmaf(ai[d], c[d], acc);
  return acc;
}

// dynamic LDS: a_i [D] | logits row [B] | red [NT/64]
__global__ __launch_bounds__(NT) void nce_lse_kernel(NceArgs a) {
  extern __shared__ float sm[];
  float* ai = sm;
  float* lrow = sm + a.D;
  float* red = lrow + a.B;
  const int i = blockIdx.x, s = blockIdx.y;
  const float* A = a.n + (int64_t)s * a.B * a.D;
  const float* C = a.n + (int64_t)(1 - s) * a.B * a.D;
  for (int d = threadIdx.x; d < a.D; d += NT) ai[d] = A[(int64_t)i * a.D + d];
  __syncthreads();
  float m = -INFINITY;
  for (int j = threadIdx.x; j < a.B; j += NT) {
    // side 0: n1_i . n2_j; side 1: n2_i . n1_j -- the same fmas in the same order as side
    // 0's (j, i) entry (fmaf is commutative in its product operands)
    const float l = row_dot(ai, C + (int64_t)j * a.D, a.D) / a.T;
    lrow[j] = l;
    m = fmaxf(m, l);
  }
  m = blk_max(m, red);
  float e = 0.f;
  for (int j = threadIdx.x; j < a.B; j += NT) e += expf(lrow[j] - m);
  e = blk_sum(e, red);
  if (threadIdx.x == 0) {
    a.lse[s * a.B + i] = m + logf(e);
    if (s == 0) a.diag[i] = lrow[i];
  }
}

__global__ __launch_bounds__(NT) void nce_loss_kernel(NceArgs a, float* __restrict__ loss) {
  __shared__ float red[NT / 64];
  float r = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < a.B; i += NT) {
    r += a.lse[i] - a.diag[i];
    c += a.lse[a.B + i] - a.diag[i];
  }
  r = blk_sum(r, red);
  c = blk_sum(c, red);
  if (threadIdx.x == 0) *loss = -(r / (float)a.B + c / (float)a.B) * 0.5f;
}

// dynamic LDS: a_i [D] | w [B] | part [NT] | dn [D] | red [NT/64]
__global__ __launch_bounds__(NT) void nce_bwd_kernel(NceArgs a, const float* __restrict__ gout,
                                                     float* dz0, float* dz1) {
  extern __shared__ float sm[];
  float* ai = sm;
  float* w = ai + a.D;
  float* part = w + a.B;
  float* dn = part + NT;
  float* red = dn + a.D;
  const int i = blockIdx.x, s = blockIdx.y;
  const float* A = a.n + (int64_t)s * a.B * a.D;
  const float* C = a.n + (int64_t)(1 - s) * a.B * a.D;
  const float* lse_own = a.lse + s * a.B;
  const float* lse_oth = a.lse + (1 - s) * a.B;
  const float coef = -(*gout) / (2.f * (float)a.B);
  for (int d = threadIdx.x; d < a.D; d += NT) ai[d] = A[(int64_t)i * a.D + d];
  __syncthreads();
  const float own = lse_own[i];
  for (int j = threadIdx.x; j < a.B; j += NT) {
    const float l = row_dot(ai, C + (int64_t)j * a.D, a.D) / a.T;
    float p = expf(l - own) + expf(l - lse_oth[j]);
    if (j == i) p -= 2.f;
    w[j] = coef * p / a.T;
  }
  __syncthreads();
  // dn[d] = sum_j w[j] C[j, d]: threads as (d within a chunk of Dc, j-group g)
  const int Dc = a.D < NT ? a.D : NT;
  const int G = NT / Dc;
  const int dl = threadIdx.x % Dc, g = threadIdx.x / Dc;
  for (int d0 = 0; d0 < a.D; d0 += Dc) {
    const int d = d0 + dl;
    float acc = 0.f;
    if (g < G && d < a.D)
      for (int j = g; j < a.B; j += G) acc = fmaf(w[j], C[(int64_t)j * a.D + d], acc);
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < Dc && d < a.D) {
      float t = 0.f;
      for (int q = 0; q < G; ++q) t += part[q * Dc + threadIdx.x];
      dn[d] = t;
    }
    __syncthreads();
  }
  // normalize backward
  float dot = 0.f;
  for (int d = threadIdx.x; d < a.D; d += NT) dot += ai[d] * dn[d];
  dot = blk_sum(dot, red);
  const float r = a.nrm[s * a.B + i];
  float* dz = (s == 0 ? dz0 : dz1) + (int64_t)i * a.D;
  for (int d = threadIdx.x; d < a.D; d += NT)
    dz[d] = r > NORM_EPS ? (dn[d] - ai[d] * dot) / r : dn[d] / NORM_EPS;
}

inline size_t lse_lds(int B, int D) { return sizeof(float) * ((size_t)D + B + NT / 64); }
inline size_t bwd_lds(int B, int D) { return sizeof(float) * (2 * (size_t)D + B + NT + NT / 64); }
constexpr size_t LDS_CAP = 64 * 1024;   // B up to ~16 K rows without a dynamic-LDS opt-in
}  // namespace

VAESNE_API int vaesne_infonce_fwd(const float* z1, const float* z2, int B, int D,
                                  float temperature, float* nz, float* nrm, float* lse,
                                  float* diag, float* loss, void* stream) {
  if (B <= 0 || D <= 0 || !(temperature > 0.f) || bwd_lds(B, D) > LDS_CAP)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  NceArgs a{{z1, z2}, nz, nrm, lse, diag, B, D, temperature};
  hipLaunchKernelGGL(nce_normalize_kernel, dim3((unsigned)cdiv(B, NT / 64), 2), dim3(NT), 0, st,
                     a);
  VAESNE_CHECK_LAUNCH();
  hipLaunchKernelGGL(nce_lse_kernel, dim3((unsigned)B, 2), dim3(NT), lse_lds(B, D), st, a);
  VAESNE_CHECK_LAUNCH();
  hipLaunchKernelGGL(nce_loss_kernel, dim3(1), dim3(NT), 0, st, a, loss);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_infonce_bwd(const float* nz, const float* nrm, const float* lse, int B,
                                  int D, float temperature, const float* gout, float* dz1,
                                  float* dz2, void* stream) {
  if (B <= 0 || D <= 0 || !(temperature > 0.f) || bwd_lds(B, D) > LDS_CAP)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  NceArgs a{{nullptr, nullptr}, const_cast<float*>(nz), const_cast<float*>(nrm),
            const_cast<float*>(lse), nullptr, B, D, temperature};
  hipLaunchKernelGGL(nce_bwd_kernel, dim3((unsigned)B, 2), dim3(NT), bwd_lds(B, D), st, a, gout,
                     dz1, dz2);
  VAESNE_CHECK_LAUNCH();
  return 0;
}
