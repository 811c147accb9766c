// Fused objectives of the VAESNe step (package/VAESNe/losses.py):
//
//   _m_iwae (losses.py:47-62), two modalities d in {0 photometry, 1 spectra}:
//     for r in {0,1} (which posterior drew z), k < K, b < B:
//       lpz  = sum_j log Laplace(z_r | pz_loc, pz_scale)
//       lqz  = LME_{m in {0,1}} sum_j log Laplace(z_r | mu_m, sc_m)
//       lpx  = sum_d llik_d * sum_l log Laplace(x_d | loc_rd, scale_rd)
//       lw[r*K + k, b] = lpz + lpx - lqz
//   m_iwae (losses.py:78-93): loss = sum_b LME_j lw[j, b]   (lme_sum)
//   elbo (losses.py:16-24 + torch/distributions/kl.py:331-338):
//     loss = mean_{k,b} ( llik * sum_l log p(x | loc, scale) ) - mean_b sum_j KL(q || pz)
//
// log Laplace(x | loc, s) = -log(2 s) - |x - loc| / s   (laplace.py:88-91);
// |.| differentiates to sign() with sign(0) = 0, as torch.abs.
// The length-L sums are wave-shuffle + LDS block reductions, one workgroup per
// (r, k, b) row; every sum has a fixed order (bitwise reproducible).  Backward
// kernels read upstream gradients from device memory (no host sync).
#include "common.h"

using namespace vaesne;

namespace {
constexpr int NT = 256;

struct IwaeArgs {
  const float* x[2];        // [B, L_d]
  float llik[2];
  int L[2];
  const float* loc[2][2];   // [r][d] -> [K, B, L_d]
  const float* scl[2][2];   // [r][d] -> [K, B, L_d]
  int64_t ks[2][2];         // [r][d] element stride between consecutive k of a cell
  const float* zs[2];       // [K, B, n]
  const float* mu[2];       // [B, n]
  const float* sc[2];       // [B, n]
  const float* pz_loc;      // [n]
  const float* pz_scale;    // [n]
  int K, B, n;
};

__device__ __forceinline__ float lap_logp(float x, float loc, float s) {
  return -logf(2.f * s) - fabsf(x - loc) / s;
}
__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__device__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// one workgroup per (r, k, b)
__global__ __launch_bounds__(NT) void iwae_lw_kernel(IwaeArgs a, float* __restrict__ lw) {
  __shared__ float red[NT / 64];
  const int b = blockIdx.x % a.B;
  const int rk = blockIdx.x / a.B;
  const int r = rk / a.K, k = rk - r * a.K;
  float lpx = 0.f;
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const int L = a.L[d];
    const float* xp = a.x[d] + (int64_t)b * L;
    const int64_t off = (int64_t)k * a.ks[r][d] + (int64_t)b * L;
    const float* lp = a.loc[r][d] + off;
    const float* sp = a.scl[r][d] + off;
    float s = 0.f;
    for (int l = threadIdx.x; l < L; l += NT) s += lap_logp(xp[l], lp[l], sp[l]);
    s = block_sum(s, red);
    lpx += a.llik[d] * s;
  }
  if (threadIdx.x == 0) {
    const float* z = a.zs[r] + ((int64_t)k * a.B + b) * a.n;
    float lpz = 0.f, lq0 = 0.f, lq1 = 0.f;
    for (int j = 0; j < a.n; ++j) {
      float zz = z[j];
      lpz += lap_logp(zz, a.pz_loc[j], a.pz_scale[j]);
      lq0 += lap_logp(zz, a.mu[0][(int64_t)b * a.n + j], a.sc[0][(int64_t)b * a.n + j]);
      lq1 += lap_logp(zz, a.mu[1][(int64_t)b * a.n + j], a.sc[1][(int64_t)b * a.n + j]);
    }
    float mx = fmaxf(lq0, lq1);
    float lqz = mx + logf(expf(lq0 - mx) + expf(lq1 - mx)) - logf(2.f);
    lw[(int64_t)rk * a.B + b] = lpz + lpx - lqz;
  }
}

// loss = sum_b LME_j lw[j, b]
__global__ __launch_bounds__(NT) void lme_sum_fwd_kernel(const float* __restrict__ lw, int J,
                                                         int B, float* __restrict__ loss,
                                                         int* __restrict__ nonfinite) {
  __shared__ float red[NT / 64];
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += NT) {
    float mx = -INFINITY;
    for (int j = 0; j < J; ++j) mx = fmaxf(mx, lw[(int64_t)j * B + b]);
    float s = 0.f;
    for (int j = 0; j < J; ++j) s += expf(lw[(int64_t)j * B + b] - mx);
    acc += mx + logf(s) - logf((float)J);
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    *loss = acc;
    if (nonfinite && !isfinite(acc)) nonfinite[1] = 1;
  }
}

// dlw[j, b] = g * softmax_j(lw[:, b])
__global__ void lme_sum_bwd_kernel(const float* __restrict__ lw, int J, int B,
                                   const float* __restrict__ gout, float* __restrict__ dlw) {
  int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float g = *gout;
  float mx = -INFINITY;
  for (int j = 0; j < J; ++j) mx = fmaxf(mx, lw[(int64_t)j * B + b]);
  float s = 0.f;
  for (int j = 0; j < J; ++j) s += expf(lw[(int64_t)j * B + b] - mx);
  float lse = mx + logf(s);
  for (int j = 0; j < J; ++j) dlw[(int64_t)j * B + b] = g * expf(lw[(int64_t)j * B + b] - lse);
}

// dloc[r][d][k, b, l] = dlw[rK+k, b] * llik_d * sign(x - loc) / s
__global__ void iwae_dloc_kernel(IwaeArgs a, const float* __restrict__ dlw, float* dl00,
                                 float* dl01, float* dl10, float* dl11) {
  const int64_t n0 = (int64_t)a.K * a.B * a.L[0];
  const int64_t per_r = n0 + (int64_t)a.K * a.B * a.L[1];
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; t < 2 * per_r; t += (int64_t)gridDim.x * blockDim.x) {
    int r = (int)(t / per_r);
    int64_t u = t - r * per_r;
    int d = u < n0 ? 0 : 1;
    int64_t e = d == 0 ? u : u - n0;
    const int L = a.L[d];
    int64_t kb = e / L;
    int l = (int)(e - kb * L);
    int b = (int)(kb % a.B);
    int k = (int)(kb / a.B);
    const int64_t idx = (int64_t)k * a.ks[r][d] + (int64_t)b * L + l;
    float x = a.x[d][(int64_t)b * L + l];
    float loc = a.loc[r][d][idx];
    float gr = dlw[(int64_t)(r * a.K + k) * a.B + b] * a.llik[d] * sgnf(x - loc) / a.scl[r][d][idx];
    float* out = r == 0 ? (d == 0 ? dl00 : dl01) : (d == 0 ? dl10 : dl11);
    if (out) out[idx] = gr;
  }
}

// latent gradients, one thread per (b, j), gw = dlw[rK+k, b]:
//   dz_r[k,b,j]  = gw ( -sgn(z - pl)/ps + sum_m alpha_m sgn(z - mu_m)/sc_m )
//   dmu_m[b,j]   = sum_{r,k} gw ( -alpha_{rk,m} sgn(z - mu_m) / sc_m )
//   dsc_m[b,j]   = sum_{r,k} gw ( -alpha_{rk,m} (-1/sc_m + |z - mu_m| / sc_m^2) )
// alpha_{rk,m} = softmax_m( sum_j log q_m(z_rk) ) (recomputed per thread).
// One workgroup per b.  Phase 1: thread t < 2K computes the mixture weights
// alpha_{rk,m} of sample (r, k) once (a thread per (b, j) recomputed them n times:
// 2K*n^2 serial log-probs per thread, ~55 us at cfg 5); phase 2: thread j < n sums
// over (r, k) in the same order as before (bitwise-identical results).
constexpr int DLAT_MAXRK = 512;
__global__ void iwae_dlat_kernel(IwaeArgs a, const float* __restrict__ dlw, float* dz0, float* dz1,
                                 float* dmu0, float* dsc0, float* dmu1, float* dsc1) {
  __shared__ float al[2][DLAT_MAXRK];
  const int b = blockIdx.x;
  const int nrk = 2 * a.K;
  for (int t = threadIdx.x; t < nrk; t += blockDim.x) {
    const int r = t / a.K, k = t - r * a.K;
    const float* zrow = a.zs[r] + ((int64_t)k * a.B + b) * a.n;
    float lq0 = 0.f, lq1 = 0.f;
    for (int jj = 0; jj < a.n; ++jj) {
      float zz = zrow[jj];
      lq0 += lap_logp(zz, a.mu[0][(int64_t)b * a.n + jj], a.sc[0][(int64_t)b * a.n + jj]);
      lq1 += lap_logp(zz, a.mu[1][(int64_t)b * a.n + jj], a.sc[1][(int64_t)b * a.n + jj]);
    }
    float mx = fmaxf(lq0, lq1);
    float e0 = expf(lq0 - mx), e1 = expf(lq1 - mx);
    al[0][t] = e0 / (e0 + e1);
    al[1][t] = e1 / (e0 + e1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.n; j += blockDim.x) {
    const int64_t t = (int64_t)b * a.n + j;
    const float mu0 = a.mu[0][t], sc0 = a.sc[0][t], mu1 = a.mu[1][t], sc1 = a.sc[1][t];
    const float pl = a.pz_loc[j], ps = a.pz_scale[j];
    float gm0 = 0.f, gs0 = 0.f, gm1 = 0.f, gs1 = 0.f;
    for (int r = 0; r < 2; ++r) {
      for (int k = 0; k < a.K; ++k) {
        const float al0 = al[0][r * a.K + k], al1 = al[1][r * a.K + k];
        float gw = dlw[(int64_t)(r * a.K + k) * a.B + b];
        float z = a.zs[r][((int64_t)k * a.B + b) * a.n + j];
        float d0 = z - mu0, d1 = z - mu1;
        float dz = gw * (-sgnf(z - pl) / ps + al0 * sgnf(d0) / sc0 + al1 * sgnf(d1) / sc1);
        float* dzr = r == 0 ? dz0 : dz1;
        if (dzr) dzr[((int64_t)k * a.B + b) * a.n + j] = dz;
        gm0 += gw * (-al0 * sgnf(d0) / sc0);
        gm1 += gw * (-al1 * sgnf(d1) / sc1);
        gs0 += gw * (-al0 * (-1.f / sc0 + fabsf(d0) / (sc0 * sc0)));
        gs1 += gw * (-al1 * (-1.f / sc1 + fabsf(d1) / (sc1 * sc1)));
      }
    }
    if (dmu0) dmu0[t] = gm0;
    if (dsc0) dsc0[t] = gs0;
    if (dmu1) dmu1[t] = gm1;
    if (dsc1) dsc1[t] = gs1;
  }
}

// ---------------------------------------------------------------- elbo ----
struct ElboArgs {
  const float* x; float llik; int L;
  const float* loc; const float* scl;  // [K, B, L]
  const float* mu; const float* sc;    // [B, n]
  const float* pz_loc; const float* pz_scale;  // [n]
  int K, B, n;
  float* lpx;                          // [K, B]
};

__global__ __launch_bounds__(NT) void elbo_lpx_kernel(ElboArgs a) {
  __shared__ float red[NT / 64];
  const int kb = blockIdx.x;
  const int b = kb % a.B;
  const float* xp = a.x + (int64_t)b * a.L;
  const float* lp = a.loc + (int64_t)kb * a.L;
  const float* sp = a.scl + (int64_t)kb * a.L;
  float s = 0.f;
  for (int l = threadIdx.x; l < a.L; l += NT) s += lap_logp(xp[l], lp[l], sp[l]);
  s = block_sum(s, red);
  if (threadIdx.x == 0) a.lpx[kb] = a.llik * s;
}

__device__ __forceinline__ float kl_lap(float mu, float sc, float pl, float ps) {
  float ratio = sc / ps;
  float t = fabsf(mu - pl);
  return -logf(ratio) + t / ps + ratio * expf(-t / sc) - 1.f;
}

// loss = mean_{k,b} lpx - mean_b sum_j KL
__global__ __launch_bounds__(NT) void elbo_loss_kernel(ElboArgs a, float* __restrict__ loss,
                                                       int* __restrict__ nonfinite) {
  __shared__ float red[NT / 64];
  float s1 = 0.f;
  for (int i = threadIdx.x; i < a.K * a.B; i += NT) s1 += a.lpx[i];
  s1 = block_sum(s1, red);
  float s2 = 0.f;
  for (int i = threadIdx.x; i < a.B * a.n; i += NT) {
    int j = i % a.n;
    s2 += kl_lap(a.mu[i], a.sc[i], a.pz_loc[j], a.pz_scale[j]);
  }
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) {
    const float l = s1 / (float)(a.K * a.B) - s2 / (float)a.B;
    *loss = l;
    if (nonfinite && !isfinite(l)) nonfinite[1] = 1;
  }
}

__global__ void elbo_dloc_kernel(ElboArgs a, const float* __restrict__ gout, float* dloc) {
  const float g = *gout / (float)(a.K * a.B);
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)a.K * a.B * a.L;
  for (; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t kb = t / a.L;
    int l = (int)(t - kb * a.L);
    int b = (int)(kb % a.B);
    float x = a.x[(int64_t)b * a.L + l];
    dloc[t] = g * a.llik * sgnf(x - a.loc[t]) / a.scl[t];
  }
}

// d/dmu, d/dsc of -mean_b sum_j KL(Laplace(mu, sc) || Laplace(pl, ps))
__global__ void elbo_dlat_kernel(ElboArgs a, const float* __restrict__ gout, float* dmu,
                                 float* dsc) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.B * a.n) return;
  const float g = -*gout / (float)a.B;
  const int j = (int)(t % a.n);
  const float mu = a.mu[t], sc = a.sc[t], pl = a.pz_loc[j], ps = a.pz_scale[j];
  const float tt = fabsf(mu - pl);
  const float e = expf(-tt / sc);
  if (dmu) dmu[t] = g * sgnf(mu - pl) * (1.f / ps) * (1.f - e);
  if (dsc) dsc[t] = g * (-1.f / sc + (1.f / ps) * e * (1.f + tt / sc));
}

inline unsigned nblk(int64_t n, int64_t cap = 65536) {
  int64_t b = (n + NT - 1) / NT;
  if (b > cap) b = cap;
  return (unsigned)(b < 1 ? 1 : b);
}

IwaeArgs make_iwae(const float* const* xs, const float* llik, const int* L,
                   const float* const* locs, const float* const* scls, const int64_t* kstride,
                   const float* const* zs,
                   const float* const* mus, const float* const* scs, const float* pz_loc,
                   const float* pz_scale, int K, int B, int n) {
  IwaeArgs a{};
  for (int d = 0; d < 2; ++d) {
    a.x[d] = xs[d];
    a.llik[d] = llik[d];
    a.L[d] = L[d];
    a.zs[d] = zs[d];
    a.mu[d] = mus[d];
    a.sc[d] = scs[d];
  }
  for (int r = 0; r < 2; ++r)
    for (int d = 0; d < 2; ++d) {
      a.loc[r][d] = locs[2 * r + d];
      a.scl[r][d] = scls[2 * r + d];
      a.ks[r][d] = kstride ? kstride[2 * r + d] : (int64_t)B * L[d];
    }
  a.pz_loc = pz_loc; a.pz_scale = pz_scale;
  a.K = K; a.B = B; a.n = n;
  return a;
}

}  // namespace

VAESNE_API int vaesne_iwae_lw_fwd(const float* const* x, const float* llik, const int* L,
                                  const float* const* loc, const float* const* scale,
                                  const int64_t* kstride,
                                  const float* const* zs, const float* const* mu,
                                  const float* const* sc, const float* pz_loc,
                                  const float* pz_scale, int K, int B, int n, float* lw,
                                  void* stream) {
  if (B <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  IwaeArgs a = make_iwae(x, llik, L, loc, scale, kstride, zs, mu, sc, pz_loc, pz_scale, K, B, n);
  hipLaunchKernelGGL(iwae_lw_kernel, dim3((unsigned)(2 * K * B)), dim3(NT), 0,
                     (hipStream_t)stream, a, lw);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_iwae_lw_bwd(const float* const* x, const float* llik, const int* L,
                                  const float* const* loc, const float* const* scale,
                                  const int64_t* kstride,
                                  const float* const* zs, const float* const* mu,
                                  const float* const* sc, const float* pz_loc,
                                  const float* pz_scale, int K, int B, int n, const float* dlw,
                                  float* const* dloc, float* const* dzs, float* const* dmu,
                                  float* const* dsc, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  IwaeArgs a = make_iwae(x, llik, L, loc, scale, kstride, zs, mu, sc, pz_loc, pz_scale, K, B, n);
  int64_t tot = 2 * (int64_t)K * B * (L[0] + L[1]);
  hipLaunchKernelGGL(iwae_dloc_kernel, dim3(nblk(tot)), dim3(NT), 0, s, a, dlw, dloc[0], dloc[1],
                     dloc[2], dloc[3]);
  VAESNE_CHECK_LAUNCH();
  if (2 * K > DLAT_MAXRK) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(iwae_dlat_kernel, dim3((unsigned)B), dim3(64), 0, s, a, dlw, dzs[0], dzs[1],
                     dmu[0], dsc[0], dmu[1], dsc[1]);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_lme_sum_fwd(const float* lw, int J, int B, float* loss, int* nonfinite,
                                  void* stream) {
  hipLaunchKernelGGL(lme_sum_fwd_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, lw, J, B,
                     loss, nonfinite);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_lme_sum_bwd(const float* lw, int J, int B, const float* gout, float* dlw,
                                  void* stream) {
  hipLaunchKernelGGL(lme_sum_bwd_kernel, dim3(nblk(B)), dim3(NT), 0, (hipStream_t)stream, lw, J,
                     B, gout, dlw);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_elbo_fwd(const float* x, int L, float llik, const float* loc,
                               const float* scale, const float* mu, const float* sc,
                               const float* pz_loc, const float* pz_scale, int K, int B, int n,
                               float* lpx, float* loss, int* nonfinite, void* stream) {
  if (B <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  ElboArgs a{x, llik, L, loc, scale, mu, sc, pz_loc, pz_scale, K, B, n, lpx};
  hipLaunchKernelGGL(elbo_lpx_kernel, dim3((unsigned)(K * B)), dim3(NT), 0, s, a);
  VAESNE_CHECK_LAUNCH();
  hipLaunchKernelGGL(elbo_loss_kernel, dim3(1), dim3(NT), 0, s, a, loss, nonfinite);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int vaesne_elbo_bwd(const float* x, int L, float llik, const float* loc,
                               const float* scale, const float* mu, const float* sc,
                               const float* pz_loc, const float* pz_scale, int K, int B, int n,
                               const float* gout, float* dloc, float* dmu, float* dsc,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  ElboArgs a{x, llik, L, loc, scale, mu, sc, pz_loc, pz_scale, K, B, n, nullptr};
  hipLaunchKernelGGL(elbo_dloc_kernel, dim3(nblk((int64_t)K * B * L)), dim3(NT), 0, s, a, gout,
                     dloc);
  VAESNE_CHECK_LAUNCH();
  hipLaunchKernelGGL(elbo_dlat_kernel, dim3(nblk((int64_t)B * n)), dim3(NT), 0, s, a, gout, dmu,
                     dsc);
  VAESNE_CHECK_LAUNCH();
  return 0;
}
