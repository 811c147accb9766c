// Post-LN residual join of TransformerBlock (util_layers.py:291-307):
//     y = LayerNorm(x + Dropout(res))      eps = 1e-5, biased variance
// fused into one pass over the [M, E] token rows (E = model_dim = 32 or 64),
// one row per lane (the row lives in registers).  The dropout mask is
// regenerated in the backward from the counter-based RNG, never stored.
#include "common.h"

using namespace vaesne;

namespace {

constexpr int NT = 256;

template <int E>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[E]) {
#pragma unroll
  for (int c = 0; c < E; c += 4) {
    float4 t = *reinterpret_cast<const float4*>(p + c);
    v[c] = t.x; v[c + 1] = t.y; v[c + 2] = t.z; v[c + 3] = t.w;
  }
}
template <int E>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[E]) {
#pragma unroll
  for (int c = 0; c < E; c += 4)
    *reinterpret_cast<float4*>(p + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
}

// dropout keep-scale for element (r, c): one 32-bit hash per pair of columns
template <int E>
__device__ __forceinline__ void drop_scales(uint32_t key, int64_t r, uint32_t thr, float inv_keep,
                                            float (&sc)[E]) {
#pragma unroll
  for (int c = 0; c < E; c += 2) {
    uint32_t h = rand_u32(key, (uint64_t)(r * (E / 2) + c / 2));
    sc[c] = ((h & 0xffffu) >= thr) ? inv_keep : 0.f;
    sc[c + 1] = ((h >> 16) >= thr) ? inv_keep : 0.f;
  }
}

template <int E>
__global__ __launch_bounds__(NT) void add_ln_fwd_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ res, int64_t ldres,
    int64_t M, const float* __restrict__ gamma, const float* __restrict__ beta, float p_drop,
    const int64_t* __restrict__ rng_state, uint32_t call_id, float* __restrict__ y, int64_t ldy,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (r >= M) return;
  float v[E], t[E];
  load_row<E>(x + r * ldx, v);
  if (res) {
    load_row<E>(res + r * ldres, t);
    if (p_drop > 0.f) {
      float sc[E];
      drop_scales<E>(key_of(rng_state, call_id), r, drop_thr16(p_drop), 1.f / (1.f - p_drop), sc);
#pragma unroll
      for (int c = 0; c < E; ++c) t[c] *= sc[c];
    }
#pragma unroll
    for (int c = 0; c < E; ++c) v[c] += t[c];
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < E; ++c) s += v[c];
  const float mu = s * (1.f / E);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < E; ++c) {
    float d = v[c] - mu;
    q = fmaf(d, d, q);
  }
  const float rs = rsqrtf(q * (1.f / E) + 1e-5f);
#pragma unroll
  for (int c = 0; c < E; ++c) v[c] = fmaf((v[c] - mu) * rs, gamma[c], beta[c]);
  store_row<E>(y + r * ldy, v);
  mean_out[r] = mu;
  rstd_out[r] = rs;
}

template <int E>
__global__ __launch_bounds__(NT) void add_ln_bwd_kernel(
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ res, int64_t ldres, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, float p_drop,
    const int64_t* __restrict__ rng_state, uint32_t call_id, float* __restrict__ dx, int64_t lddx,
    int accum_dx, float* __restrict__ dres, int64_t lddres, int accum_dres,
    float* __restrict__ partial /* [grid][2E] */) {
  __shared__ float red[NT / 64][2 * E];
  float dg[E], dbt[E];
#pragma unroll
  for (int c = 0; c < E; ++c) { dg[c] = 0.f; dbt[c] = 0.f; }
  const uint32_t key = (res && p_drop > 0.f) ? key_of(rng_state, call_id) : 0u;
  const uint32_t thr = drop_thr16(p_drop);
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  for (int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x; r < M; r += (int64_t)gridDim.x * NT) {
    float v[E], g[E], sc[E];
    load_row<E>(x + r * ldx, v);
    if (res) {
      float t[E];
      load_row<E>(res + r * ldres, t);
      if (p_drop > 0.f) {
        drop_scales<E>(key, r, thr, inv_keep, sc);
#pragma unroll
        for (int c = 0; c < E; ++c) t[c] *= sc[c];
      } else {
#pragma unroll
        for (int c = 0; c < E; ++c) sc[c] = 1.f;
      }
#pragma unroll
      for (int c = 0; c < E; ++c) v[c] += t[c];
    }
    load_row<E>(dy + r * lddy, g);
    const float mu = mean_in[r], rs = rstd_in[r];
    float mg = 0.f, mgx = 0.f;
#pragma unroll
    for (int c = 0; c < E; ++c) {
      float xh = (v[c] - mu) * rs;
      dg[c] = fmaf(g[c], xh, dg[c]);
      dbt[c] += g[c];
      float gg = g[c] * gamma[c];
      v[c] = xh;
      g[c] = gg;
      mg += gg;
      mgx = fmaf(gg, xh, mgx);
    }
    mg *= (1.f / E);
    mgx *= (1.f / E);
#pragma unroll
    for (int c = 0; c < E; ++c) g[c] = rs * (g[c] - mg - v[c] * mgx);
    if (dx) {
      if (accum_dx) {
        float o[E];
        load_row<E>(dx + r * lddx, o);
#pragma unroll
        for (int c = 0; c < E; ++c) o[c] += g[c];
        store_row<E>(dx + r * lddx, o);
      } else {
        store_row<E>(dx + r * lddx, g);
      }
    }
    if (res && dres) {
#pragma unroll
      for (int c = 0; c < E; ++c) g[c] *= sc[c];
      if (accum_dres) {
        float o[E];
        load_row<E>(dres + r * lddres, o);
#pragma unroll
        for (int c = 0; c < E; ++c) o[c] += g[c];
        store_row<E>(dres + r * lddres, o);
      } else {
        store_row<E>(dres + r * lddres, g);
      }
    }
  }
  // block reduction of dgamma / dbeta (fixed order)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < E; ++c) {
    float a = wave_sum(dg[c]);
    float b = wave_sum(dbt[c]);
    if (lane == 0) { red[wave][c] = a; red[wave][E + c] = b; }
  }
  __syncthreads();
  if (threadIdx.x < 2 * E) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[w][threadIdx.x];
    partial[(int64_t)blockIdx.x * 2 * E + threadIdx.x] = s;
  }
}

int ln_grid(int64_t M) {
  int64_t b = (M + NT - 1) / NT;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

}  // namespace

VAESNE_API int vaesne_add_ln_fwd(const float* x, int64_t ldx, const float* res, int64_t ldres,
                                 int64_t M, int E, const float* gamma, const float* beta,
                                 float p_drop, const int64_t* rng_state, uint32_t call_id,
                                 float* y, int64_t ldy, float* mean, float* rstd, void* stream) {
  if (M <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((M + NT - 1) / NT));
  if (E == 32)
    hipLaunchKernelGGL(add_ln_fwd_kernel<32>, grid, dim3(NT), 0, s, x, ldx, res, ldres, M, gamma,
                       beta, p_drop, rng_state, call_id, y, ldy, mean, rstd);
  else if (E == 64)
    hipLaunchKernelGGL(add_ln_fwd_kernel<64>, grid, dim3(NT), 0, s, x, ldx, res, ldres, M, gamma,
                       beta, p_drop, rng_state, call_id, y, ldy, mean, rstd);
  else
    return (int)hipErrorInvalidValue;
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int64_t vaesne_add_ln_bwd_workspace(int64_t M, int E) {
  return (int64_t)ln_grid(M) * 2 * E * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_add_ln_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                 const float* res, int64_t ldres, int64_t M, int E,
                                 const float* gamma, const float* mean, const float* rstd,
                                 float p_drop, const int64_t* rng_state, uint32_t call_id,
                                 float* dx, int64_t lddx, int accum_dx, float* dres,
                                 int64_t lddres, int accum_dres, float* dgamma, float* dbeta,
                                 int accum_param, float* workspace, vaesne_colsum_list* defer,
                                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int G = ln_grid(M);
  if (M <= 0) {
    hipError_t me = hipMemsetAsync(workspace, 0, sizeof(float) * 2 * E, s);
    if (me != hipSuccess) return (int)me;
    G = 1;
  } else if (E == 32) {
    hipLaunchKernelGGL(add_ln_bwd_kernel<32>, dim3(G), dim3(NT), 0, s, dy, lddy, x, ldx, res,
                       ldres, M, gamma, mean, rstd, p_drop, rng_state, call_id, dx, lddx, accum_dx,
                       dres, lddres, accum_dres, workspace);
  } else if (E == 64) {
    hipLaunchKernelGGL(add_ln_bwd_kernel<64>, dim3(G), dim3(NT), 0, s, dy, lddy, x, ldx, res,
                       ldres, M, gamma, mean, rstd, p_drop, rng_state, call_id, dx, lddx, accum_dx,
                       dres, lddres, accum_dres, workspace);
  } else {
    return (int)hipErrorInvalidValue;
  }
  VAESNE_CHECK_LAUNCH();
  if (!defer) return launch_colsum(workspace, G, 2 * E, dgamma, dbeta, E, accum_param, s);
  const int rc = colsum_or_defer(defer, workspace, 2 * E, G, E, dgamma, accum_param, s);
  return rc ? rc : colsum_or_defer(defer, workspace + E, 2 * E, G, E, dbeta, accum_param, s);
}

// generic fixed-order partial-sum reduction (used by the host for other
// per-workgroup partial buffers): out0[f] (+)= sum_g partial[g][f], f < split;
// out1[f - split] likewise for f >= split.
VAESNE_API int vaesne_reduce_partials(const float* partial, int G, int F, float* out0, float* out1,
                                      int split, int accum, void* stream) {
  return launch_colsum(partial, G, F, out0, out1, split, accum, (hipStream_t)stream);
}
