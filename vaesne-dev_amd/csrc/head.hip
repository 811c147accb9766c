// Fused decoder output head: singlelayerMLP(E -> 1) on the decoder's residual sum,
//   y[t] = W2 . relu(W1 (x[t] + h[t]) + b1) + b2
// (util_layers.py:9-18 fc2(relu(fc1(.))), as SpectraLayers.py:63 get_flux(x + h) and
// PhotometricLayers.py:69 get_photo(x + h) call it).  Two nn.Linear launches and the
// stored [M, E] pre-activation become one pass over the tokens; the backward
// recomputes the pre-activation and writes d(x + h) and the fc1 pre-activation
// gradient (the fc1 weight gradient's input) in one pass, the fc2 weight / bias
// gradients as per-workgroup partials (fixed-order column sum, deferrable).
// Thread = token; the weights sit in LDS and are read as wave-wide broadcasts
// (as scalar-register operands the compiler keeps all 1024 of W1 live and spills
// them into VGPR lanes: one v_readlane per FMA).
#include <algorithm>

#include "common.h"

using namespace vaesne;

namespace {

constexpr int HE = 32;        // model_dim of the reference decoders
constexpr int HNT = 256;
constexpr int HPART = HE + 1; // partial row: dW2[0..E), db2

__device__ __forceinline__ void head_input(const float* __restrict__ x, int64_t ldx,
                                           const float* __restrict__ h, int64_t ldh, int64_t t,
                                           float (&s)[HE]) {
#pragma unroll
  for (int i = 0; i < HE; i += 4) {
    const float4 a = *reinterpret_cast<const float4*>(x + t * ldx + i);
    s[i] = a.x; s[i + 1] = a.y; s[i + 2] = a.z; s[i + 3] = a.w;
  }
  if (h) {
#pragma unroll
    for (int i = 0; i < HE; i += 4) {
      const float4 b = *reinterpret_cast<const float4*>(h + t * ldh + i);
      s[i] += b.x; s[i + 1] += b.y; s[i + 2] += b.z; s[i + 3] += b.w;
    }
  }
}

// W row-major [HE][HE] into LDS, optionally transposed
// (all of a thread's loads in flight before its LDS stores)
__device__ __forceinline__ void stage_w(float* dst, const float* __restrict__ W, bool transpose) {
  static_assert(HE * HE % HNT == 0, "stage_w: every thread stages the same count of W");
  constexpr int N = HE * HE / HNT;
  float r[N];
#pragma unroll
  for (int j = 0; j < N; ++j) r[j] = W[threadIdx.x + j * HNT];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int k = threadIdx.x + j * HNT, o = k / HE, i = k - o * HE;
    dst[transpose ? i * HE + o : k] = r[j];
  }
}
typedef float f2 __attribute__((ext_vector_type(2)));

// dot of LDS row r (broadcast float4 reads) with v held as 16 packed pairs: 16 packed
// FMAs (v_pk_fma_f32) and one add; written out so the compiler's pair-building
// vectoriser has nothing to do (left to itself it copies every operand pair)
__device__ __forceinline__ float row_dot(const float* r, const f2 (&v)[HE / 2], float acc) {
  f2 a = (f2){acc, 0.f};
#pragma unroll
  for (int i = 0; i < HE / 2; i += 2) {
    const float4 w = *reinterpret_cast<const float4*>(r + 2 * i);
    a = __builtin_elementwise_fma((f2){w.x, w.y}, v[i], a);
    a = __builtin_elementwise_fma((f2){w.z, w.w}, v[i + 1], a);
  }
  return a.x + a.y;
}

__global__ __launch_bounds__(HNT) void head_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ h, int64_t ldh,
                                                        int64_t M, const float* __restrict__ W1,
                                                        const float* __restrict__ b1,
                                                        const float* __restrict__ W2,
                                                        const float* __restrict__ b2,
                                                        float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float Ws[HE * HE];
  __shared__ float Bs[HE], W2s[HE];
  stage_w(Ws, W1, false);
  if (threadIdx.x < HE) { Bs[threadIdx.x] = b1[threadIdx.x]; W2s[threadIdx.x] = W2[threadIdx.x]; }
  __syncthreads();
  const float bias2 = b2[0];
  for (int64_t t = (int64_t)blockIdx.x * HNT + threadIdx.x; t < M; t += (int64_t)gridDim.x * HNT) {
    float sv[HE];
    head_input(x, ldx, h, ldh, t, sv);
    f2 s[HE / 2];
#pragma unroll
    for (int i = 0; i < HE / 2; ++i) s[i] = (f2){sv[2 * i], sv[2 * i + 1]};
    float acc = bias2;
#pragma unroll 4
    for (int o = 0; o < HE; ++o)
      acc = fmaf(W2s[o], fmaxf(row_dot(Ws + o * HE, s, Bs[o]), 0.f), acc);
    y[t] = acc;
  }
}

// ds = d(x + h) [M, E], g = dz1 [M, E]; part[block][HPART] = (sum_t dy a, sum_t dy)
__global__ __launch_bounds__(HNT) void head_bwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ h, int64_t ldh,
                                                        const float* __restrict__ dy, int64_t M,
                                                        const float* __restrict__ W1,
                                                        const float* __restrict__ b1,
                                                        const float* __restrict__ W2,
                                                        float* __restrict__ ds,
                                                        float* __restrict__ g,
                                                        float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float Ws[HE * HE];
  __shared__ __attribute__((aligned(16))) float WT[HE * HE];
  __shared__ float Bs[HE], W2s[HE];
  __shared__ float red[HNT / 64][HPART];
  stage_w(Ws, W1, false);
  stage_w(WT, W1, true);
  if (threadIdx.x < HE) { Bs[threadIdx.x] = b1[threadIdx.x]; W2s[threadIdx.x] = W2[threadIdx.x]; }
  __syncthreads();
  float aw[HE], ab = 0.f;
#pragma unroll
  for (int o = 0; o < HE; ++o) aw[o] = 0.f;
  for (int64_t t = (int64_t)blockIdx.x * HNT + threadIdx.x; t < M; t += (int64_t)gridDim.x * HNT) {
    float sv[HE], go[HE];
    head_input(x, ldx, h, ldh, t, sv);
    f2 s[HE / 2], gp[HE / 2];
#pragma unroll
    for (int i = 0; i < HE / 2; ++i) s[i] = (f2){sv[2 * i], sv[2 * i + 1]};
    const float d = dy[t];
    ab += d;
    // (compiler barriers per output: without them the scheduler hoists the LDS rows
    // of every iteration and spills)
#pragma unroll
    for (int o = 0; o < HE; ++o) {
      const float z = row_dot(Ws + o * HE, s, Bs[o]);
      aw[o] = fmaf(d, fmaxf(z, 0.f), aw[o]);
      go[o] = z > 0.f ? d * W2s[o] : 0.f;       // relu'(z) = 1 for z > 0 (torch)
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int o = 0; o < HE; o += 4)
      *reinterpret_cast<float4*>(g + t * HE + o) = make_float4(go[o], go[o + 1], go[o + 2], go[o + 3]);
#pragma unroll
    for (int i = 0; i < HE / 2; ++i) gp[i] = (f2){go[2 * i], go[2 * i + 1]};
#pragma unroll
    for (int i = 0; i < HE; ++i) {
      sv[i] = row_dot(WT + i * HE, gp, 0.f);     // W1^T go
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < HE; i += 4)
      *reinterpret_cast<float4*>(ds + t * HE + i) = make_float4(sv[i], sv[i + 1], sv[i + 2], sv[i + 3]);
  }
  // fixed-order workgroup sums of the fc2 partials
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 0; o < HE; ++o) {
    const float v = wave_sum(aw[o]);
    if (lane == 0) red[w][o] = v;
  }
  {
    const float v = wave_sum(ab);
    if (lane == 0) red[w][HE] = v;
  }
  __syncthreads();
  if (threadIdx.x < HPART) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < HNT / 64; ++k) v += red[k][threadIdx.x];
    part[(int64_t)blockIdx.x * HPART + threadIdx.x] = v;
  }
}

int head_blocks(int64_t M) {
  return (int)std::min<int64_t>(1024, (M + HNT - 1) / HNT);
}

bool head_args_ok(const float* x, int64_t ldx, const float* h, int64_t ldh, int E) {
  return E == HE && x && (uintptr_t)x % 16 == 0 && ldx % 4 == 0 &&
         (!h || ((uintptr_t)h % 16 == 0 && ldh % 4 == 0));
}

}  // namespace

VAESNE_API int vaesne_mlp_head_fwd(const float* x, int64_t ldx, const float* h, int64_t ldh,
                                   int64_t M, int E, const float* W1, const float* b1,
                                   const float* W2, const float* b2, float* y, void* stream) {
  if (M <= 0) return 0;
  if (!head_args_ok(x, ldx, h, ldh, E) || !W1 || !b1 || !W2 || !b2 || !y)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(head_fwd_kernel, dim3((unsigned)head_blocks(M)), dim3(HNT), 0,
                     (hipStream_t)stream, x, ldx, h, ldh, M, W1, b1, W2, b2, y);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

VAESNE_API int64_t vaesne_mlp_head_bwd_workspace(int64_t M, int E) {
  if (M <= 0 || E != HE) return 0;
  return (int64_t)head_blocks(M) * HPART * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_mlp_head_bwd(const float* x, int64_t ldx, const float* h, int64_t ldh,
                                   const float* dy, int64_t M, int E, const float* W1,
                                   const float* b1, const float* W2, float* ds, float* g,
                                   float* dW2, float* db2, float* workspace,
                                   vaesne_colsum_list* defer, void* stream) {
  if (M <= 0) return 0;
  if (!head_args_ok(x, ldx, h, ldh, E) || !dy || !W1 || !b1 || !W2 || !ds || !g || !workspace ||
      (uintptr_t)ds % 16 || (uintptr_t)g % 16)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int G = head_blocks(M);
  hipLaunchKernelGGL(head_bwd_kernel, dim3((unsigned)G), dim3(HNT), 0, s, x, ldx, h, ldh, dy, M,
                     W1, b1, W2, ds, g, workspace);
  VAESNE_CHECK_LAUNCH();
  int rc = colsum_or_defer(defer, workspace, HPART, G, HE, dW2, 0, s);
  if (rc) return rc;
  return colsum_or_defer(defer, workspace + HE, HPART, G, 1, db2, 0, s);
}
