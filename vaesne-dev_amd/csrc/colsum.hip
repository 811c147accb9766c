// Deterministic partial-sum reduction shared by every weight / LayerNorm /
// embedding gradient (see common.h).
#include "common.h"

namespace vaesne {

__global__ void __launch_bounds__(1024) colsum_kernel(const float* __restrict__ P, int G, int F, int64_t ld,
                                                      float* __restrict__ out0,
                                                      float* __restrict__ out1, int split,
                                                      int accum) {
  __shared__ float red[16][65];
  const int fl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + fl;
  float s = 0.f;
  if (f < F) {
    int64_t g = sl;
    // 4 independent loads in flight per iteration; the sum order stays fixed
    for (; g + 48 < G; g += 64) {
      float a = P[g * ld + f], b = P[(g + 16) * ld + f];
      float c = P[(g + 32) * ld + f], d = P[(g + 48) * ld + f];
      s += a; s += b; s += c; s += d;
    }
    for (; g < G; g += 16) s += P[g * ld + f];
  }
  red[sl][fl] = s;
  __syncthreads();
  if (sl == 0 && f < F) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][fl];
    if (f < split) {
      if (out0) out0[f] = accum ? out0[f] + t : t;
    } else if (out1) {
      out1[f - split] = accum ? out1[f - split] + t : t;
    }
  }
}

int launch_colsum(const float* P, int G, int F, float* out0, float* out1, int split, int accum,
                  hipStream_t s) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((F + 63) / 64), dim3(1024), 0, s, P, G, F, (int64_t)F,
                     out0, out1, split, accum);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int launch_colsum_strided(const float* P, int G, int F, int64_t ld, float* out, hipStream_t s) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((F + 63) / 64), dim3(1024), 0, s, P, G, F, ld, out,
                     (float*)nullptr, F, 0);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

}  // namespace vaesne
