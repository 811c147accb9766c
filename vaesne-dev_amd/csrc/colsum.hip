// Deterministic partial-sum reduction shared by every weight / LayerNorm /
// embedding gradient (see common.h), immediate or deferred to one batched
// launch per backward pass (vaesne_colsum_flush).
#include <cstdlib>

#include "common.h"

namespace vaesne {

// 4 adjacent columns f..f+3 of a [G][ld] partial block, 16 row slices per 1024-thread
// block (slice sl sums rows sl, sl + 16, ... in order; the slices are then summed in
// order): per column exactly colsum_kernel's summation order.  Thread sl == 0 returns
// the totals (others: unspecified).
__device__ __forceinline__ float4 colsum4(const float* __restrict__ P, int G, int F, int64_t ld,
                                          int f, float4 (*red4)[64]) {
  const int fl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (f < F) {
    int64_t g = sl;
    for (; g + 48 < G; g += 64) {
      const float4 a = *reinterpret_cast<const float4*>(P + g * ld + f);
      const float4 c = *reinterpret_cast<const float4*>(P + (g + 16) * ld + f);
      const float4 d = *reinterpret_cast<const float4*>(P + (g + 32) * ld + f);
      const float4 e = *reinterpret_cast<const float4*>(P + (g + 48) * ld + f);
      s.x += a.x; s.x += c.x; s.x += d.x; s.x += e.x;
      s.y += a.y; s.y += c.y; s.y += d.y; s.y += e.y;
      s.z += a.z; s.z += c.z; s.z += d.z; s.z += e.z;
      s.w += a.w; s.w += c.w; s.w += d.w; s.w += e.w;
    }
    for (; g < G; g += 16) {
      const float4 a = *reinterpret_cast<const float4*>(P + g * ld + f);
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red4[sl][fl] = s;
  __syncthreads();
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sl == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float4 r = red4[k][fl];
      t.x += r.x; t.y += r.y; t.z += r.z; t.w += r.w;
    }
  }
  return t;
}

// colsum_kernel with 4 columns per thread (F % 4 == 0, ld % 4 == 0, P 16-byte aligned)
__global__ void __launch_bounds__(1024) colsum4_kernel(const float* __restrict__ P, int G, int F,
                                                       int64_t ld, float* __restrict__ out0,
                                                       float* __restrict__ out1, int split,
                                                       int accum) {
  __shared__ float4 red4[16][64];
  const int f = blockIdx.x * 256 + (threadIdx.x & 63) * 4;
  const float4 t = colsum4(P, G, F, ld, f, red4);
  if ((threadIdx.x >> 6) == 0 && f < F) {
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int fc = f + c;
      if (fc < split) {
        if (out0) out0[fc] = accum ? out0[fc] + tv[c] : tv[c];
      } else if (out1) {
        out1[fc - split] = accum ? out1[fc - split] + tv[c] : tv[c];
      }
    }
  }
}

bool colsum_vec_ok(const float* P, int F, int64_t ld) {
  return ld % 4 == 0 && F % 4 == 0 && (uintptr_t)P % 16 == 0;
}

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
  if (colsum_vec_ok(P, F, F))
    hipLaunchKernelGGL(colsum4_kernel, dim3((F + 255) / 256), dim3(1024), 0, s, P, G, F,
                       (int64_t)F, out0, out1, split, accum);
  else
    hipLaunchKernelGGL(colsum_kernel, dim3((F + 63) / 64), dim3(1024), 0, s, P, G, F, (int64_t)F,
                       out0, out1, split, accum);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int launch_colsum_strided(const float* P, int G, int F, int64_t ld, float* out, hipStream_t s) {
  if (F <= 0) return 0;
  if (colsum_vec_ok(P, F, ld))
    hipLaunchKernelGGL(colsum4_kernel, dim3((F + 255) / 256), dim3(1024), 0, s, P, G, F, ld, out,
                       (float*)nullptr, F, 0);
  else
    hipLaunchKernelGGL(colsum_kernel, dim3((F + 63) / 64), dim3(1024), 0, s, P, G, F, ld, out,
                       (float*)nullptr, F, 0);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Batched column sums: up to CS_MAX independent (partials, ld, groups, cols,
// out, accum) sums in ONE launch; block b serves entry i with
// start[i] <= b < start[i + 1] (64 columns per block, the colsum_kernel body).
// ---------------------------------------------------------------------------
namespace {
constexpr int CS_MAX = 64;
struct ColsumBatch {
  const float* P[CS_MAX];
  float* out[CS_MAX];
  int64_t ld[CS_MAX];
  int G[CS_MAX];
  int F[CS_MAX];
  int accum[CS_MAX];
  int vec[CS_MAX];          // 4 columns per thread (16-byte aligned rows)
  int start[CS_MAX + 1];
  int count;
};

__global__ void __launch_bounds__(1024) colsum_batch_kernel(ColsumBatch b) {
  __shared__ float4 red4[16][64];
  int i = 0;
  while (i + 1 < b.count && (int)blockIdx.x >= b.start[i + 1]) ++i;
  const float* P = b.P[i];
  const int64_t ld = b.ld[i];
  const int G = b.G[i], F = b.F[i];
  const int fl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  if (b.vec[i]) {   // 4 adjacent columns per thread (16-byte row loads)
    const int f = ((int)blockIdx.x - b.start[i]) * 256 + fl * 4;
    const float4 t = colsum4(P, G, F, ld, f, red4);
    if (sl == 0 && f < F) {
      float* o = b.out[i] + f;
      const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) o[c] = b.accum[i] ? o[c] + tv[c] : tv[c];
    }
    return;
  }
  float (*red)[65] = reinterpret_cast<float (*)[65]>(&red4[0][0]);
  const int f = ((int)blockIdx.x - b.start[i]) * 64 + fl;
  float s = 0.f;
  if (f < F) {
    int64_t g = sl;
    for (; g + 48 < G; g += 64) {
      float a = P[g * ld + f], c = P[(g + 16) * ld + f];
      float d = P[(g + 32) * ld + f], e = P[(g + 48) * ld + f];
      s += a; s += c; s += d; s += e;
    }
    for (; g < G; g += 16) s += P[g * ld + f];
  }
  red[sl][fl] = s;
  __syncthreads();
  if (sl == 0 && f < F) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][fl];
    float* o = b.out[i] + f;
    *o = b.accum[i] ? *o + t : t;
  }
}

bool overlaps(const vaesne_colsum_entry& a, const vaesne_colsum_entry& c) {
  return a.out < c.out + c.cols && c.out < a.out + a.cols;
}
}  // namespace

int colsum_or_defer(vaesne_colsum_list* defer, const float* P, int64_t ld, int G, int F,
                    float* out, int accum, hipStream_t s) {
  if (F <= 0 || !out) return 0;
  if (defer) {
    if (defer->count >= defer->capacity || !defer->entries) return (int)hipErrorOutOfMemory;
    defer->entries[defer->count++] = vaesne_colsum_entry{P, ld, G, F, out, accum};
    return 0;
  }
  if (colsum_vec_ok(P, F, ld))
    hipLaunchKernelGGL(colsum4_kernel, dim3((F + 255) / 256), dim3(1024), 0, s, P, G, F, ld, out,
                       (float*)nullptr, F, accum);
  else
    hipLaunchKernelGGL(colsum_kernel, dim3((F + 63) / 64), dim3(1024), 0, s, P, G, F, ld, out,
                       (float*)nullptr, F, accum);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

}  // namespace vaesne

using namespace vaesne;

VAESNE_API int vaesne_colsum_flush(vaesne_colsum_list* list, void* stream) {
  if (!list || list->count <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  int i = 0;
  while (i < list->count) {
    ColsumBatch b{};
    int blocks = 0;
    while (i < list->count && b.count < CS_MAX) {
      const vaesne_colsum_entry& e = list->entries[i];
      bool clash = false;   // an output shared with an entry of this launch: next launch
      for (int j = 0; j < b.count && !clash; ++j)
        clash = overlaps(e, vaesne_colsum_entry{nullptr, 0, 0, b.F[j], b.out[j], 0});
      if (clash) break;
      if (e.cols > 0 && e.out) {
        b.P[b.count] = e.partial; b.out[b.count] = e.out; b.ld[b.count] = e.ld;
        b.G[b.count] = e.groups; b.F[b.count] = e.cols; b.accum[b.count] = e.accum;
        // cols % 4 == 0: the float4 at f < cols stays inside the row
        const int vec = colsum_vec_ok(e.partial, e.cols, e.ld);
        b.vec[b.count] = vec;
        b.start[b.count] = blocks;
        blocks += vec ? (e.cols + 255) / 256 : (e.cols + 63) / 64;
        ++b.count;
      }
      ++i;
    }
    b.start[b.count] = blocks;
    if (b.count > 0) {
      hipLaunchKernelGGL(colsum_batch_kernel, dim3(blocks), dim3(1024), 0, s, b);
      VAESNE_CHECK_LAUNCH();
    }
  }
  list->count = 0;
  return 0;
}
