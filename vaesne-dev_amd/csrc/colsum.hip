// Deterministic partial-sum reduction shared by every weight / LayerNorm /
// embedding gradient (see common.h), immediate or deferred to one batched
// launch per backward pass (vaesne_colsum_flush).
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
  int start[CS_MAX + 1];
  int count;
};

__global__ void __launch_bounds__(1024) colsum_batch_kernel(ColsumBatch b) {
  __shared__ float red[16][65];
  int i = 0;
  while (i + 1 < b.count && (int)blockIdx.x >= b.start[i + 1]) ++i;
  const float* P = b.P[i];
  const int64_t ld = b.ld[i];
  const int G = b.G[i], F = b.F[i];
  const int fl = threadIdx.x & 63, sl = threadIdx.x >> 6;
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
        b.start[b.count] = blocks;
        blocks += (e.cols + 63) / 64;
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
