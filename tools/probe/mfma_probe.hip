// Hardware probe (not product): the gfx950 operand maps this round's split-f16 attention
// kernels rely on, checked with exact integer-valued data.
//  * v_mfma_f32_16x16x32_f16: A lane l = A[l&15][8(l>>4)+j], B lane l = B[8(l>>4)+j][l&15],
//    D lane l = D[4(l>>4)+r][l&15]
//  * ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, cols 4p..4p+3 of a
//    4 x 16 block of 16-bit elements; lane i receives column i (row q in element q)
//  * hi/lo split: cvt_pk_f16_f32 + v_fma_mixlo/hi_f16
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

// A [16][32], B [32][16] row-major f16 -> D [16][16] f32 using the assumed maps
extern "C" __global__ void mfma_map(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x, r16 = l & 15, g = l >> 4;
  h8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r16 * 32 + 8 * g + j];
    b[j] = B[(8 * g + j) * 16 + r16];
  }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + r16] = d[r];
}

// M [R][16] 16-bit elements in LDS (row-major, 32 B rows); each 16-lane group g reads the
// block at rows 4g..4g+3: out[lane][0..3]
extern "C" __global__ void tr16_map(const short* M, short* out) {
  __shared__ __attribute__((aligned(16))) short s[16 * 16];
  const int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) s[i] = M[i];
  __syncthreads();
  const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
  const short* addr = s + (4 * g + q) * 16 + 4 * p;
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)addr);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

__device__ __forceinline__ uint32_t split_lo(float a, float b, uint32_t hi) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(r) : "v"(a), "v"(b), "v"(hi));
  return r;
}
extern "C" __global__ void split_k(const float* x, uint32_t* hi, uint32_t* lo, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * t + 1 >= n) return;
  const h2 h = __builtin_convertvector((f2){x[2 * t], x[2 * t + 1]}, h2);
  const uint32_t hb = __builtin_bit_cast(uint32_t, h);
  hi[t] = hb;
  lo[t] = split_lo(x[2 * t], x[2 * t + 1], hb);
}

extern "C" int probe_mfma(const void* A, const void* B, void* D, void* s) {
  hipLaunchKernelGGL(mfma_map, dim3(1), dim3(64), 0, (hipStream_t)s, (const _Float16*)A,
                     (const _Float16*)B, (float*)D);
  return (int)hipGetLastError();
}
extern "C" int probe_tr16(const void* M, void* out, void* s) {
  hipLaunchKernelGGL(tr16_map, dim3(1), dim3(64), 0, (hipStream_t)s, (const short*)M, (short*)out);
  return (int)hipGetLastError();
}
extern "C" int probe_split(const void* x, void* hi, void* lo, int n, void* s) {
  hipLaunchKernelGGL(split_k, dim3((n / 2 + 255) / 256), dim3(256), 0, (hipStream_t)s,
                     (const float*)x, (uint32_t*)hi, (uint32_t*)lo, n);
  return (int)hipGetLastError();
}

// raw fragments: Af/Bf [64 lanes][8] f16, Df [64][4] f32 (no layout assumption)
extern "C" __global__ void mfma_raw(const _Float16* Af, const _Float16* Bf, float* Df, int bf) {
  const int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = Af[l * 8 + j]; b[j] = Bf[l * 8 + j]; }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) Df[l * 4 + r] = d[r];
}
extern "C" int probe_raw(const void* A, const void* B, void* D, void* s) {
  hipLaunchKernelGGL(mfma_raw, dim3(1), dim3(64), 0, (hipStream_t)s, (const _Float16*)A,
                     (const _Float16*)B, (float*)D, 0);
  return (int)hipGetLastError();
}
