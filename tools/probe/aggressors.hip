// Probe (not product): minimal kernels that each exercise one instruction class of the
// split-f16 attention kernels, launched beside another kernel to see which class (if any)
// disturbs it: f16 MFMA 16x16x32, f32 -> f16 packed conversions, permlane swaps, exp.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

extern "C" __global__ void agg_mfma(float* out, int iters) {
  h8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(0.5f); }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  if (c[0] == 12345.f) out[threadIdx.x] = c[1];
}
extern "C" __global__ void agg_mfma_all(float* out, int iters) {
  h8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f + i); b[i] = (_Float16)(0.5f); }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  if ((c[0] + c[1]) + (c[2] + c[3]) == 12345.f) out[threadIdx.x] = c[1];
}
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
extern "C" __global__ void agg_mfma_kind(float* out, int iters, int kind) {
  f4 c = {0.f, 0.f, 0.f, 0.f};
  f16v c16 = {};
  const float t = threadIdx.x * 0.001f;
  if (kind == 0) {          // bf16 16x16x32
    b8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(t + i); b[i] = (__bf16)0.5f; }
    for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  } else if (kind == 1) {   // f16 16x16x16 (the CDNA3 shape)
    h4 a, b;
    for (int i = 0; i < 4; ++i) { a[i] = (_Float16)(t + i); b[i] = (_Float16)0.5f; }
    for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  } else if (kind == 2) {   // f32 16x16x4
    for (int it = 0; it < iters; ++it) c = __builtin_amdgcn_mfma_f32_16x16x4f32(t, 0.5f, c, 0, 0, 0);
  } else {                  // f32 32x32x2 (the decoder-tail kernels' shape)
    for (int it = 0; it < iters; ++it) c16 = __builtin_amdgcn_mfma_f32_32x32x2f32(t, 0.5f, c16, 0, 0, 0);
    c[0] = c16[0] + c16[15];
  }
  if ((c[0] + c[1]) + (c[2] + c[3]) == 12345.f) out[threadIdx.x] = c[1];
}
extern "C" __global__ void agg_cvt(float* out, int iters) {
  float x = threadIdx.x * 0.37f, y = 1.5f;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    const h2v h = __builtin_convertvector((f2v){x, y}, h2v);
    acc ^= __builtin_bit_cast(uint32_t, h);
    x += 0.25f;
  }
  if (acc == 7u) out[threadIdx.x] = x;
}
extern "C" __global__ void agg_perm(float* out, int iters) {
  uint32_t v = threadIdx.x, w = threadIdx.x * 3;
  for (int it = 0; it < iters; ++it) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, w, false, false);
    v = r[0] + 1; w = r[1];
    const auto q = __builtin_amdgcn_permlane16_swap(v, w, false, false);
    v = q[0]; w = q[1] + 1;
  }
  if (v == 7u) out[threadIdx.x] = (float)w;
}
extern "C" __global__ void agg_exp(float* out, int iters) {
  float x = threadIdx.x * 1e-3f;
  for (int it = 0; it < iters; ++it) x = __builtin_amdgcn_exp2f(x * 0.5f) - 1.f;
  if (x == 12345.f) out[threadIdx.x] = x;
}

extern "C" int agg_launch(int which, float* out, int blocks, int iters, void* stream) {
  const dim3 g(blocks), b(256);
  hipStream_t s = (hipStream_t)stream;
  switch (which) {
    case 0: hipLaunchKernelGGL(agg_mfma, g, b, 0, s, out, iters); break;
    case 1: hipLaunchKernelGGL(agg_cvt, g, b, 0, s, out, iters); break;
    case 2: hipLaunchKernelGGL(agg_perm, g, b, 0, s, out, iters); break;
    case 3: hipLaunchKernelGGL(agg_exp, g, b, 0, s, out, iters); break;
    case 4: hipLaunchKernelGGL(agg_mfma_all, g, b, 0, s, out, iters); break;
    default: hipLaunchKernelGGL(agg_mfma_kind, g, b, 0, s, out, iters, which - 5); break;
  }
  return (int)hipGetLastError();
}

// ---- victims: a chain of fp32 FMAs whose exact result is known (small integers) ----
typedef float f2 __attribute__((ext_vector_type(2)));
// mode 0: scalar v_fma_f32; 1: compiler-generated packed f32 (v_pk_fma_f32); 2: inline-asm
// v_pk_fma_f32 with op_sel broadcast (the packed-VALU attention kernels' form)
extern "C" __global__ void victim(int mode, int iters, int* bad) {
  int wrong = 0;
  if (mode == 0) {
    float acc = 0.f, a = 1.f, b = (float)(threadIdx.x & 7);
    for (int it = 0; it < iters; ++it) acc = __builtin_fmaf(a, b, acc);
    wrong = acc != (float)iters * (float)(threadIdx.x & 7);
  } else if (mode == 1) {
    f2 acc = {0.f, 0.f}, a = {1.f, 2.f}, b = {(float)(threadIdx.x & 7), 1.f};
    for (int it = 0; it < iters; ++it) acc = __builtin_elementwise_fma(a, b, acc);
    wrong = acc.x != (float)iters * (float)(threadIdx.x & 7) || acc.y != 2.f * iters;
  } else if (mode == 4 || mode == 5) {
    // LDS round trips: rows of known values read back with ds_read_b128 and summed
    __shared__ __attribute__((aligned(16))) float buf[64 * 8];
    for (int i = threadIdx.x; i < 64 * 8; i += blockDim.x) buf[i] = (float)(i & 15);
    __syncthreads();
    float acc = 0.f;
    f2 pacc = {0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
      const float4 r = *reinterpret_cast<const float4*>(buf + ((it * 8 + threadIdx.x) & 63) * 8);
      if (mode == 4) acc += (r.x + r.y) + (r.z + r.w);
      else asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(pacc) : "v"((f2){r.x + r.y, r.z + r.w}), "v"((f2){1.f, 1.f}));
    }
    // row k holds 8k..8k+7 & 15: sum of its first four = (8k&15)*4 + 6
    float e = 0.f;
    for (int it = 0; it < iters; ++it) { const int k = (it * 8 + threadIdx.x) & 63; e += (float)((8 * k) & 15) * 4.f + 6.f; }
    wrong = mode == 4 ? acc != e : (pacc.x + pacc.y) != e;
  } else if (mode == 6) {
    // op_sel [0,1,0] op_sel_hi [1,1,1]: b's HIGH half broadcast
    f2 acc = {0.f, 0.f}, a = {1.f, 2.f}, b = {1.f, (float)(threadIdx.x & 7)};
    for (int it = 0; it < iters; ++it)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(a), "v"(b));
    const float e = (float)iters * (float)(threadIdx.x & 7);
    wrong = acc.x != e || acc.y != 2.f * e;
  } else if (mode == 9 || mode == 10) {
    // as 6 with padding between the dependent FMAs (9: s_nop 4 before each), or with no
    // dependence between consecutive FMAs (10: four independent accumulators)
    f2 a = {1.f, 2.f}, b = {1.f, (float)(threadIdx.x & 7)};
    if (mode == 9) {
      f2 acc = {0.f, 0.f};
      for (int it = 0; it < iters; ++it)
        asm volatile("s_nop 4\nv_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]\ns_nop 4" : "+v"(acc) : "v"(a), "v"(b));
      const float e = (float)iters * (float)(threadIdx.x & 7);
      wrong = acc.x != e || acc.y != 2.f * e;
    } else {
      f2 c0 = {0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
      for (int it = 0; it < iters; it += 4)
        asm volatile("v_pk_fma_f32 %0, %4, %5, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]\n"
                     "v_pk_fma_f32 %1, %4, %5, %1 op_sel:[0,1,0] op_sel_hi:[1,1,1]\n"
                     "v_pk_fma_f32 %2, %4, %5, %2 op_sel:[0,1,0] op_sel_hi:[1,1,1]\n"
                     "v_pk_fma_f32 %3, %4, %5, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]"
                     : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b));
      const float e = (float)(iters / 4) * (float)(threadIdx.x & 7);
      wrong = c0.x != e || c3.x != e || c1.y != 2.f * e || c2.y != 2.f * e;
    }
  } else if (mode == 11 || mode == 12) {
    f2 acc = {0.f, 0.f}, b = {1.f, (float)(threadIdx.x & 7)};
    for (int it = 0; it < iters; ++it) {
      f2 t;
      if (mode == 11)
        asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(t) : "v"((f2){0.f, 0.f}), "v"(b));
      else
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(t) : "v"((f2){1.f, 1.f}), "v"(b));
      acc += t;
    }
    const float e = (float)iters * (float)(threadIdx.x & 7);
    wrong = acc.x != e || acc.y != e;
  } else if (mode == 13) {
    // SGPR pair source, low lane reads its high half (hipcc's scalar-broadcast multiply)
    const float hv = (float)__builtin_amdgcn_readfirstlane(iters & 7) + 1.f;    // uniform
    const f2 sp = {0.f, hv};
    f2 acc = {0.f, 0.f};
    const f2 b = {(float)(threadIdx.x & 7), (float)(threadIdx.x & 7)};
    for (int it = 0; it < iters; ++it) {
      f2 t;
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(t) : "s"(sp), "v"(b));
      acc += t;
    }
    const float e = (float)iters * hv * (float)(threadIdx.x & 7);
    wrong = acc.x != e || acc.y != e;
  } else if (mode == 14) {
    // v_pk_mov_b32 moving a VGPR pair's high half into the low lane (hipcc's shuffles)
    f2 src = {0.f, (float)(threadIdx.x & 7)};
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
      f2 t;
      asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]" : "=v"(t) : "v"(src));
      acc += t.x;
    }
    wrong = acc != (float)iters * (float)(threadIdx.x & 7);
  } else if (mode == 7) {
    // compiler packed mul / add with neg modifiers (the kernels' exp-argument / max paths)
    f2 acc = {0.f, 0.f}, m = {3.f, 5.f};
    const f2 one = {1.f, 1.f};
    for (int it = 0; it < iters; ++it) {
      f2 t = (m - one) * one;      // {2, 4}
      acc = acc + (t - (f2){1.f, 3.f});   // {1, 1}
      m = m + (f2){0.f, 0.f};
    }
    wrong = acc.x != (float)iters || acc.y != (float)iters;
  } else if (mode == 8) {
    // 64-bit moves (v_mov_b64) of pairs and max3
    double d = (double)(threadIdx.x & 7);
    float mx = -1e30f, acc = 0.f;
    for (int it = 0; it < iters; ++it) {
      volatile double e = d;
      const double f = e;
      mx = fmaxf(fmaxf(mx, (float)f), (float)(it & 3));
      acc += (float)f;
    }
    wrong = acc != (float)iters * (float)(threadIdx.x & 7);
  } else if (mode == 3) {
    // two dependent chains interleaved in one statement: each chain's next FMA one
    // instruction after its last (the packed-VALU attention kernels' qk_chains2 form)
    f2 x = {0.f, 0.f}, y = {0.f, 0.f}, a = {1.f, 2.f}, b = {(float)(threadIdx.x & 7), 1.f};
    for (int it = 0; it < iters; it += 4)
      asm volatile("v_pk_fma_f32 %0, %2, %3, %0 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %1, %2, %3, %1 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %0, %2, %3, %0 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %1, %2, %3, %1 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %0, %2, %3, %0 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %1, %2, %3, %1 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %0, %2, %3, %0 op_sel_hi:[1,0,1]\n"
                   "v_pk_fma_f32 %1, %2, %3, %1 op_sel_hi:[1,0,1]"
                   : "+v"(x), "+v"(y) : "v"(a), "v"(b));
    const float e = (float)iters * (float)(threadIdx.x & 7);
    wrong = x.x != e || y.x != e || x.y != 2.f * e || y.y != 2.f * e;
  } else {
    f2 acc = {0.f, 0.f}, a = {1.f, 2.f}, b = {(float)(threadIdx.x & 7), 1.f};
    for (int it = 0; it < iters; ++it)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(a), "v"(b));
    // op_sel_hi [1,0,1]: b's low half broadcast -> acc += a * b.x
    wrong = acc.x != (float)iters * (float)(threadIdx.x & 7) || acc.y != 2.f * iters * (float)(threadIdx.x & 7);
  }
  if (wrong) atomicAdd(bad, 1);
}
extern "C" int victim_launch(int mode, int blocks, int iters, int* bad, void* stream) {
  hipLaunchKernelGGL(victim, dim3(blocks), dim3(256), 0, (hipStream_t)stream, mode, iters, bad);
  return (int)hipGetLastError();
}
