// Probe (not product): fill the LDS of every CU with a NaN pattern (one 160 KiB workgroup
// per CU slot), so a kernel launched next that reads LDS it never wrote sees NaN.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void lds_poison_kernel(uint32_t pattern, int words) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < words; i += blockDim.x) lds[i] = pattern;
  __syncthreads();
  if (lds[(threadIdx.x * 7) % words] != pattern) lds[0] = 0u;   // keep the stores
}

extern "C" int lds_poison(uint32_t pattern, int blocks, void* stream) {
  const int bytes = 160 * 1024;
  hipError_t e = hipFuncSetAttribute((const void*)lds_poison_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(1024), bytes, (hipStream_t)stream,
                     pattern, bytes / 4);
  return (int)hipGetLastError();
}
