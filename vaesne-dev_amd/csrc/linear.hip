// Token-wise linear layers (nn.Linear on [*, K] -> [*, N]) for the VAESNe
// transformer stacks: in-projections (32->96), out-projections and FFN
// (32->32), the MLP heads (32->32->1 / Dz) and the embedding MLPs (64->32,
// 96->32).  Reference: torch.nn.Linear as used throughout
// package/VAESNe/util_layers.py:9-34,131-149,257-309.
//
// Forward / backward-data kernel (one kernel, two weight orientations):
//   out[r, n] = (accum ? out[r, n] : 0) + bias[n] + sum_k in[r, k] * Wt[n, k]
//   in[r, k]  = (a[r, k] + a2[r, k]) * (act_in_grad ? act'(zin[r, k]) : 1)
//   optional activation on the way out (relu / exact-erf gelu), pre-activation
//   optionally stored for the backward.
// Geometry: 256-thread workgroup = 4 waves; a 64-row tile puts one row on each
// lane; wave w owns the contiguous output columns [w*C, (w+1)*C).  The weight
// (<= 128 x 128 fp32) sits in LDS once per workgroup and is read as broadcast
// float4s; workgroups walk row tiles with a grid stride.
//
// Backward-weight kernel: dW[o, i] = sum_r dz[r, o] x[r, i], db[o] = sum_r dz[r, o]
// with dz = dy * act'(z) recomputed on the fly; per-workgroup partial sums in a
// workspace, then a fixed-order reduction (bitwise reproducible).
#include "common.h"

using namespace vaesne;

namespace {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

struct LinArgs {
  const float* a; int64_t lda;
  const float* a2; int64_t lda2;
  const float* zin; int64_t ldzin; int act_in_grad;
  const float* W; int w_trans; const float* bias;
  int K; int N; int64_t M;
  float* out; int64_t ldo; int accum; int act_out;
  float* zout; int64_t ldzo;
};

__device__ __forceinline__ float act_fwd(int act, float v) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_GELU) return gelu_erf(v);
  return v;
}
__device__ __forceinline__ float act_grad(int act, float z) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_GELU) return gelu_erf_grad(z);
  return 1.f;
}

constexpr int ROWS = 64;
constexpr int NT = 256;
constexpr int MAXK = 128;
constexpr int MAXN = 128;

template <int C, bool VEC>
__global__ __launch_bounds__(NT) void linear_kernel(LinArgs p) {
  __shared__ float4 Ws4[MAXN * (MAXK / 4)];
  const int KP = (p.K + 3) & ~3;
  const int KP4 = KP >> 2;
  float* Ws = reinterpret_cast<float*>(Ws4);
  // stage Wt[n][k] (zero padded in k)
  for (int idx = threadIdx.x; idx < p.N * KP; idx += NT) {
    int n = idx / KP, k = idx - n * KP;
    float w = 0.f;
    if (k < p.K) w = p.w_trans ? p.W[(int64_t)k * p.N + n] : p.W[(int64_t)n * p.K + k];
    Ws[idx] = w;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n0 = wave * C;
  if (n0 >= p.N) return;  // no barrier after this point
  const int nc = min(C, p.N - n0);
  float bias[C];
#pragma unroll
  for (int c = 0; c < C; ++c) bias[c] = (p.bias && c < nc) ? p.bias[n0 + c] : 0.f;

  const int64_t tiles = (p.M + ROWS - 1) / ROWS;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t r = t * ROWS + lane;
    if (r >= p.M) continue;
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = bias[c];
    const float* arow = p.a + r * p.lda;
    const float* a2row = p.a2 ? p.a2 + r * p.lda2 : nullptr;
    const float* zrow = p.act_in_grad ? p.zin + r * p.ldzin : nullptr;
    for (int k4 = 0; k4 < KP4; ++k4) {
      float4 xv;
      if (VEC) {
        xv = *reinterpret_cast<const float4*>(arow + 4 * k4);
        if (a2row) {
          float4 x2 = *reinterpret_cast<const float4*>(a2row + 4 * k4);
          xv.x += x2.x; xv.y += x2.y; xv.z += x2.z; xv.w += x2.w;
        }
        if (zrow) {
          float4 zv = *reinterpret_cast<const float4*>(zrow + 4 * k4);
          xv.x *= act_grad(p.act_in_grad, zv.x); xv.y *= act_grad(p.act_in_grad, zv.y);
          xv.z *= act_grad(p.act_in_grad, zv.z); xv.w *= act_grad(p.act_in_grad, zv.w);
        }
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int k = 4 * k4 + j;
          float v = 0.f;
          if (k < p.K) {
            v = arow[k];
            if (a2row) v += a2row[k];
            if (zrow) v *= act_grad(p.act_in_grad, zrow[k]);
          }
          e[j] = v;
        }
        xv = make_float4(e[0], e[1], e[2], e[3]);
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (c < nc) {
          float4 w = Ws4[(n0 + c) * KP4 + k4];
          acc[c] = fmaf(xv.x, w.x, acc[c]);
          acc[c] = fmaf(xv.y, w.y, acc[c]);
          acc[c] = fmaf(xv.z, w.z, acc[c]);
          acc[c] = fmaf(xv.w, w.w, acc[c]);
        }
      }
    }
    float* orow = p.out + r * p.ldo + n0;
    float* zorow = p.zout ? p.zout + r * p.ldzo + n0 : nullptr;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (c < nc) {
        float v = acc[c];
        if (p.accum) v += orow[c];
        if (zorow) zorow[c] = v;
        orow[c] = act_fwd(p.act_out, v);
      }
    }
  }
}

template <int C>
int launch_linear_c(const LinArgs& p, hipStream_t s) {
  int64_t tiles = (p.M + ROWS - 1) / ROWS;
  int grid = (int)(tiles < 2048 ? tiles : 2048);
  if (grid < 1) return 0;
  bool vec = (p.K % 4 == 0) && (p.lda % 4 == 0) && ((uintptr_t)p.a % 16 == 0) &&
             (!p.a2 || ((p.lda2 % 4 == 0) && ((uintptr_t)p.a2 % 16 == 0))) &&
             (!p.act_in_grad || ((p.ldzin % 4 == 0) && ((uintptr_t)p.zin % 16 == 0)));
  if (vec)
    hipLaunchKernelGGL((linear_kernel<C, true>), dim3(grid), dim3(NT), 0, s, p);
  else
    hipLaunchKernelGGL((linear_kernel<C, false>), dim3(grid), dim3(NT), 0, s, p);
  VAESNE_CHECK_LAUNCH();
  return 0;
}

int launch_linear(const LinArgs& p, hipStream_t s) {
  if (p.K < 1 || p.K > MAXK || p.N < 1 || p.N > MAXN) return (int)hipErrorInvalidValue;
  if (p.M <= 0) return 0;
  int c = (p.N + 3) / 4;
  if (c <= 1) return launch_linear_c<1>(p, s);
  if (c <= 2) return launch_linear_c<2>(p, s);
  if (c <= 4) return launch_linear_c<4>(p, s);
  if (c <= 8) return launch_linear_c<8>(p, s);
  if (c <= 16) return launch_linear_c<16>(p, s);
  if (c <= 24) return launch_linear_c<24>(p, s);
  return launch_linear_c<32>(p, s);
}

// ---------------------------------------------------------------------------
// backward weight
// ---------------------------------------------------------------------------
struct WgtArgs {
  const float* dy; int64_t lddy;
  const float* z; int64_t ldz; int act;  // dz = dy * act'(z)
  const float* x; int64_t ldx;
  const float* x2; int64_t ldx2;         // x := x + x2
  int64_t M; int O; int I;
  float* partial;                        // [gridDim][O*(I+1)]
};

constexpr int WROWS = 64;

template <int E>
__global__ __launch_bounds__(NT) void linear_wgrad_kernel(WgtArgs p) {
  __shared__ float Dz[WROWS * MAXN];
  __shared__ float Xs[WROWS * (MAXK + 1)];
  const int I1 = p.I + 1;
  const int F = p.O * I1;
  float acc[E];
  int fo[E], fi[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc[e] = 0.f;
    int f = threadIdx.x + NT * e;
    fo[e] = f < F ? f / I1 : 0;
    fi[e] = f < F ? f - fo[e] * I1 : 0;
  }
  const int64_t tiles = (p.M + WROWS - 1) / WROWS;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t r0 = t * WROWS;
    const int nr = (int)min((int64_t)WROWS, p.M - r0);
    __syncthreads();
    for (int idx = threadIdx.x; idx < WROWS * p.O; idx += NT) {
      int rr = idx / p.O, o = idx - rr * p.O;
      float v = 0.f;
      if (rr < nr) {
        int64_t r = r0 + rr;
        v = p.dy[r * p.lddy + o];
        if (p.act) v *= act_grad(p.act, p.z[r * p.ldz + o]);
      }
      Dz[rr * p.O + o] = v;
    }
    for (int idx = threadIdx.x; idx < WROWS * I1; idx += NT) {
      int rr = idx / I1, i = idx - rr * I1;
      float v = 0.f;
      if (rr < nr) {
        int64_t r = r0 + rr;
        if (i < p.I) {
          v = p.x[r * p.ldx + i];
          if (p.x2) v += p.x2[r * p.ldx2 + i];
        } else {
          v = 1.f;
        }
      }
      Xs[rr * I1 + i] = v;
    }
    __syncthreads();
    for (int rr = 0; rr < nr; ++rr) {
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = fmaf(Dz[rr * p.O + fo[e]], Xs[rr * I1 + fi[e]], acc[e]);
    }
  }
  // partial layout [G][O*I (dW) | O (db)] so one column-sum splits at O*I
  float* out = p.partial + (int64_t)blockIdx.x * F;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    int f = threadIdx.x + NT * e;
    if (f < F) out[fi[e] < p.I ? fo[e] * p.I + fi[e] : p.O * p.I + fo[e]] = acc[e];
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
VAESNE_API int vaesne_linear_fwd(const float* x, int64_t ldx, const float* x2, int64_t ldx2,
                                 int64_t M, int K, const float* W, const float* b, int N,
                                 float* y, int64_t ldy, float* z, int64_t ldz, int act,
                                 int accum, void* stream) {
  LinArgs p{};
  p.a = x; p.lda = ldx; p.a2 = x2; p.lda2 = ldx2;
  p.zin = nullptr; p.ldzin = 0; p.act_in_grad = 0;
  p.W = W; p.w_trans = 0; p.bias = b;
  p.K = K; p.N = N; p.M = M;
  p.out = y; p.ldo = ldy; p.accum = accum; p.act_out = act;
  p.zout = z; p.ldzo = ldz;
  return launch_linear(p, (hipStream_t)stream);
}

VAESNE_API int vaesne_linear_bwd_data(const float* dy, int64_t lddy, const float* z, int64_t ldz,
                                      int act, int64_t M, int N, const float* W, int K,
                                      float* dx, int64_t lddx, int accum, void* stream) {
  // dx[M, K] (+)= (dy * act'(z))[M, N] @ W[N, K]
  LinArgs p{};
  p.a = dy; p.lda = lddy; p.a2 = nullptr; p.lda2 = 0;
  p.zin = act ? z : nullptr; p.ldzin = ldz; p.act_in_grad = act;
  p.W = W; p.w_trans = 1; p.bias = nullptr;
  p.K = N; p.N = K; p.M = M;
  p.out = dx; p.ldo = lddx; p.accum = accum; p.act_out = ACT_NONE;
  p.zout = nullptr; p.ldzo = 0;
  return launch_linear(p, (hipStream_t)stream);
}

VAESNE_API int64_t vaesne_linear_bwd_weight_workspace(int64_t M, int O, int I) {
  int64_t tiles = (M + WROWS - 1) / WROWS;
  int64_t g = tiles < 512 ? tiles : 512;
  if (g < 1) g = 1;
  return g * (int64_t)O * (I + 1) * (int64_t)sizeof(float);
}

VAESNE_API int vaesne_linear_bwd_weight(const float* dy, int64_t lddy, const float* z, int64_t ldz,
                                        int act, const float* x, int64_t ldx, const float* x2,
                                        int64_t ldx2, int64_t M, int O, int I, float* dW,
                                        float* db, int accum, float* workspace, void* stream) {
  if (O < 1 || O > MAXN || I < 1 || I > MAXK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  int64_t tiles = (M + WROWS - 1) / WROWS;
  int G = (int)(tiles < 512 ? tiles : 512);
  const int F = O * (I + 1);
  if (G < 1) {
    // empty batch: gradient is zero
    G = 1;
    hipError_t me = hipMemsetAsync(workspace, 0, sizeof(float) * F, s);
    if (me != hipSuccess) return (int)me;
  } else {
    WgtArgs p{dy, lddy, z, ldz, act, x, ldx, x2, ldx2, M, O, I, workspace};
    int e = (F + NT - 1) / NT;
    if (e <= 4)
      hipLaunchKernelGGL(linear_wgrad_kernel<4>, dim3(G), dim3(NT), 0, s, p);
    else if (e <= 8)
      hipLaunchKernelGGL(linear_wgrad_kernel<8>, dim3(G), dim3(NT), 0, s, p);
    else if (e <= 16)
      hipLaunchKernelGGL(linear_wgrad_kernel<16>, dim3(G), dim3(NT), 0, s, p);
    else if (e <= 40)
      hipLaunchKernelGGL(linear_wgrad_kernel<40>, dim3(G), dim3(NT), 0, s, p);
    else
      return (int)hipErrorInvalidValue;
    VAESNE_CHECK_LAUNCH();
  }
  return launch_colsum(workspace, G, F, dW, db, O * I, accum, s);
}
