// Fused small-batch Linear kernels for the generic engine (fp32): the engine's "kernel injection"
// (`"amd": {"fused_linear": true}`) swaps nn.Linear (+ a following nn.ReLU) for one forward
// launch and ONE backward launch per layer, in place of autograd's addmm + relu forward and
// mm / mm / sum / threshold_backward backward.  At the reference's shapes
// (batch 4, 20 -> 64 -> 1) every one of those is a sub-microsecond kernel whose cost is its
// launch or its graph node; the win is the node count, so the kernels are plain one-output-per-
// thread dot products (exact fp32 FMA chains, no MFMA tiling: there is nothing to tile).
// Reference: train.py:29-33 (Linear / ReLU / Linear), 107 (forward), 113 (backward).
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

// y[m][n] = act(b[n] + sum_k x[m][k] W[n][k])
__global__ __launch_bounds__(256) void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                          const float* __restrict__ b, float* __restrict__ y, int M,
                                                          int N, int K, int relu) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i % N;
  const float* xr = x + (long long)m * K;
  const float* wr = W + (long long)n * K;
  float acc = 0.f;
  int k = 0;
  if ((K & 3) == 0) {
    for (; k < K; k += 4) {
      const float4 xv = *reinterpret_cast<const float4*>(xr + k);
      const float4 wv = *reinterpret_cast<const float4*>(wr + k);
      acc = fmaf(xv.x, wv.x, acc);
      acc = fmaf(xv.y, wv.y, acc);
      acc = fmaf(xv.z, wv.z, acc);
      acc = fmaf(xv.w, wv.w, acc);
    }
  }
  for (; k < K; ++k) acc = fmaf(xr[k], wr[k], acc);
  float v = acc + (b ? b[n] : 0.f);
  if (relu) v = fmaxf(v, 0.f);
  y[i] = v;
}

// g = dy * 1[y > 0] (relu) or dy.  One launch, three thread ranges:
//   [0, N*K)            dW[n][k] (+)= sum_m g[m][n] x[m][k]
//   [N*K, N*K+N)        db[n]    (+)= sum_m g[m][n]               (if db)
// accumulate: add into dW / db (they are the parameters' .grad views into the engine's flat bucket)
//   [.., + M*K)         dx[m][k] = sum_n g[m][n] W[n][k]         (if dx)
__global__ __launch_bounds__(256) void linear_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          const float* __restrict__ W, const float* __restrict__ y,
                                                          float* __restrict__ dx, float* __restrict__ dW,
                                                          float* __restrict__ db, int M, int N, int K,
                                                          int accumulate) {
  int i = blockIdx.x * 256 + threadIdx.x;
  auto g = [&](int m, int n) {
    const float d = dy[(long long)m * N + n];
    return (y && !(y[(long long)m * N + n] > 0.f)) ? 0.f : d;
  };
  if (i < N * K) {
    const int n = i / K, k = i % K;
    float acc = 0.f;
    for (int m = 0; m < M; ++m) acc = fmaf(g(m, n), x[(long long)m * K + k], acc);
    dW[i] = accumulate ? dW[i] + acc : acc;
    return;
  }
  i -= N * K;
  if (db) {
    if (i < N) {
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc += g(m, i);
      db[i] = accumulate ? db[i] + acc : acc;
      return;
    }
    i -= N;
  }
  if (dx && i < M * K) {
    const int m = i / K, k = i % K;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc = fmaf(g(m, n), W[(long long)n * K + k], acc);
    dx[i] = acc;
  }
}

hipError_t linear_fwd(const float* x, const float* W, const float* b, float* y, int M, int N, int K, bool relu,
                      hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  const long long total = (long long)M * N;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, W, b, y, M,
                     N, K, relu ? 1 : 0);
  return hipGetLastError();
}

hipError_t linear_bwd(const float* dy, const float* x, const float* W, const float* y, float* dx, float* dW,
                      float* db, int M, int N, int K, bool accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipErrorInvalidValue;
  const long long total = (long long)N * K + (db ? N : 0) + (dx ? (long long)M * K : 0);
  hipLaunchKernelGGL(linear_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, dy, x, W, y,
                     dx, dW, db, M, N, K, accumulate ? 1 : 0);
  return hipGetLastError();
}

}  // namespace dgt
