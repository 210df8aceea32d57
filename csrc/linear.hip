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

// ---------------------------------------------------------------- two-layer chains in one launch
// The reference model is exactly two Linear layers (train.py:29-33): at its shapes each layer's
// kernel is sub-microsecond and the step pays per launch (eager) or per graph node.  One workgroup
// runs both layers: the hidden activation goes to global memory (the backward's saved input) and to
// LDS for the second layer.  Every output is the same fmaf chain in the same order as the per-layer
// kernels above, so the chain is bitwise the per-layer path.
constexpr int kChain2MaxHidden = 4096;  // M * H floats of the hidden activation / gradient in LDS
constexpr int kChain2StageW2 = 4096;    // O * H floats of W2 staged in LDS by the forward

// h = act1(x W1^T + b1) [M, H]; y = act2(h W2^T + b2) [M, O]
__global__ __launch_bounds__(256) void linear2_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W1,
                                                           const float* __restrict__ b1, const float* __restrict__ W2,
                                                           const float* __restrict__ b2, float* __restrict__ h,
                                                           float* __restrict__ y, int M, int K, int H, int O,
                                                           int relu1, int relu2) {
  __shared__ float hs[kChain2MaxHidden];
  __shared__ float w2s[kChain2StageW2];
  // layer 2's few dot products each walk a whole W2 row in a dependent fma chain: read from global
  // memory that chain waits on a batch of loads every few steps (~5 of the kernel's ~10 us in a
  // graph-replayed step); staged into LDS by all 256 threads at once (same products, same order)
  const bool stage = O * H <= kChain2StageW2;
  if (stage)
    for (int i = threadIdx.x; i < O * H; i += 256) w2s[i] = W2[i];
  for (int i = threadIdx.x; i < M * H; i += 256) {
    const int m = i / H, n = i % H;
    const float* xr = x + (long long)m * K;
    const float* wr = W1 + (long long)n * K;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc = fmaf(xr[k], wr[k], acc);
    float v = acc + (b1 ? b1[n] : 0.f);
    if (relu1) v = fmaxf(v, 0.f);
    hs[i] = v;
    h[i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < M * O; i += 256) {
    const int m = i / O, o = i % O;
    const float* hr = hs + m * H;
    float acc = 0.f;
    if (stage) {  // (separate loops: both operands as LDS reads, not flat loads)
      const float* wr = w2s + o * H;
      for (int k = 0; k < H; ++k) acc = fmaf(hr[k], wr[k], acc);
    } else {
      const float* wr = W2 + (long long)o * H;
      for (int k = 0; k < H; ++k) acc = fmaf(hr[k], wr[k], acc);
    }
    float v = acc + (b2 ? b2[o] : 0.f);
    if (relu2) v = fmaxf(v, 0.f);
    y[i] = v;
  }
}

// Backward of the chain above from dy [M, O]: g2 = dy * 1[y > 0] (relu2) or dy; dW2 (+)= g2^T h,
// db2 (+)= sum_m g2, dh = g2 W2 (LDS); g1 = dh * 1[h > 0] (relu1) or dh; dW1 (+)= g1^T x,
// db1 (+)= sum_m g1, dx = g1 W1 (optional).  acc1 / acc2: accumulate into layer 1's / 2's grads.
__global__ __launch_bounds__(256) void linear2_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ W1,
    const float* __restrict__ h, const float* __restrict__ W2, const float* __restrict__ y, float* __restrict__ dx,
    float* __restrict__ dW1, float* __restrict__ db1, float* __restrict__ dW2, float* __restrict__ db2, int M, int K,
    int H, int O, int relu1, int acc1, int acc2) {
  __shared__ float dhs[kChain2MaxHidden];
  auto g2 = [&](int m, int o) {
    const float d = dy[(long long)m * O + o];
    return (y && !(y[(long long)m * O + o] > 0.f)) ? 0.f : d;
  };
  // layer 2: dW2 [O, H], db2 [O], dh [M, H]
  for (int i = threadIdx.x; i < O * H + (db2 ? O : 0) + M * H; i += 256) {
    if (i < O * H) {
      const int o = i / H, n = i % H;
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc = fmaf(g2(m, o), h[(long long)m * H + n], acc);
      dW2[i] = acc2 ? dW2[i] + acc : acc;
    } else if (db2 && i < O * H + O) {
      const int o = i - O * H;
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc += g2(m, o);
      db2[o] = acc2 ? db2[o] + acc : acc;
    } else {
      const int j = i - O * H - (db2 ? O : 0), m = j / H, n = j % H;
      float acc = 0.f;
      for (int o = 0; o < O; ++o) acc = fmaf(g2(m, o), W2[(long long)o * H + n], acc);
      dhs[j] = (relu1 && !(h[j] > 0.f)) ? 0.f : acc;  // g1
    }
  }
  __syncthreads();
  // layer 1: dW1 [H, K], db1 [H], dx [M, K]
  for (int i = threadIdx.x; i < H * K + (db1 ? H : 0) + (dx ? M * K : 0); i += 256) {
    if (i < H * K) {
      const int n = i / K, k = i % K;
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc = fmaf(dhs[m * H + n], x[(long long)m * K + k], acc);
      dW1[i] = acc1 ? dW1[i] + acc : acc;
    } else if (db1 && i < H * K + H) {
      const int n = i - H * K;
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc += dhs[m * H + n];
      db1[n] = acc1 ? db1[n] + acc : acc;
    } else {
      const int j = i - H * K - (db1 ? H : 0), m = j / K, k = j % K;
      float acc = 0.f;
      for (int n = 0; n < H; ++n) acc = fmaf(dhs[m * H + n], W1[(long long)n * K + k], acc);
      dx[j] = acc;
    }
  }
}

bool linear2_fits(int M, int K, int H, int O) {
  return M > 0 && K > 0 && H > 0 && O > 0 && (long long)M * H <= kChain2MaxHidden &&
         (long long)M * H * K + (long long)M * O * H <= (1LL << 20);
}

hipError_t linear2_fwd(const float* x, const float* W1, const float* b1, const float* W2, const float* b2, float* h,
                       float* y, int M, int K, int H, int O, bool relu1, bool relu2, hipStream_t stream) {
  if (!linear2_fits(M, K, H, O)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(linear2_fwd_kernel, dim3(1), dim3(256), 0, stream, x, W1, b1, W2, b2, h, y, M, K, H, O,
                     relu1 ? 1 : 0, relu2 ? 1 : 0);
  return hipGetLastError();
}

hipError_t linear2_bwd(const float* dy, const float* x, const float* W1, const float* h, const float* W2,
                       const float* y, float* dx, float* dW1, float* db1, float* dW2, float* db2, int M, int K, int H,
                       int O, bool relu1, bool acc1, bool acc2, hipStream_t stream) {
  if (!linear2_fits(M, K, H, O)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(linear2_bwd_kernel, dim3(1), dim3(256), 0, stream, dy, x, W1, h, W2, y, dx, dW1, db1, dW2, db2,
                     M, K, H, O, relu1 ? 1 : 0, acc1 ? 1 : 0, acc2 ? 1 : 0);
  return hipGetLastError();
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
