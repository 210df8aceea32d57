// Fused BCE-with-logits (mean) for the engine path: ONE kernel computes the loss AND the gradient
// with respect to the logits (saved for backward), replacing torch's ~11 loss kernels per step
// (log_sigmoid_forward, fill, sub, mul, sub, mean; ones_like, sigmoid, sub, mul, div) — in a
// HIP-graph-replayed step each node costs a few microseconds, whatever it computes.
//   loss = mean_i[(1 - y_i) z_i - log_sigmoid(z_i)],   dz_i = (sigmoid(z_i) - y_i) / N
// One workgroup walks the N elements in a fixed order and reduces in a fixed tree: deterministic.
// Reference: nn.BCEWithLogitsLoss() at train.py:96, applied at train.py:112.
#include <hip/hip_bf16.h>
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

template <typename T>
DGT_DEVICE float to_f(T v);
template <>
DGT_DEVICE float to_f<float>(float v) { return v; }
template <>
DGT_DEVICE float to_f<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }

template <typename T>
__global__ __launch_bounds__(1024) void bce_logits_kernel(const T* __restrict__ z, const float* __restrict__ y, long long n,
                                                          float* __restrict__ loss, float* __restrict__ dz,
                                                          __hip_bfloat16* __restrict__ dz_lp,
                                                          double* __restrict__ sum_into) {
  __shared__ float red[32];
  const float inv_n = 1.f / (float)n;
  float acc = 0.f;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    const float zi = to_f<T>(z[i]), yi = y[i];
    const float e = __expf(-fabsf(zi));
    const float r = 1.f / (1.f + e);
    const float sig = zi >= 0.f ? r : e * r;
    acc += (1.f - yi) * zi - (fminf(zi, 0.f) - log1pf(e));
    const float d = (sig - yi) * inv_n;
    dz[i] = d;
    if (dz_lp) dz_lp[i] = __float2bfloat16(d);  // the product with a unit seed, rounded once
  }
  acc = wave_sum(acc);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    const float l = s * inv_n;
    *loss = l;
    if (sum_into) *sum_into += (double)l;  // the loss log (train.py:115's running sum), as loss_acc += loss
  }
}

hipError_t bce_logits(const void* z, int z_dtype, const float* y, long long n, float* loss, float* dz, void* dz_lp,
                      double* sum_into, hipStream_t stream) {
  if (n < 1) return hipErrorInvalidValue;
  const int threads = n >= 1024 ? 1024 : (int)((n + 63) / 64 * 64);
  if (z_dtype == kBF16)
    hipLaunchKernelGGL(bce_logits_kernel<__hip_bfloat16>, dim3(1), dim3(threads), 0, stream,
                       static_cast<const __hip_bfloat16*>(z), y, n, loss, dz,
                       static_cast<__hip_bfloat16*>(dz_lp), sum_into);
  else
    hipLaunchKernelGGL(bce_logits_kernel<float>, dim3(1), dim3(threads), 0, stream, static_cast<const float*>(z), y,
                       n, loss, dz, static_cast<__hip_bfloat16*>(dz_lp), sum_into);
  return hipGetLastError();
}

}  // namespace dgt
