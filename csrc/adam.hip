// Flat fused Adam/AdamW: ONE launch over the engine's flat fp32 master buffer replaces torch's
// seven _foreach_* multi-tensor launches plus the DeepSpeed 1/world_size scale and the host-side
// bias-correction .item() syncs.  Memory-bound: 16-byte vector accesses on
// every stream (Guideline 13), grid capped near 8 blocks/CU with a grid-stride loop.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static DGT_DEVICE f32x4 load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static DGT_DEVICE void store(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
};
template <> struct Vec4<__hip_bfloat16> {
  static DGT_DEVICE f32x4 load(const __hip_bfloat16* p) {
    const uint2 raw = *reinterpret_cast<const uint2*>(p);
    f32x4 r;
    r[0] = __uint_as_float(raw.x << 16);
    r[1] = __uint_as_float(raw.x & 0xffff0000u);
    r[2] = __uint_as_float(raw.y << 16);
    r[3] = __uint_as_float(raw.y & 0xffff0000u);
    return r;
  }
  static DGT_DEVICE void store(__hip_bfloat16* p, f32x4 v) {
    __hip_bfloat16 b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = __float2bfloat16(v[i]);
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<uint2*>(b);
  }
};
template <> struct Vec4<__half> {
  static DGT_DEVICE f32x4 load(const __half* p) {
    const uint2 raw = *reinterpret_cast<const uint2*>(p);
    const __half* h = reinterpret_cast<const __half*>(&raw);
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __half2float(h[i]);
    return r;
  }
  static DGT_DEVICE void store(__half* p, f32x4 v) {
    __half b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = __float2half(v[i]);
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<uint2*>(b);
  }
};

template <typename GT, typename LT>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamFlatArgs a) {
  const long long n4 = a.n >> 2;
  float step_size_neg = a.step_size_neg, bc2_sqrt = a.bc2_sqrt;
  if (a.step_dev) {  // graph replay: bias corrections from the device step counter, in double
    __shared__ float sc[2];
    if (threadIdx.x == 0) {
      const double t = (double)*a.step_dev;
      sc[0] = (float)(-(a.lr_d / (1.0 - pow(a.beta1_d, t))));
      sc[1] = (float)sqrt(1.0 - pow(a.beta2_d, t));
    }
    __syncthreads();
    step_size_neg = sc[0];
    bc2_sqrt = sc[1];
  }
  float scale = a.grad_scale;
  if (a.grad_scale_dev) scale *= *a.grad_scale_dev;
  const GT* __restrict__ grad = static_cast<const GT*>(a.grad);
  LT* __restrict__ lp = static_cast<LT*>(a.param_lp);
  // two float4 groups per thread per iteration: 8 independent 16-byte loads in flight per lane
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += 2 * stride) {
    const bool two = i + stride < n4;
    const long long o0 = 4 * i, o1 = 4 * (i + stride);
    f32x4 p0 = Vec4<float>::load(a.master + o0), g0 = Vec4<GT>::load(grad + o0);
    f32x4 m0 = Vec4<float>::load(a.exp_avg + o0), v0 = Vec4<float>::load(a.exp_avg_sq + o0);
    f32x4 p1, g1, m1, v1;
    if (two) {
      p1 = Vec4<float>::load(a.master + o1);
      g1 = Vec4<GT>::load(grad + o1);
      m1 = Vec4<float>::load(a.exp_avg + o1);
      v1 = Vec4<float>::load(a.exp_avg_sq + o1);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mm = m0[e], vv = v0[e];
      p0[e] = adam_update(p0[e], g0[e] * scale, mm, vv, a.hp, step_size_neg, bc2_sqrt);
      m0[e] = mm;
      v0[e] = vv;
    }
    Vec4<float>::store(a.master + o0, p0);
    Vec4<float>::store(a.exp_avg + o0, m0);
    Vec4<float>::store(a.exp_avg_sq + o0, v0);
    if (lp) Vec4<LT>::store(lp + o0, p0);
    if (two) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float mm = m1[e], vv = v1[e];
        p1[e] = adam_update(p1[e], g1[e] * scale, mm, vv, a.hp, step_size_neg, bc2_sqrt);
        m1[e] = mm;
        v1[e] = vv;
      }
      Vec4<float>::store(a.master + o1, p1);
      Vec4<float>::store(a.exp_avg + o1, m1);
      Vec4<float>::store(a.exp_avg_sq + o1, v1);
      if (lp) Vec4<LT>::store(lp + o1, p1);
    }
  }
}

template <typename GT>
static hipError_t launch_adam_g(const AdamFlatArgs& a, hipStream_t s, int grid) {
  switch (a.param_lp ? a.lp_dtype : kF32) {
    case kBF16: hipLaunchKernelGGL((adam_flat_kernel<GT, __hip_bfloat16>), dim3(grid), dim3(256), 0, s, a); break;
    case kF16: hipLaunchKernelGGL((adam_flat_kernel<GT, __half>), dim3(grid), dim3(256), 0, s, a); break;
    default: {
      AdamFlatArgs b = a;
      b.param_lp = nullptr;  // fp32 params are the master buffer itself
      hipLaunchKernelGGL((adam_flat_kernel<GT, float>), dim3(grid), dim3(256), 0, s, b);
    }
  }
  return hipGetLastError();
}

__global__ void step_increment_kernel(long long* c) { *c += 1; }

hipError_t step_increment(long long* counter, hipStream_t stream) {
  hipLaunchKernelGGL(step_increment_kernel, dim3(1), dim3(1), 0, stream, counter);
  return hipGetLastError();
}

hipError_t adam_flat(const AdamFlatArgs& a, hipStream_t stream) {
  if (a.n % 4 != 0) return hipErrorInvalidValue;
  const long long n4 = a.n / 4;
  long long grid = (n4 + 511) / 512;
  if (grid > 4096) grid = 4096;  // 16 blocks per CU: enough loads in flight to stream HBM
  if (grid < 1) grid = 1;
  switch (a.grad_dtype) {
    case kBF16: return launch_adam_g<__hip_bfloat16>(a, stream, (int)grid);
    case kF16: return launch_adam_g<__half>(a, stream, (int)grid);
    default: return launch_adam_g<float>(a, stream, (int)grid);
  }
}

}  // namespace dgt
