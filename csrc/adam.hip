// Flat fused Adam/AdamW: ONE launch over the engine's flat fp32 master buffer replaces torch's
// seven _foreach_* multi-tensor launches plus the DeepSpeed 1/world_size scale and the host-side
// bias-correction .item() syncs.  Memory-bound: 16-byte vector accesses on
// every stream (Guideline 13), nontemporal hints on the state streams (each byte is touched once;
// not on the 16-bit compute copy, which the next forward reads), one float4 group per
// thread over a full grid.  On the bench MLP's 67M parameters (profiles/r1_adam_v8_ab.txt): 5.41 TB/s
// with fp32 gradients, 6.43 TB/s with bf16 gradients where the streaming hints pay (6.12 without).
// The round-1/2 loop-shape variants (two groups per thread, 8-element groups, the Adam + W^T matrix
// kernel) measured no better and were removed; their A/B records stay in profiles/.
// Reference: torch.optim.Adam created at train.py:85, stepped by model_engine.step() at train.py:114.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include "dgt_common.h"
#include "dgt_kernels.h"
#include <algorithm>

namespace dgt {

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// 16-byte (fp32) / 8-byte (16-bit) vector accesses; NT = streaming (nontemporal) hint: every
// element is touched exactly once, so nothing is worth keeping in L2 / MALL.
template <bool NT, typename V>
DGT_DEVICE V vload(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename V>
DGT_DEVICE void vstore(V* p, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <typename T, bool NT> struct Vec4;
template <bool NT> struct Vec4<float, NT> {
  static DGT_DEVICE f32x4 load(const float* p) { return vload<NT>(reinterpret_cast<const f32x4*>(p)); }
  static DGT_DEVICE void store(float* p, f32x4 v) { vstore<NT>(reinterpret_cast<f32x4*>(p), v); }
};
template <bool NT> struct Vec4<__hip_bfloat16, NT> {
  static DGT_DEVICE f32x4 load(const __hip_bfloat16* p) {
    const u32x2 raw = vload<NT>(reinterpret_cast<const u32x2*>(p));
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
    vstore<NT>(reinterpret_cast<u32x2*>(p), *reinterpret_cast<u32x2*>(b));
  }
};
template <bool NT> struct Vec4<__half, NT> {
  static DGT_DEVICE f32x4 load(const __half* p) {
    const u32x2 raw = vload<NT>(reinterpret_cast<const u32x2*>(p));
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
    vstore<NT>(reinterpret_cast<u32x2*>(p), *reinterpret_cast<u32x2*>(b));
  }
};

template <typename GT, typename LT, bool NT, bool LPNT = NT>
DGT_DEVICE f32x4 adam_group(const AdamFlatArgs& a, const GT* __restrict__ grad, LT* __restrict__ lp, long long o,
                            float scale, float step_size_neg, float bc2_sqrt) {
  f32x4 p = Vec4<float, NT>::load(a.master + o), g = Vec4<GT, NT>::load(grad + o);
  f32x4 m = Vec4<float, NT>::load(a.exp_avg + o), v = Vec4<float, NT>::load(a.exp_avg_sq + o);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float mm = m[e], vv = v[e];
    p[e] = adam_update(p[e], g[e] * scale, mm, vv, a.hp, step_size_neg, bc2_sqrt);
    m[e] = mm;
    v[e] = vv;
  }
  Vec4<float, NT>::store(a.master + o, p);
  Vec4<float, NT>::store(a.exp_avg + o, m);
  Vec4<float, NT>::store(a.exp_avg_sq + o, v);
  if (lp) Vec4<LT, LPNT>::store(lp + o, p);
  return p;
}

// Bias corrections of this update: host scalars, or (graph replay) formed on the device from the
// step counter in double, exactly as torch's non-capturable Adam does on the host.
DGT_DEVICE void adam_bias_corrections(const AdamFlatArgs& a, float& step_size_neg, float& bc2_sqrt) {
  step_size_neg = a.step_size_neg;
  bc2_sqrt = a.bc2_sqrt;
  if (a.step_dev) {
    __shared__ float sc[2];
    if (threadIdx.x == 0) {
      const double t = (double)(*a.step_dev + (a.step_ticket ? 1 : 0));
      sc[0] = (float)(-(a.lr_d / (1.0 - pow(a.beta1_d, t))));
      sc[1] = (float)sqrt(1.0 - pow(a.beta2_d, t));
    }
    __syncthreads();
    step_size_neg = sc[0];
    bc2_sqrt = sc[1];
  }
}

// The counter advance of a launch that read *step_dev (thread 0 of every block, in
// adam_bias_corrections): each block's thread 0 takes a ticket once it is done; the last one
// stores the new step and rewinds the ticket for the next launch (vector atomics and stores).
DGT_DEVICE void advance_step(const AdamFlatArgs& a) {
  if (threadIdx.x != 0) return;
  __threadfence();
  const unsigned prev = atomicAdd(a.step_ticket, 1u);
  if (prev == gridDim.x - 1) {
    __threadfence();
    __hip_atomic_store(a.step_dev, *a.step_dev + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.step_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one float4 group per thread over a full grid (grid-stride past 2^20 blocks)
template <typename GT, typename LT>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamFlatArgs a) {
  const long long n4 = a.n >> 2;
  float step_size_neg, bc2_sqrt;
  adam_bias_corrections(a, step_size_neg, bc2_sqrt);
  float scale = a.grad_scale;
  if (a.grad_scale_dev) scale *= *a.grad_scale_dev;
  const GT* __restrict__ grad = static_cast<const GT*>(a.grad);
  LT* __restrict__ lp = static_cast<LT*>(a.param_lp);
  const long long stride = (long long)gridDim.x * blockDim.x;
  // the state streams are nontemporal; the 16-bit compute copy is stored with the default policy:
  // its 8-byte lane pieces then merge into whole lines in L2 (streamed, they went out as partial-line
  // writes) and it stays in the Infinity Cache for the next forward -- 302 -> 280 us over the bench
  // MLP's 67M weights (profiles/r3_adam_lp_policy_ab.txt)
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride)
    adam_group<GT, LT, true, false>(a, grad, lp, 4 * i, scale, step_size_neg, bc2_sqrt);
  if (a.step_ticket) advance_step(a);
}

template <typename GT, typename LT>
static void launch_adam_v(const AdamFlatArgs& a, hipStream_t s) {
  const long long grid = std::min<long long>(std::max<long long>((a.n / 4 + 255) / 256, 1), 1 << 20);
  hipLaunchKernelGGL((adam_flat_kernel<GT, LT>), dim3((int)grid), dim3(256), 0, s, a);
}

template <typename GT>
static hipError_t launch_adam_g(const AdamFlatArgs& a, hipStream_t s) {
  switch (a.param_lp ? a.lp_dtype : kF32) {
    case kBF16: launch_adam_v<GT, __hip_bfloat16>(a, s); break;
    case kF16: launch_adam_v<GT, __half>(a, s); break;
    default: {
      AdamFlatArgs b = a;
      b.param_lp = nullptr;  // fp32 params are the master buffer itself
      launch_adam_v<GT, float>(b, s);
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
  switch (a.grad_dtype) {
    case kBF16: return launch_adam_g<__hip_bfloat16>(a, stream);
    case kF16: return launch_adam_g<__half>(a, stream);
    default: return launch_adam_g<float>(a, stream);
  }
}

}  // namespace dgt
