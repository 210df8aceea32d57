// Flat fused Adam/AdamW: ONE launch over the engine's flat fp32 master buffer replaces torch's
// seven _foreach_* multi-tensor launches plus the DeepSpeed 1/world_size scale and the host-side
// bias-correction .item() syncs.  Memory-bound: 16-byte vector accesses on
// every stream (Guideline 13), nontemporal hints (each byte is touched once), one float4 group per
// thread over a full grid.  On the bench MLP's 67M parameters (profiles/r1_adam_v8_ab.txt): 5.41 TB/s
// with fp32 gradients (the plain variant 3 ties it), 6.43 TB/s with bf16 gradients where the
// streaming hints pay (6.12 without) - the bf16 MLP step is the case the default is tuned for.
// Reference: torch.optim.Adam created at train.py:85, stepped by model_engine.step() at train.py:114.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include "dgt_common.h"
#include "dgt_kernels.h"
#include <algorithm>
#include <cstdlib>

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

template <typename GT, typename LT, bool NT>
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
  if (lp) Vec4<LT, NT>::store(lp + o, p);
  return p;
}

// Eight consecutive elements per thread: the 16-bit streams (bf16/fp16 gradients and the compute
// copy) then move as 16-byte vectors too, instead of the 8-byte accesses of a float4 group.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <typename T> DGT_DEVICE T from_f32(float x);
template <> DGT_DEVICE __hip_bfloat16 from_f32<__hip_bfloat16>(float x) { return __float2bfloat16(x); }
template <> DGT_DEVICE __half from_f32<__half>(float x) { return __float2half(x); }
template <typename T, bool NT> struct Vec8 {  // 16-bit types: one 16-byte access
  static DGT_DEVICE void load(const T* p, f32x4& lo, f32x4& hi) {
    const u32x4 raw = vload<NT>(reinterpret_cast<const u32x4*>(p));
    const T* h = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (float)h[i];
      hi[i] = (float)h[4 + i];
    }
  }
  static DGT_DEVICE void store(T* p, const f32x4& lo, const f32x4& hi) {
    T b[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      b[i] = from_f32<T>(lo[i]);
      b[4 + i] = from_f32<T>(hi[i]);
    }
    vstore<NT>(reinterpret_cast<u32x4*>(p), *reinterpret_cast<u32x4*>(b));
  }
};
template <bool NT> struct Vec8<float, NT> {
  static DGT_DEVICE void load(const float* p, f32x4& lo, f32x4& hi) {
    lo = Vec4<float, NT>::load(p);
    hi = Vec4<float, NT>::load(p + 4);
  }
  static DGT_DEVICE void store(float* p, const f32x4& lo, const f32x4& hi) {
    Vec4<float, NT>::store(p, lo);
    Vec4<float, NT>::store(p + 4, hi);
  }
};

template <typename GT, typename LT, bool NT>
DGT_DEVICE void adam_group8(const AdamFlatArgs& a, const GT* __restrict__ grad, LT* __restrict__ lp, long long o,
                            float scale, float step_size_neg, float bc2_sqrt) {
  f32x4 p[2], g[2], m[2], v[2];
  Vec8<float, NT>::load(a.master + o, p[0], p[1]);
  Vec8<GT, NT>::load(grad + o, g[0], g[1]);
  Vec8<float, NT>::load(a.exp_avg + o, m[0], m[1]);
  Vec8<float, NT>::load(a.exp_avg_sq + o, v[0], v[1]);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mm = m[h][e], vv = v[h][e];
      p[h][e] = adam_update(p[h][e], g[h][e] * scale, mm, vv, a.hp, step_size_neg, bc2_sqrt);
      m[h][e] = mm;
      v[h][e] = vv;
    }
  Vec8<float, NT>::store(a.master + o, p[0], p[1]);
  Vec8<float, NT>::store(a.exp_avg + o, m[0], m[1]);
  Vec8<float, NT>::store(a.exp_avg_sq + o, v[0], v[1]);
  if (lp) Vec8<LT, NT>::store(lp + o, p[0], p[1]);
}

// Bias corrections of this update: host scalars, or (graph replay) formed on the device from the
// step counter in double, exactly as torch's non-capturable Adam does on the host.
DGT_DEVICE void adam_bias_corrections(const AdamFlatArgs& a, float& step_size_neg, float& bc2_sqrt) {
  step_size_neg = a.step_size_neg;
  bc2_sqrt = a.bc2_sqrt;
  if (a.step_dev) {
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
}

// GROUPS float4 groups per thread per grid-stride iteration
template <typename GT, typename LT, bool NT, int GROUPS>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamFlatArgs a) {
  const long long n4 = a.n >> 2;
  float step_size_neg, bc2_sqrt;
  adam_bias_corrections(a, step_size_neg, bc2_sqrt);
  float scale = a.grad_scale;
  if (a.grad_scale_dev) scale *= *a.grad_scale_dev;
  const GT* __restrict__ grad = static_cast<const GT*>(a.grad);
  LT* __restrict__ lp = static_cast<LT*>(a.param_lp);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += GROUPS * stride) {
#pragma unroll
    for (int gi = 0; gi < GROUPS; ++gi)
      if (gi == 0 || i + gi * stride < n4)
        adam_group<GT, LT, NT>(a, grad, lp, 4 * (i + gi * stride), scale, step_size_neg, bc2_sqrt);
  }
}

// one 8-element group per thread; a trailing float4 group (n % 8 == 4) goes to thread n / 8
template <typename GT, typename LT, bool NT>
__global__ __launch_bounds__(256) void adam_flat8_kernel(AdamFlatArgs a) {
  float step_size_neg, bc2_sqrt;
  adam_bias_corrections(a, step_size_neg, bc2_sqrt);
  float scale = a.grad_scale;
  if (a.grad_scale_dev) scale *= *a.grad_scale_dev;
  const GT* __restrict__ grad = static_cast<const GT*>(a.grad);
  LT* __restrict__ lp = static_cast<LT*>(a.param_lp);
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x, n8 = a.n >> 3;
  if (i < n8) adam_group8<GT, LT, NT>(a, grad, lp, 8 * i, scale, step_size_neg, bc2_sqrt);
  else if (i == n8 && (a.n & 4)) adam_group<GT, LT, NT>(a, grad, lp, 8 * i, scale, step_size_neg, bc2_sqrt);
}

// Loop shape chosen by measurement (scripts/bench_adam.py).  DGT_ADAM_VARIANT (read ONCE, at the
// first launch: no getenv on the launch path) or adam_set_variant() selects another for A/B runs.
static int g_adam_variant = -1;

static int adam_variant() {
  if (g_adam_variant < 0) {
    const char* e = getenv("DGT_ADAM_VARIANT");
    const int v = e ? atoi(e) : 0;
    g_adam_variant = (v >= 0 && v <= 4) ? v : 0;
  }
  return g_adam_variant;
}

bool adam_set_variant(int v) {
  if (v < 0 || v > 4) return false;
  g_adam_variant = v;
  return true;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <typename GT, typename LT>
static void launch_adam_v(const AdamFlatArgs& a, hipStream_t s) {
  const long long n4 = a.n / 4;
  long long grid;
  switch (adam_variant()) {
    case 1:  // two groups per thread, plain, capped grid
      grid = std::min<long long>(std::max<long long>((n4 + 511) / 512, 1), 4096);
      hipLaunchKernelGGL((adam_flat_kernel<GT, LT, false, 2>), dim3((int)grid), dim3(256), 0, s, a);
      break;
    case 2:  // two groups, streaming hints, capped grid
      grid = std::min<long long>(std::max<long long>((n4 + 511) / 512, 1), 4096);
      hipLaunchKernelGGL((adam_flat_kernel<GT, LT, true, 2>), dim3((int)grid), dim3(256), 0, s, a);
      break;
    case 3:  // one group per thread, plain, full grid
      grid = std::min<long long>(std::max<long long>((n4 + 255) / 256, 1), 1 << 20);
      hipLaunchKernelGGL((adam_flat_kernel<GT, LT, false, 1>), dim3((int)grid), dim3(256), 0, s, a);
      break;
    case 4:  // one 8-element group per thread (16-byte 16-bit streams), streaming hints, full grid
      // 16-byte loads/stores of the 16-bit streams: a slice at a 4-element offset takes the default
      if ((sizeof(GT) == 2 && !aligned16(a.grad)) || (a.param_lp && sizeof(LT) == 2 && !aligned16(a.param_lp))) {
        grid = std::min<long long>(std::max<long long>((n4 + 255) / 256, 1), 1 << 20);
        hipLaunchKernelGGL((adam_flat_kernel<GT, LT, true, 1>), dim3((int)grid), dim3(256), 0, s, a);
        break;
      }
      grid = std::max<long long>((a.n / 8 + 1 + 255) / 256, 1);
      hipLaunchKernelGGL((adam_flat8_kernel<GT, LT, true>), dim3((int)grid), dim3(256), 0, s, a);
      break;
    default:  // one group per thread, streaming hints, full grid
      grid = std::min<long long>(std::max<long long>((n4 + 255) / 256, 1), 1 << 20);
      hipLaunchKernelGGL((adam_flat_kernel<GT, LT, true, 1>), dim3((int)grid), dim3(256), 0, s, a);
  }
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

// Adam over one row-major fp32 weight matrix [rows, cols] that writes the bf16 compute copy AND
// its transpose (the dgrad GEMM's B operand, csrc/gemm.hip) in the same pass, instead of Adam
// followed by a transpose kernel that re-reads the bf16 copy (the MLP trainer's W^T refresh).
// Lane (rb, cg) of a wave updates rows 8rb..8rb+7 x cols 4cg..4cg+3 (rb, cg in 0..7): the eight
// lanes of one rb read a whole 128-byte line of every fp32 stream per row, and the eight lanes of
// one cg write a whole 128-byte line of W^T (64 rows x bf16) per column with 16-byte stores.
// No LDS: every transposed value is already in the register that stores it.  A block's four
// waves sit side by side along the columns: block tile = 64 rows x 128 cols.
template <typename GT>
__global__ __launch_bounds__(256) void adam_matrix_t_kernel(AdamFlatArgs a, __hip_bfloat16* __restrict__ lpT,
                                                            int rows, int cols) {
  float step_size_neg, bc2_sqrt;
  adam_bias_corrections(a, step_size_neg, bc2_sqrt);
  float scale = a.grad_scale;
  if (a.grad_scale_dev) scale *= *a.grad_scale_dev;
  const GT* __restrict__ grad = static_cast<const GT*>(a.grad);
  __hip_bfloat16* __restrict__ lp = static_cast<__hip_bfloat16*>(a.param_lp);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cg = lane & 7, rb = lane >> 3;
  const int c = blockIdx.x * 128 + wave * 32 + cg * 4;
  const int r = blockIdx.y * 64 + rb * 8;
  unsigned short b[8][4];  // bf16 bits of the updated 8 x 4 block
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const f32x4 p = adam_group<GT, __hip_bfloat16, true>(a, grad, lp, (long long)(r + k) * cols + c, scale,
                                                         step_size_neg, bc2_sqrt);
#pragma unroll
    for (int e = 0; e < 4; ++e) b[k][e] = __bfloat16_as_ushort(__float2bfloat16(p[e]));
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    u32x4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (unsigned)b[2 * q][e] | ((unsigned)b[2 * q + 1][e] << 16);
    *reinterpret_cast<u32x4*>(lpT + (long long)(c + e) * rows + r) = v;
  }
}

hipError_t adam_matrix_t(const AdamFlatArgs& a, void* lpT, int rows, int cols, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || rows % 64 || cols % 128 || a.n != (long long)rows * cols || !a.param_lp ||
      a.lp_dtype != kBF16 || !lpT)
    return hipErrorInvalidValue;
  const dim3 grid(cols / 128, rows / 64);
  switch (a.grad_dtype) {
    case kBF16:
      hipLaunchKernelGGL(adam_matrix_t_kernel<__hip_bfloat16>, grid, dim3(256), 0, stream, a,
                         static_cast<__hip_bfloat16*>(lpT), rows, cols);
      break;
    case kF32:
      hipLaunchKernelGGL(adam_matrix_t_kernel<float>, grid, dim3(256), 0, stream, a,
                         static_cast<__hip_bfloat16*>(lpT), rows, cols);
      break;
    default:
      return hipErrorInvalidValue;
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
