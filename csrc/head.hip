// Skinny bf16 Linear (N <= 4 outputs) for the engine's MFMA Linear chain (ops/linear.py): the
// binary head of an MLP, Linear(K, 1) on the last hidden activation, which no 128x128 MFMA tile
// fits.  Left to F.linear it runs a vendor GEMV / GEMM (hipBLASLt); here it is two bandwidth-bound
// passes over the activation with 16-byte accesses.
//   forward   z[M, N] = a[M, K] . W[N, K]^T + b     one wave per row, fp32 accumulation, bf16 out
//   backward  g = (dz . W) * 1[a > 0] (+ g^T)       one wave per 64 x 64 tile of a, 8 x 8 per lane:
//             dW += dz^T . a, db += sum dz          eight 16-B row loads of a, eight 16-B row stores
//                                                   of g and eight of g^T per lane, no LDS; each tile
//                                                   stores its dW partial, a second pass sums them in
//                                                   row-tile order (no atomics: bit-reproducible, so a
//                                                   resumed run replays the uninterrupted one exactly)
// g (masked by the ReLU that produced a) and g^T are exactly the top hidden layer's pre-activation
// gradient in both layouts, which its wgrad and dgrad GEMMs read next (csrc/gemm.hip).
// Reference: the Linear(64, 1) output layer of train.py:32, widened (SyntheticMLP's head).
#include <hip/hip_bf16.h>

#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

namespace {
typedef unsigned short u16;
DGT_DEVICE float b2f(u16 u) { return __uint_as_float(((unsigned)u) << 16); }
DGT_DEVICE u16 f2b(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<u16*>(&b);
}
DGT_DEVICE void unpack8(const uint4& v, float (&o)[8]) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o[2 * q] = b2f((u16)(w[q] & 0xffff));
    o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
}  // namespace

template <int N>
__global__ __launch_bounds__(256) void skinny_fwd_kernel(const u16* __restrict__ a, const u16* __restrict__ W,
                                                         const u16* __restrict__ b, u16* __restrict__ z, int M, int K) {
  const int l = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const u16* ar = a + (long long)row * K;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
#pragma unroll 4  // the row's 16-byte loads in flight together
  for (int c = l * 8; c < K; c += 64 * 8) {
    float av[8];
    unpack8(*reinterpret_cast<const uint4*>(ar + c), av);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float wv[8];
      unpack8(*reinterpret_cast<const uint4*>(W + (long long)n * K + c), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[n] = fmaf(av[e], wv[e], acc[n]);
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = wave_sum(acc[n]);
  if (l < N) {
    float v = acc[0];
#pragma unroll
    for (int n = 1; n < N; ++n) v = l == n ? acc[n] : v;
    z[(long long)row * N + l] = f2b(v + (b ? b2f(b[l]) : 0.f));
  }
}

template <int N>
__global__ __launch_bounds__(256) void skinny_bwd_kernel(const u16* __restrict__ dz, const u16* __restrict__ a,
                                                         const u16* __restrict__ W, int mask, u16* __restrict__ g,
                                                         u16* __restrict__ gT, float* __restrict__ part_ws,
                                                         void* __restrict__ db, int db_bf16, int acc, int M, int K,
                                                         float* __restrict__ bias_part) {
  const int l = threadIdx.x & 63, cg = l & 7, rb = l >> 3, wv = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + rb * 8, c = (blockIdx.x * (blockDim.x >> 6) + wv) * 64 + cg * 8;
  float w[N][8];
#pragma unroll
  for (int n = 0; n < N; ++n) unpack8(*reinterpret_cast<const uint4*>(W + (long long)n * K + c), w[n]);
  uint4 av[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) av[k] = *reinterpret_cast<const uint4*>(a + (long long)(r + k) * K + c);
  float part[N][8];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int e = 0; e < 8; ++e) part[n][e] = 0.f;
  u16 gb[8][8];
  float gsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums of g (bias_part)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float d[N];
#pragma unroll
    for (int n = 0; n < N; ++n) d[n] = b2f(dz[(long long)(r + k) * N + n]);
    float x[8];
    unpack8(av[k], x);
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        s = fmaf(d[n], w[n][e], s);
        part[n][e] = fmaf(d[n], x[e], part[n][e]);
      }
      gb[k][e] = f2b((!mask || x[e] > 0.f) ? s : 0.f);
      gsum[e] += b2f(gb[k][e]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (unsigned)gb[k][2 * q] | ((unsigned)gb[k][2 * q + 1] << 16);
    *reinterpret_cast<uint4*>(g + (long long)(r + k) * K + c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  if (gT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      unsigned o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (unsigned)gb[2 * q][e] | ((unsigned)gb[2 * q + 1][e] << 16);
      *reinterpret_cast<uint4*>(gT + (long long)(c + e) * M + r) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
  // dW partial of the tile: sum its 8 row-blocks (lanes cg, cg + 8, ..., cg + 56), stored at
  // part_ws[row tile][n][column]
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = part[n][e];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 16);
      x += __shfl_xor(x, 32);
      part[n][e] = x;
    }
  if (bias_part) {  // per-64-row-tile column sums of g: the layer below's bias-gradient partials
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = gsum[e];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 16);
      x += __shfl_xor(x, 32);
      gsum[e] = x;
    }
    if (rb == 0) {
      float4* o = reinterpret_cast<float4*>(bias_part + (long long)blockIdx.y * K + c);
      o[0] = make_float4(gsum[0], gsum[1], gsum[2], gsum[3]);
      o[1] = make_float4(gsum[4], gsum[5], gsum[6], gsum[7]);
    }
  }
  if (rb == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float4* o = reinterpret_cast<float4*>(part_ws + ((long long)blockIdx.y * N + n) * K + c);
      o[0] = make_float4(part[n][0], part[n][1], part[n][2], part[n][3]);
      o[1] = make_float4(part[n][4], part[n][5], part[n][6], part[n][7]);
    }
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && wv == 0) {  // db, in a fixed order
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float s = 0.f;
      for (int i0 = l; i0 < M; i0 += 64 * 8) {  // 8 loads per lane in flight, added in row order
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i0 + 64 * u < M ? b2f(dz[(long long)(i0 + 64 * u) * N + n]) : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
      }
      s = wave_sum(s);
      if (l == 0) {
        if (db_bf16) {
          u16* d = static_cast<u16*>(db) + n;
          *d = f2b((acc ? b2f(*d) : 0.f) + s);
        } else {
          float* d = static_cast<float*>(db) + n;
          *d = (acc ? *d : 0.f) + s;
        }
      }
    }
  }
}

// out[i] (+)= sum over row tiles t (in order) of part[t][i], i < n; out fp32 or bf16 (the sum in
// fp32, rounded once).  One float4 column group per thread, its tiles' loads issued 8 at a time
// (independent), then added in tile order.
template <bool BF>
__global__ __launch_bounds__(64) void partials_reduce_kernel(const float* __restrict__ part_ws, void* __restrict__ out,
                                                             int tiles, int nk, int acc) {
  const int i = (blockIdx.x * 64 + threadIdx.x) * 4;
  if (i >= nk) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int t0 = 0; t0 < tiles; t0 += 8) {
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t0 + j < tiles) p[j] = *reinterpret_cast<const float4*>(part_ws + (long long)(t0 + j) * nk + i);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t0 + j < tiles) s.x += p[j].x, s.y += p[j].y, s.z += p[j].z, s.w += p[j].w;
  }
  if constexpr (BF) {
    u16* d = static_cast<u16*>(out) + i;
    if (acc) s = make_float4(b2f(d[0]) + s.x, b2f(d[1]) + s.y, b2f(d[2]) + s.z, b2f(d[3]) + s.w);
    const unsigned lo = (unsigned)f2b(s.x) | ((unsigned)f2b(s.y) << 16);
    const unsigned hi = (unsigned)f2b(s.z) | ((unsigned)f2b(s.w) << 16);
    *reinterpret_cast<uint2*>(d) = make_uint2(lo, hi);
  } else {
    float4* d = reinterpret_cast<float4*>(static_cast<float*>(out) + i);
    if (acc) {
      const float4 o = *d;
      s = make_float4(o.x + s.x, o.y + s.y, o.z + s.z, o.w + s.w);
    }
    *d = s;
  }
}

// ReduceSegs: every segment's float4 columns in one grid; each thread finds its segment by a
// uniform scan of <= kMaxReduceSegs prefix sums, then sums its column's tiles in order (the
// partials_reduce order, so the same bits as separate launches).
__global__ __launch_bounds__(64) void partials_reduce_multi_kernel(ReduceSegs r, ReduceAdam ad) {
  int i = (blockIdx.x * 64 + threadIdx.x) * 4;
  int s = 0;
  while (s < r.count && i >= r.n[s]) i -= r.n[s++];
  if (s >= r.count) return;
  const float* part = r.part[s];
  const int tiles = r.tiles[s], n = r.n[s];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int t0 = 0; t0 < tiles; t0 += 8) {
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t0 + j < tiles) p[j] = *reinterpret_cast<const float4*>(part + (long long)(t0 + j) * n + i);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (t0 + j < tiles) acc.x += p[j].x, acc.y += p[j].y, acc.z += p[j].z, acc.w += p[j].w;
  }
  const int fl = r.flags[s];
  if (fl & 1) {  // bf16 out (the engine's gradient bucket views): the sum in fp32, rounded once
    u16* d = static_cast<u16*>(r.out[s]) + i;
    if (fl & 2) acc = make_float4(b2f(d[0]) + acc.x, b2f(d[1]) + acc.y, b2f(d[2]) + acc.z, b2f(d[3]) + acc.w);
    const unsigned lo = (unsigned)f2b(acc.x) | ((unsigned)f2b(acc.y) << 16);
    const unsigned hi = (unsigned)f2b(acc.z) | ((unsigned)f2b(acc.w) << 16);
    *reinterpret_cast<uint2*>(d) = make_uint2(lo, hi);
    return;
  }
  float4* d = reinterpret_cast<float4*>(static_cast<float*>(r.out[s]) + i);
  if (fl & 2) {
    const float4 o = *d;
    acc = make_float4(o.x + acc.x, o.y + acc.y, o.z + acc.z, o.w + acc.w);
  }
  *d = acc;
  if (ad.on) {  // the region's Adam step on these four elements (adam_flat's per-element op order)
    const long long o = (long long)(static_cast<const float*>(r.out[s]) - ad.grads) + i;
    float4 p = *reinterpret_cast<const float4*>(ad.master + o);
    float4 m = *reinterpret_cast<const float4*>(ad.m + o);
    float4 v = *reinterpret_cast<const float4*>(ad.v + o);
    float* pp = &p.x;
    float* mp = &m.x;
    float* vp = &v.x;
    const float* gp = &acc.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) pp[e] = adam_update(pp[e], gp[e] * ad.grad_scale, mp[e], vp[e], ad.hp, ad.step_size_neg, ad.bc2_sqrt);
    *reinterpret_cast<float4*>(ad.master + o) = p;
    *reinterpret_cast<float4*>(ad.m + o) = m;
    *reinterpret_cast<float4*>(ad.v + o) = v;
  }
}

// fp32 skinny Linear (N <= 4 outputs): the binary head of an fp32 MLP on the engine's fused Linear
// path (ops/linear.py).  A 64 x 64 MFMA tile computing one useful column (forward, wgrad) or one
// useful k step (dgrad) wastes the matrix cores and still pays a split-K reduce; these are the two
// bandwidth-bound passes over the activation instead.
//   forward   z[M, N] = act(a[M, K] . W[N, K]^T + b)            one wave per row, float4 loads
//   backward  g = dz * 1[y > 0] (y: the head's own ReLU output, optional)
//             dx = (g . W) * 1[a > 0] (mask: a is the layer below's ReLU output)
//             dW (+)= g^T . a as per-64-row-tile partials + the fixed-order partials_reduce,
//             db (+)= sum g in row order: deterministic, no atomics
template <int N>
__global__ __launch_bounds__(256) void skinny_f32_fwd_kernel(const float* __restrict__ a, const float* __restrict__ W,
                                                             const float* __restrict__ b, float* __restrict__ z,
                                                             int M, int K, int relu) {
  const int l = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* ar = a + (long long)row * K;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
#pragma unroll 4
  for (int c = l * 4; c < K; c += 64 * 4) {
    const float4 av = *reinterpret_cast<const float4*>(ar + c);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float4 wv = *reinterpret_cast<const float4*>(W + (long long)n * K + c);
      acc[n] = fmaf(av.x, wv.x, acc[n]);
      acc[n] = fmaf(av.y, wv.y, acc[n]);
      acc[n] = fmaf(av.z, wv.z, acc[n]);
      acc[n] = fmaf(av.w, wv.w, acc[n]);
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = wave_sum(acc[n]);
  if (l < N) {
    float v = acc[0];
#pragma unroll
    for (int n = 1; n < N; ++n) v = l == n ? acc[n] : v;
    v += b ? b[l] : 0.f;
    z[(long long)row * N + l] = relu ? fmaxf(v, 0.f) : v;
  }
}

// one wave per 64 x 32 tile of a: lane (cg = l & 7, rb = l >> 3) owns rows rb*8 .. +7, columns cg*4 .. +3
template <int N>
__global__ __launch_bounds__(256) void skinny_f32_bwd_kernel(const float* __restrict__ dz, const float* __restrict__ y,
                                                             const float* __restrict__ a, const float* __restrict__ W,
                                                             int mask, float* __restrict__ dx,
                                                             float* __restrict__ part_ws, float* __restrict__ db,
                                                             int acc, int M, int K) {
  const int l = threadIdx.x & 63, cg = l & 7, rb = l >> 3, wv = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + rb * 8, c = (blockIdx.x * (blockDim.x >> 6) + wv) * 32 + cg * 4;
  float w[N][4];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const float4 t = *reinterpret_cast<const float4*>(W + (long long)n * K + c);
    w[n][0] = t.x, w[n][1] = t.y, w[n][2] = t.z, w[n][3] = t.w;
  }
  float4 av[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) av[k] = *reinterpret_cast<const float4*>(a + (long long)(r + k) * K + c);
  float part[N][4];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int e = 0; e < 4; ++e) part[n][e] = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float d[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const long long o = (long long)(r + k) * N + n;
      d[n] = (y && !(y[o] > 0.f)) ? 0.f : dz[o];
    }
    const float x[4] = {av[k].x, av[k].y, av[k].z, av[k].w};
    float o4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = 0.f;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        s = fmaf(d[n], w[n][e], s);
        part[n][e] = fmaf(d[n], x[e], part[n][e]);
      }
      o4[e] = (!mask || x[e] > 0.f) ? s : 0.f;
    }
    if (dx) *reinterpret_cast<float4*>(dx + (long long)(r + k) * K + c) = make_float4(o4[0], o4[1], o4[2], o4[3]);
  }
  // the tile's dW partial: its 8 row blocks (lanes cg, cg + 8, ..., cg + 56) summed
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = part[n][e];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 16);
      x += __shfl_xor(x, 32);
      part[n][e] = x;
    }
  if (rb == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n)
      *reinterpret_cast<float4*>(part_ws + ((long long)blockIdx.y * N + n) * K + c) =
          make_float4(part[n][0], part[n][1], part[n][2], part[n][3]);
  }
  if (db && blockIdx.x == 0 && blockIdx.y == 0 && wv == 0) {  // db, in a fixed order
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float s = 0.f;
      for (int i0 = l; i0 < M; i0 += 64 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long long o = (long long)(i0 + 64 * u) * N + n;
          v[u] = (i0 + 64 * u < M && !(y && !(y[o] > 0.f))) ? dz[o] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
      }
      s = wave_sum(s);
      if (l == 0) db[n] = (acc ? db[n] : 0.f) + s;
    }
  }
}

hipError_t partials_reduce_multi(const ReduceSegs& r, const ReduceAdam& adam, hipStream_t stream) {
  if (r.count < 1 || r.count > kMaxReduceSegs) return hipErrorInvalidValue;
  long long total = 0;
  for (int s = 0; s < r.count; ++s) {
    if (r.n[s] <= 0 || r.n[s] % 4 || r.tiles[s] < 1 || (reinterpret_cast<uintptr_t>(r.part[s]) & 15) ||
        (reinterpret_cast<uintptr_t>(r.out[s]) & ((r.flags[s] & 1) ? 7 : 15)) || (adam.on && r.flags[s]))
      return hipErrorInvalidValue;
    total += r.n[s];
  }
  const dim3 grid((unsigned)((total / 4 + 63) / 64)), blk(64);
  hipLaunchKernelGGL(partials_reduce_multi_kernel, grid, blk, 0, stream, r, adam);
  return hipGetLastError();
}

hipError_t partials_reduce(const float* part, void* out, int out_bf16, int tiles, int n, int accumulate,
                           hipStream_t stream) {
  if (n % 4 || tiles < 1 || (reinterpret_cast<uintptr_t>(part) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & (out_bf16 ? 7 : 15)))
    return hipErrorInvalidValue;
  const dim3 grid((n / 4 + 63) / 64), blk(64);
  if (out_bf16) hipLaunchKernelGGL(partials_reduce_kernel<true>, grid, blk, 0, stream, part, out, tiles, n, accumulate);
  else hipLaunchKernelGGL(partials_reduce_kernel<false>, grid, blk, 0, stream, part, out, tiles, n, accumulate);
  return hipGetLastError();
}

hipError_t skinny_fwd_bf16(const void* a, const void* W, const void* b, void* z, int M, int N, int K,
                           hipStream_t stream) {
  if (N < 1 || N > 4 || K % 8 || M <= 0) return hipErrorInvalidValue;
  const dim3 grid((M + 3) / 4), blk(256);
  const u16 *ap = static_cast<const u16*>(a), *wp = static_cast<const u16*>(W), *bp = static_cast<const u16*>(b);
  u16* zp = static_cast<u16*>(z);
  switch (N) {
    case 1: hipLaunchKernelGGL(skinny_fwd_kernel<1>, grid, blk, 0, stream, ap, wp, bp, zp, M, K); break;
    case 2: hipLaunchKernelGGL(skinny_fwd_kernel<2>, grid, blk, 0, stream, ap, wp, bp, zp, M, K); break;
    case 3: hipLaunchKernelGGL(skinny_fwd_kernel<3>, grid, blk, 0, stream, ap, wp, bp, zp, M, K); break;
    default: hipLaunchKernelGGL(skinny_fwd_kernel<4>, grid, blk, 0, stream, ap, wp, bp, zp, M, K);
  }
  return hipGetLastError();
}

hipError_t skinny_bwd_bf16(const void* dz, const void* a, const void* W, int mask, void* g, void* gT, void* dW,
                           void* db, int dw_bf16, int accumulate, float* part_ws, int M, int N, int K,
                           hipStream_t stream, float* bias_part) {
  if (N < 1 || N > 4 || M % 64 || K % 64 || M <= 0 || K <= 0) return hipErrorInvalidValue;
  const int wpb = K % 256 == 0 ? 4 : 1;  // 4 tiles per block side by side when the width allows
  const dim3 grid(K / (64 * wpb), M / 64), blk(64 * wpb);
  const u16 *dp = static_cast<const u16*>(dz), *ap = static_cast<const u16*>(a), *wp = static_cast<const u16*>(W);
  u16 *gp = static_cast<u16*>(g), *gtp = static_cast<u16*>(gT);
  switch (N) {
    case 1: hipLaunchKernelGGL(skinny_bwd_kernel<1>, grid, blk, 0, stream, dp, ap, wp, mask, gp, gtp, part_ws, db, dw_bf16, accumulate, M, K, bias_part); break;
    case 2: hipLaunchKernelGGL(skinny_bwd_kernel<2>, grid, blk, 0, stream, dp, ap, wp, mask, gp, gtp, part_ws, db, dw_bf16, accumulate, M, K, bias_part); break;
    case 3: hipLaunchKernelGGL(skinny_bwd_kernel<3>, grid, blk, 0, stream, dp, ap, wp, mask, gp, gtp, part_ws, db, dw_bf16, accumulate, M, K, bias_part); break;
    default: hipLaunchKernelGGL(skinny_bwd_kernel<4>, grid, blk, 0, stream, dp, ap, wp, mask, gp, gtp, part_ws, db, dw_bf16, accumulate, M, K, bias_part);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (!dW) return hipSuccess;  // part_ws is the caller's: it reduces the partials (partials_reduce_multi)
  return partials_reduce(part_ws, dW, dw_bf16, M / 64, N * K, accumulate, stream);  // K % 64: whole float4s
}

hipError_t skinny_f32_fwd(const float* a, const float* W, const float* b, float* z, int M, int N, int K, int relu,
                          hipStream_t stream) {
  if (N < 1 || N > 4 || K % 4 || M <= 0) return hipErrorInvalidValue;
  const dim3 grid((M + 3) / 4), blk(256);
  switch (N) {
    case 1: hipLaunchKernelGGL(skinny_f32_fwd_kernel<1>, grid, blk, 0, stream, a, W, b, z, M, K, relu); break;
    case 2: hipLaunchKernelGGL(skinny_f32_fwd_kernel<2>, grid, blk, 0, stream, a, W, b, z, M, K, relu); break;
    case 3: hipLaunchKernelGGL(skinny_f32_fwd_kernel<3>, grid, blk, 0, stream, a, W, b, z, M, K, relu); break;
    default: hipLaunchKernelGGL(skinny_f32_fwd_kernel<4>, grid, blk, 0, stream, a, W, b, z, M, K, relu);
  }
  return hipGetLastError();
}

hipError_t skinny_f32_bwd(const float* dz, const float* y, const float* a, const float* W, int mask, float* dx,
                          float* dW, float* db, int accumulate, float* part_ws, int M, int N, int K,
                          hipStream_t stream) {
  if (N < 1 || N > 4 || M % 64 || K % 32 || M <= 0 || K <= 0 || !dW) return hipErrorInvalidValue;
  const int wpb = K % 128 == 0 ? 4 : 1;  // 4 tiles per block side by side when the width allows
  const dim3 grid(K / (32 * wpb), M / 64), blk(64 * wpb);
  switch (N) {
    case 1: hipLaunchKernelGGL(skinny_f32_bwd_kernel<1>, grid, blk, 0, stream, dz, y, a, W, mask, dx, part_ws, db, accumulate, M, K); break;
    case 2: hipLaunchKernelGGL(skinny_f32_bwd_kernel<2>, grid, blk, 0, stream, dz, y, a, W, mask, dx, part_ws, db, accumulate, M, K); break;
    case 3: hipLaunchKernelGGL(skinny_f32_bwd_kernel<3>, grid, blk, 0, stream, dz, y, a, W, mask, dx, part_ws, db, accumulate, M, K); break;
    default: hipLaunchKernelGGL(skinny_f32_bwd_kernel<4>, grid, blk, 0, stream, dz, y, a, W, mask, dx, part_ws, db, accumulate, M, K);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return partials_reduce(part_ws, dW, 0, M / 64, N * K, accumulate, stream);  // K % 32: whole float4s
}

}  // namespace dgt
