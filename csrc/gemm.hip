// bf16 GEMM on the CDNA4 matrix cores for the bench-size synthetic MLP, plus the small fused
// kernels around it (transpose, bias-gradient row sums, BCE head).
//
//   C[M, N] = A[M, K] . B[N, K]^T      (both operands K-contiguous: the "NT" form)
//
// Every product of an MLP training step is expressed in this one form by keeping transposed
// copies where a product needs one (activations and output gradients are written in both layouts
// by the producing epilogue; W^T is refreshed after each optimizer step):
//   forward  a_l   = relu(a_{l-1} . W_l^T + b_l)      NT(a_{l-1}, W_l)      -> a_l, a_l^T
//   dgrad    g_l-1 = (g_l . W_l) * 1[a_{l-1} > 0]     NT(g_l, W_l^T)        -> g_{l-1}, g_{l-1}^T
//   wgrad    dW_l  = g_l^T . a_{l-1}                  NT(g_l^T, a_{l-1}^T)  -> fp32 grad buffer
//
// Kernel structure (cdna_hip_programming.md §5): 128x128 block tile, BK = 64, 256 threads = 4 waves
// in 2x2, each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles.  Operands are staged
// global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR round trip), two LDS stages so
// the next K-tile streams in while the current one is consumed.  The LDS image is lane-linear (an
// LDS-DMA writes base + 16*lane), so the bank-conflict XOR swizzle (chunk ^= row & 7 on 128-B rows)
// is applied to the per-lane GLOBAL source address and undone on the ds_read_b128 side (rule 21).
// Block ids are remapped so blocks sharing an XCD (id % 8) get neighbouring tiles (T1).
#include <hip/hip_bf16.h>
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;

constexpr int GBM = 128, GBN = 128, GBK = 64;

DGT_DEVICE u16 f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<u16*>(&b);
}
DGT_DEVICE float bf2f(u16 u) { return __uint_as_float(((unsigned)u) << 16); }

// one 128 x 64 bf16 operand tile: 16 LDS-DMA wave-instructions of 1 KiB (8 rows each), 4 per wave
DGT_DEVICE void stage_tile(const u16* __restrict__ src, int ld, int row0, int k0, u16* lds, int w, int l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rblk = (w * 4 + i) * 8;          // first of the 8 rows this wave-instruction writes
    const int row = rblk + (l >> 3);
    const int p = l & 7;                       // LDS 16-B chunk this lane lands in
    const int c = p ^ (row & 7);               // logical chunk fetched (source-side swizzle)
    const u16* g = src + (long long)(row0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(g), reinterpret_cast<int*>(lds + rblk * GBK), 16, 0,
                                     0);
  }
}

DGT_DEVICE bf16x8 read_frag(const u16* lds, int row, int chunk) {
  const int p = chunk ^ (row & 7);
  return *reinterpret_cast<const bf16x8*>(lds + row * GBK + p * 8);
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][GBM * GBK];  // [stage][A|B] = 64 KiB
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int nbm = g.M / GBM, nbn = g.N / GBN, nwg = nbm * nbn;
  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous range
  const int bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  // group 8 block-rows together so consecutive wgids reuse the same B panel from L2
  const int GROUP = 8;
  const int group = wgid / (GROUP * nbn), first_m = group * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int tm = first_m + (wgid % (GROUP * nbn)) % gsize, tn = (wgid % (GROUP * nbn)) / gsize;
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int wr = w >> 1, wc = w & 1;
  const u16* A = static_cast<const u16*>(g.A);
  const u16* B = static_cast<const u16*>(g.B);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / GBK;
  stage_tile(A, g.lda, m0, 0, lds[0][0], w, l);
  stage_tile(B, g.ldb, n0, 0, lds[0][1], w, l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage_tile(A, g.lda, m0, (kt + 1) * GBK, lds[cur ^ 1][0], w, l);
      stage_tile(B, g.ldb, n0, (kt + 1) * GBK, lds[cur ^ 1][1], w, l);
    }
    const u16* As = lds[cur][0];
    const u16* Bs = lds[cur][1];
#pragma unroll
    for (int kk = 0; kk < GBK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag(As, wr * 64 + i * 16 + (l & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag(Bs, wc * 64 + j * 16 + (l & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: D col = l&15 (n), row = 4*(l>>4) + r (m)
  const float* bias = g.bias;
  const u16* mask = static_cast<const u16*>(g.mask);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + (l & 15);
      const int mb = m0 + wr * 64 + i * 16 + 4 * (l >> 4);
      const float bn = (EPI & kEpiBias) ? bias[n] : 0.f;
      float v[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float x = acc[i][j][rr] * g.alpha + bn;
        if (EPI & kEpiRelu) x = fmaxf(x, 0.f);
        if (EPI & kEpiMask) x = bf2f(mask[(long long)(mb + rr) * g.ldmask + n]) > 0.f ? x : 0.f;
        v[rr] = x;
      }
      if (EPI & kEpiOutF32) {
        float* C = static_cast<float*>(g.C);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float* p = C + (long long)(mb + rr) * g.ldc + n;
          *p = (EPI & kEpiAccumulate) ? *p + v[rr] : v[rr];
        }
      } else if (g.C) {
        u16* C = static_cast<u16*>(g.C);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) C[(long long)(mb + rr) * g.ldc + n] = f2bf(v[rr]);
      }
      if (EPI & kEpiStoreT) {  // C^T[n][m..m+3]: 4 consecutive bf16 per lane
        u16* CT = static_cast<u16*>(g.CT);
        uint2 packed;
        packed.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        packed.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(CT + (long long)n * g.ldct + mb) = packed;
      }
    }
  }
}

hipError_t gemm_nt(const GemmArgs& g, int epi, hipStream_t stream) {
  if (g.M % GBM || g.N % GBN || g.K % GBK || g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  const int grid = (g.M / GBM) * (g.N / GBN);
#define DGT_EPI_CASE(E)                                                                   \
  case E:                                                                                 \
    hipLaunchKernelGGL((gemm_nt_kernel<E>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
  switch (epi) {
    DGT_EPI_CASE(0)
    DGT_EPI_CASE(kEpiBias | kEpiRelu | kEpiStoreT)                 // hidden-layer forward
    DGT_EPI_CASE(kEpiBias | kEpiRelu)                              // forward, no transposed copy
    DGT_EPI_CASE(kEpiMask | kEpiStoreT)                            // dgrad through ReLU
    DGT_EPI_CASE(kEpiOutF32)                                       // wgrad into fp32 grads
    DGT_EPI_CASE(kEpiOutF32 | kEpiAccumulate)                      // wgrad, gradient accumulation
    DGT_EPI_CASE(kEpiOutF32 | kEpiBias)                            // generic fp32 out
    default:
      return hipErrorInvalidValue;
  }
#undef DGT_EPI_CASE
  return hipGetLastError();
}

// ------------------------------------------------------------------ transpose (bf16, 64x64 tiles)
// 16-byte global loads and stores: a thread moves one 8-element row chunk in and one 8-element
// column chunk out; the tile sits in LDS with a 2-element pad per row (no 32-way column conflicts).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const u16* __restrict__ in, u16* __restrict__ out,
                                                             int rows, int cols) {
  __shared__ u16 tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  const bool full = (r0 + 64 <= rows) && (c0 + 64 <= cols) && (cols % 8 == 0) && (rows % 8 == 0);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i;          // 512 chunks of 8 elements
    const int rr = idx >> 3, cc = (idx & 7) * 8;
    if (full) {
      const uint4 v = *reinterpret_cast<const uint4*>(in + (long long)(r0 + rr) * cols + c0 + cc);
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tile[rr][cc + 2 * e] = (u16)(w[e] & 0xffff);
        tile[rr][cc + 2 * e + 1] = (u16)(w[e] >> 16);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (r0 + rr < rows && c0 + cc + e < cols) tile[rr][cc + e] = in[(long long)(r0 + rr) * cols + c0 + cc + e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i;
    const int oc = idx >> 3, orr = (idx & 7) * 8;  // output row = input column oc, 8 input rows orr..
    if (full) {
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)tile[orr + 2 * e][oc] | ((unsigned)tile[orr + 2 * e + 1][oc] << 16);
      *reinterpret_cast<uint4*>(out + (long long)(c0 + oc) * rows + r0 + orr) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + oc < cols && r0 + orr + e < rows) out[(long long)(c0 + oc) * rows + r0 + orr + e] = tile[orr + e][oc];
    }
  }
}

hipError_t transpose_bf16(const void* in, void* out, int rows, int cols, hipStream_t stream) {
  dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, stream, static_cast<const u16*>(in),
                     static_cast<u16*>(out), rows, cols);
  return hipGetLastError();
}

// ------------------------------------------------------------------ row sums (bias gradients)
// out[r] (+)= sum_c in[r][c] for a bf16 [rows, cols] matrix: one wave per row, 16-B loads.
__global__ __launch_bounds__(256) void rowsum_bf16_kernel(const u16* __restrict__ in, float* __restrict__ out,
                                                          int rows, int cols, int accumulate) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= rows) return;
  const u16* p = in + (long long)row * cols;
  float s = 0.f;
  for (int c = l * 8; c < cols; c += 64 * 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + c);
    s += bf2f(v.x & 0xffff) + bf2f(v.x >> 16) + bf2f(v.y & 0xffff) + bf2f(v.y >> 16) + bf2f(v.z & 0xffff) +
         bf2f(v.z >> 16) + bf2f(v.w & 0xffff) + bf2f(v.w >> 16);
  }
  s = wave_sum(s);
  if (l == 0) out[row] = accumulate ? out[row] + s : s;
}

hipError_t rowsum_bf16(const void* in, float* out, int rows, int cols, int accumulate, hipStream_t stream) {
  if (cols % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rowsum_bf16_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, static_cast<const u16*>(in),
                     out, rows, cols, accumulate);
  return hipGetLastError();
}

// ------------------------------------------------------------------ BCE head
// z[b] = a[b,:] . w + b0; loss += mean BCE; dz = (sigmoid(z) - y) / B;
// g[b,:] = dz[b] * w * 1[a[b,:] > 0] (bf16, and g^T); dw += sum_b dz[b] a[b,:]; db += sum_b dz[b].
// Kernel 1: one wave per row computes z, loss, dz.  Kernel 2: per (row-block, col-block) tile
// writes g / g^T and accumulates dw with one atomic per column per block.
__global__ __launch_bounds__(256) void head_fwd_kernel(const u16* __restrict__ a, const float* __restrict__ w,
                                                       const float* __restrict__ b0, const float* __restrict__ y,
                                                       int B, int D, float* __restrict__ dz, float* __restrict__ db,
                                                       double* __restrict__ loss_acc) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= B) return;
  const u16* p = a + (long long)row * D;
  float s = 0.f;
  for (int c = l * 8; c < D; c += 64 * 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + c);
    const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) s += bf2f(u[e] & 0xffff) * w[c + 2 * e] + bf2f(u[e] >> 16) * w[c + 2 * e + 1];
  }
  s = wave_sum(s);
  if (l == 0) {
    const float z = s + *b0, yy = y[row];
    const float e = __expf(-fabsf(z));
    const float sig = z >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
    const float d = (sig - yy) / (float)B;
    dz[row] = d;
    atomicAdd(db, d);
    atomicAdd(loss_acc, (double)(((1.f - yy) * z - (fminf(z, 0.f) - log1pf(e))) / (float)B));
  }
}

__global__ __launch_bounds__(256) void head_bwd_kernel(const u16* __restrict__ a, const float* __restrict__ w,
                                                       const float* __restrict__ dz, int B, int D,
                                                       u16* __restrict__ g, u16* __restrict__ gT,
                                                       float* __restrict__ dw) {
  // block: 64 rows x 64 cols; thread t: col c = t & 63, rows (t >> 6) + 4i
  __shared__ u16 tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64, t = threadIdx.x;
  const int c = c0 + (t & 63);
  const float wc = w[c];
  float part = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rr = (t >> 6) + 4 * i, row = r0 + rr;
    const float av = bf2f(a[(long long)row * D + c]);
    const float d = dz[row];
    part += d * av;
    const u16 gv = f2bf(av > 0.f ? d * wc : 0.f);
    g[(long long)row * D + c] = gv;
    tile[rr][t & 63] = gv;
  }
  atomicAdd(&dw[c], part);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int cc = (t >> 6) + 4 * i, rr = t & 63;
    gT[(long long)(c0 + cc) * B + r0 + rr] = tile[rr][cc];
  }
}

hipError_t mlp_head(const HeadArgs& h, hipStream_t stream) {
  if (h.B % 64 || h.D % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_fwd_kernel, dim3((h.B + 3) / 4), dim3(256), 0, stream, static_cast<const u16*>(h.a), h.w,
                     h.b0, h.y, h.B, h.D, h.dz, h.db, h.loss_acc);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(h.D / 64, h.B / 64), dim3(256), 0, stream, static_cast<const u16*>(h.a),
                     h.w, h.dz, h.B, h.D, static_cast<u16*>(h.g), static_cast<u16*>(h.gT), h.dw);
  return hipGetLastError();
}

}  // namespace dgt
