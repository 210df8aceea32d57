// Exact-fp32 GEMM on the CDNA4 matrix cores (v_mfma_f32_16x16x4_f32) for the engine's fp32
// nn.Linear layers beyond the small-batch kernels of linear.hip ("bf16 + fp32").
//
//   C[M, N] (op)= epi( sum_k A(m, k) * B(n, k) )
//
// Each operand is read in whichever of its two row-major layouts it already has, so no Linear
// product needs a transposed copy:
//   A: LA = 0 "MK" A[m * lda + k]   (k contiguous)       LA = 1 "KM" A[k * lda + m]   (m contiguous)
//   B: LB = 0 "NK" B[n * ldb + k]                        LB = 1 "KN" B[k * ldb + n]
// The three products of a Linear layer y = x W^T + b (x [M, K], W [N, K], dy [M, N]):
//   forward  y  = x . W^T          A = x  (MK), B = W  (NK)     epilogue: + bias, ReLU
//   dgrad    dx = g . W            A = g  (MK), B = W  (KN)     g = dy * 1[y > 0] (ReLU mask on A)
//   wgrad    dW = g^T . x          A = g  (KM), B = x  (KN)     epilogue: accumulate into .grad
//
// Numerics: the f32-input MFMA is bitwise an fp32 fmaf chain (cdna_hip_programming.md §3 "FP32-input
// MFMA"): no TF32-style rounding of the inputs, so results agree with an fp32 reference to
// summation-order rounding only.
//
// Design (round 5; the LDS-staged 32x32x2 kernel with split-K it replaces ran 0.52x hipBLASLt at
// 1024^3, profiles/r4_gemm_f32_vs_hipblaslt.jsonl).  fp32 MFMA issues at 1/16 of the bf16 rate, so
// the kernel is bound by keeping every SIMD's matrix pipe fed, not by bytes: at 32 cycles per
// 16x16x4 MFMA a 64x64 wave tile consumes 8 KiB of operands per 2,048 MFMA cycles.  So:
//  * NO LDS staging and no barrier in the main loop: every wave loads its own MFMA fragments
//    straight from global memory (L2) into registers with 16-byte loads, one 16-deep k chunk ahead
//    of the MFMAs that consume them (two register stages, loads never waited on inside a chunk);
//  * the fragment layout follows the operand's memory layout, so every load is 16 bytes per lane.
//    The 16x16x4 MFMA takes one f32 per lane and operand (lane l: row l & 15, k-slot q = l >> 4);
//    over a 16-deep chunk lane quad q owns k = 4q + s for the chunk's four MFMA steps s:
//      - a k-contiguous operand (MK / NK): a lane loads its row's 4 k values (k = 4q .. 4q + 3) as
//        one float4, element s feeding step s; one load per 16-row tile (16 rows x 64 B);
//      - a row-contiguous operand (KM / KN): a lane loads 4 consecutive ROWS at k = 4q + s as one
//        float4, element e feeding the 16-row tile {r0 + 4i + e}: a 64-row group is four
//        interleaved tiles; one load per (64-row group, step) (4 k rows x 256 B);
//    the output tile of an interleaved column group keeps 4 adjacent columns in one lane, so a KN
//    product's epilogue stores float4s;
//  * the workgroup (4 waves) covers WGM x WGN wave tiles and splits K WGK ways; the K-split partial
//    tiles are summed once at the end through LDS in wave order (deterministic), each wave then
//    finishing 1/WGK of the tile's rows -- a small grid (1024^3: 64x64 tiles = 256 workgroups =
//    1,024 waves, one per SIMD) fills the chip without a split-K launch or a reduce kernel;
//  * smaller grids (fewer than 256 64x64 tiles) also split K across workgroups in the same launch
//    (gemm_f32_split; the last workgroup of a tile to arrive sums the partials in slice order);
//  * workgroup ids go through the XCD-aware remap (T1) so an XCD's workgroups share panels in L2.
// Reference: the fp32 nn.Linear layers of train.py:29-33 (forward train.py:107, backward :113).
#include <algorithm>

#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {
namespace f32g {

// ----------------------------------------------------------------------------- bias gradient
// part[s][n] = sum over rows m of slice s of dy[m][n] * (y ? 1[y[m][n] > 0] : 1); 64 columns x 4
// row lanes per block, rows strided by 4, combined in LDS in a fixed order.
__global__ __launch_bounds__(256) void colsum_f32_partial(const float* __restrict__ dy, const float* __restrict__ y,
                                                         float* __restrict__ part, int M, int N, int rows_per) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s = 0.f;
  if (n < N) {
    // unrolled so eight rows' loads are in flight before their (in-order) adds: one dependent
    // memory round trip per row made this kernel latency-bound (~7 us for 8 MB)
#pragma unroll 8
    for (int m = r0 + rl; m < r1; m += 4) {
      const long long off = (long long)m * N + n;
      const float d = dy[off];
      s += (y && !(y[off] > 0.f)) ? 0.f : d;
    }
  }
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) part[(long long)blockIdx.y * N + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

__global__ __launch_bounds__(256) void colsum_f32_final(const float* __restrict__ part, float* __restrict__ db,
                                                       int N, int slices, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int z = 0; z < slices; ++z) s += part[(long long)z * N + n];
  db[n] = accumulate ? db[n] + s : s;
}

}  // namespace f32g

hipError_t gemm_f32_l00(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream);
hipError_t gemm_f32_l01(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream);
hipError_t gemm_f32_l10(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream);
hipError_t gemm_f32_l11(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream);

GemmF32Plan gemm_f32_plan(int M, int N, int K, int force_cfg) {
  // the largest wave tile whose grid still puts a wave on every SIMD (256 CUs x 4 = 1,024 waves);
  // failing that, the configuration with the most waves (ties: the larger tile)
  struct C {
    int cfg, bm, bn;
  };
  const C cands[] = {{kF32Wave128, 256, 128}, {kF32Wave64, 128, 128}, {kF32Wave64Split2, 64, 128},
                     {kF32Wave64Split4, 64, 64}};
  GemmF32Plan p;
  if (force_cfg >= 0 && force_cfg < 4) {
    p.cfg = force_cfg;
    return p;
  }
  long long best_waves = -1;
  p.cfg = kF32Wave64Split4;
  for (const C& c : cands) {
    const long long waves = 4LL * ((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    if (waves >= 1024) {
      p.cfg = c.cfg;
      return p;
    }
    if (waves > best_waves) {
      best_waves = waves;
      p.cfg = c.cfg;
    }
  }
  (void)K;
  return p;
}

int gemm_f32_split(int M, int N, int K, const GemmF32Plan& p, int force) {
  // the 64x64 tile with its K split 4 ways inside the workgroup is the small-grid configuration;
  // when even it leaves SIMDs idle (tiles < 256: e.g. M = 256, N = 1024 is 64 tiles = 256 waves on
  // 1,024 SIMDs), split K across workgroups too, while every wave keeps >= 4 16-deep chunks.  At
  // most one workgroup per CU: two (the 64 KiB reduce buffer allows it) measured 1.5-1.9x slower
  // (profiles/r6_gemm_f32_split_k.jsonl)
  if (p.cfg != kF32Wave64Split4 || force == 0 || force == 1) return 1;
  const long long tiles = (long long)((M + 63) / 64) * ((N + 63) / 64);
  const int cap = force > 1 ? std::min(force, 8) : 8;  // (f32g::kF32MaxSplit)
  int s = 1;
  while (s < cap && tiles * s * 2 <= 256 && K / (16 * 4 * s * 2) >= 4) s *= 2;
  return s;
}

hipError_t gemm_f32(const GemmF32Args& a, int la, int lb, const GemmF32Plan& p, hipStream_t stream) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || la < 0 || la > 1 || lb < 0 || lb > 1) return hipErrorInvalidValue;
  // 16-byte loads need the contiguous extent, the leading dims and the bases aligned to 4 floats
  const int ca = la == 0 ? a.K : a.M, cb = lb == 0 ? a.K : a.N;
  const bool vec = (ca % 4 == 0) && (cb % 4 == 0) && (a.lda % 4 == 0) && (a.ldb % 4 == 0) &&
                   ((uintptr_t)a.A % 16 == 0) && ((uintptr_t)a.B % 16 == 0) &&
                   (a.maskA == nullptr || (uintptr_t)a.maskA % 16 == 0) && ((uintptr_t)a.C % 16 == 0) &&
                   (a.bias == nullptr || (uintptr_t)a.bias % 16 == 0) &&
                   (a.maskC == nullptr || (uintptr_t)a.maskC % 16 == 0);
  if (a.split > 1 && (p.cfg != kF32Wave64Split4 || a.rowsum || !a.sk_slab || !a.sk_flags)) return hipErrorInvalidValue;
  switch (la * 2 + lb) {
    case 0: return gemm_f32_l00(a, p, vec, stream);
    case 1: return gemm_f32_l01(a, p, vec, stream);
    case 3: return gemm_f32_l11(a, p, vec, stream);
    default: return gemm_f32_l10(a, p, vec, stream);
  }
}

int colsum_f32_slices(int M, int N) {
  const int cb = (N + 63) / 64;
  int s = 1;
  while (cb * s < 512 && M / (s * 2) >= 64) s *= 2;
  return s;
}

hipError_t colsum_f32(const float* dy, const float* y, float* db, float* part, int M, int N, int slices,
                      bool accumulate, hipStream_t stream) {
  if (M <= 0 || N <= 0 || slices <= 0) return hipErrorInvalidValue;
  const int rows_per = (M + slices - 1) / slices;
  hipLaunchKernelGGL(f32g::colsum_f32_partial, dim3((unsigned)((N + 63) / 64), (unsigned)slices), dim3(256), 0, stream,
                     dy, y, part, M, N, rows_per);
  hipLaunchKernelGGL(f32g::colsum_f32_final, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, stream, part, db, N,
                     slices, accumulate ? 1 : 0);
  return hipGetLastError();
}

}  // namespace dgt
