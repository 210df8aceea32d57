// Exact-fp32 GEMM on the CDNA4 matrix cores (v_mfma_f32_32x32x2_f32) for the engine's fp32
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
// Numerics: v_mfma_f32_32x32x2_f32 is bitwise an fp32 fmaf chain (cdna_hip_programming.md §3
// "FP32-input MFMA"): no TF32-style rounding of the inputs, so results agree with an fp32 reference
// to summation-order rounding only.
//
// Block: BM x BN (128 x 128 or 64 x 64), BK = 32, 256 threads = 4 waves in 2 x 2, each wave
// (BM/2) x (BN/2) = TM x TN 32 x 32 accumulators.  The MFMA takes ONE f32 per lane per operand:
// lane l holds A[row l & 31][k-slot l >> 5].  Every 8-deep k group is consumed as 4 MFMA steps in
// which lane half h takes physical k = 8g + 4h + s (s = 0..3), the same map for both operands, so:
//   an MK/NK tile sits in LDS as [row][32 k] (128-B rows) and a lane fetches its 4 k values of a
//     group with ONE ds_read_b128; the 16-B chunk is XOR-swizzled by (row >> 1) & 7, which makes
//     all four 16-lane groups of the b128 read conflict-free (checked exhaustively for the gfx950
//     lane groups of MI355X_MICROARCH.md §LDS);
//   a KM/KN tile sits in LDS as [32 k][rows] as it lies in memory, and a lane fetches k = 8g+4h+s
//     with ds_read_b32 (each 32-lane half reads 32 consecutive rows of one k: conflict-free).
// Staging is global -> VGPR -> LDS (16-B loads, zero-filled outside M / N / K, which is what makes
// ragged shapes exact), double-buffered: the next K-tile's loads are in flight while the current
// one feeds the MFMAs, one barrier per K-tile.  fp32 MFMA runs at 1/16 of the bf16 rate, so the
// staging path is far from the bound; what matters is keeping 2+ waves per SIMD (two 128x128 blocks
// or four 64x64 blocks per CU) and enough blocks for 256 CUs, hence the 64x64 tile and split-K for
// small grids.  Block ids go through the XCD-aware remap (T1) so an XCD's blocks share panels in L2.
// Reference: the fp32 nn.Linear layers of train.py:29-33 (forward train.py:107, backward :113).
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {
namespace f32g {

constexpr int BK = 32;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ----------------------------------------------------------------------------- staging
// One operand tile of ROWS rows x BK k.  MK form: ROWS*BK/4 16-byte chunks, chunk c of row r ->
// LDS [r][c ^ ((r >> 1) & 7)].  KM form: chunk = 4 consecutive rows of one k -> LDS [k][rows].
// load() only ISSUES the global loads (every load unconditional, out-of-range ones on a clamped
// in-range address, their lanes remembered in `oob`); store() zero-fills those lanes, applies the
// ReLU mask (MASKED) and writes LDS.  Nothing reads the loaded values until store(), so a tile's
// loads stay in flight while earlier tiles are consumed, and every path through the loop issues the
// same number of loads (the compiler's vmcnt accounting then keeps all prefetched tiles in flight).
template <bool KMAJ, int ROWS, bool VEC, bool MASKED, int NT>
struct Tile {
  static constexpr int CHUNKS = ROWS * BK / 4;
  static constexpr int PER = CHUNKS / NT;  // chunks per thread (NT threads)
  f32x4 v[PER];
  f32x4 m[MASKED ? PER : 1];
  unsigned oob;  // bit 4i+e: element e of chunk i is outside the operand

  DGT_DEVICE static void chunk_pos(int c, int& r, int& k) {
    if (!KMAJ) {
      r = c / (BK / 4);
      k = (c % (BK / 4)) * 4;
    } else {
      k = c / (ROWS / 4);
      r = (c % (ROWS / 4)) * 4;
    }
  }

  // rows [r0, r0 + ROWS) of the operand, k-tile [k0, k0 + BK); extent nr rows, nk k; ld elements
  DGT_DEVICE void load(const float* __restrict__ p, const float* __restrict__ mask, long long ld, int r0, int k0,
                       int nr, int nk, int tid) {
    oob = 0u;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int r, k;
      chunk_pos(tid + NT * i, r, k);
      const int gr = r0 + r, gk = k0 + k;
      if (VEC) {
        // the contiguous extent is a multiple of 4 here: a chunk is all in or all out
        const bool ok = gr < nr && gk < nk;
        const long long off = ok ? (KMAJ ? (long long)gk * ld + gr : (long long)gr * ld + gk) : 0;
        v[i] = *reinterpret_cast<const f32x4*>(p + off);
        if constexpr (MASKED) m[i] = *reinterpret_cast<const f32x4*>(mask + off);
        oob |= ok ? 0u : (15u << (4 * i));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = KMAJ ? gr + e : gr, kk = KMAJ ? gk : gk + e;
          const bool ok = rr < nr && kk < nk;
          const long long off = ok ? (KMAJ ? (long long)kk * ld + rr : (long long)rr * ld + kk) : 0;
          v[i][e] = p[off];
          if constexpr (MASKED) m[i][e] = mask[off];
          oob |= ok ? 0u : (1u << (4 * i + e));
        }
      }
    }
  }

  // rs (optional): per-chunk running sums of the stored values by operand row -- 4 rows of one k
  // (KMAJ) or one row's 4 k (MK); a thread's chunks sit at the same rows in every K-tile
  DGT_DEVICE void store(float* lds, int tid, f32x4* rs = nullptr) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + NT * i;
      int off;
      if (!KMAJ) {
        const int r = c / (BK / 4), ch = c % (BK / 4);
        off = r * BK + ((ch ^ ((r >> 1) & 7)) << 2);
      } else {
        off = c * 4;  // [k][ROWS], chunks in memory order
      }
      f32x4 x = v[i];
      // interior chunks (every chunk of an interior tile) need no select: the zero-fill is for the
      // ragged edges only, and the VALU it costs per K-tile showed up in the counters (PMC)
      if (MASKED || ((oob >> (4 * i)) & 15u) != 0u) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bool keep = !((oob >> (4 * i + e)) & 1u);
          if constexpr (MASKED) keep = keep && m[i][e] > 0.f;
          x[e] = keep ? x[e] : 0.f;
        }
      }
      *reinterpret_cast<f32x4*>(lds + off) = x;
      if (rs) rs[i] += x;
    }
  }
};

// A lane's 4 values (s = 0..3) of k group g for the 32-row MFMA tile starting at row rb.
template <bool KMAJ, int ROWS>
DGT_DEVICE f32x4 frag(const float* lds, int rb, int g, int lane) {
  const int r = rb + (lane & 31), h = lane >> 5;
  if (!KMAJ) {
    const int ch = 2 * g + h;
    return *reinterpret_cast<const f32x4*>(lds + r * BK + ((ch ^ ((r >> 1) & 7)) << 2));
  } else {
    const int k = 8 * g + 4 * h;
    f32x4 x;
#pragma unroll
    for (int s = 0; s < 4; ++s) x[s] = lds[(k + s) * ROWS + r];
    return x;
  }
}

// XCD-aware bijective remap (T1): blocks b and b + 8 run on one XCD; each XCD gets a contiguous run
// of tile ids, walked in groups of GROUP block-rows so neighbours reuse B panels in the XCD's L2.
DGT_DEVICE void tile_of(int bid, int nbm, int nbn, int& tm, int& tn) {
  const int nwg = nbm * nbn, xcd = bid % 8, q = nwg / 8, rm = nwg % 8;
  const int wgid = (xcd < rm ? xcd * (q + 1) : rm * (q + 1) + (xcd - rm) * q) + bid / 8;
  constexpr int GROUP = 8;
  const int group = wgid / (GROUP * nbn), first = group * GROUP;
  const int gsize = min(nbm - first, GROUP);
  tm = first + (wgid % (GROUP * nbn)) % gsize;
  tn = (wgid % (GROUP * nbn)) / gsize;
}

// grid.x = tiles, grid.y = split-K slices.  Split slices write raw partial sums to ws[z][M][N]
// (epilogue in gemm_f32_splitk_reduce); an unsplit launch applies the epilogue itself.
template <int LA, int LB, int BM, int BN, bool VEC, bool MASKED, int NT>
__global__ __launch_bounds__(NT, 2) void gemm_f32_kernel(GemmF32Args a) {
  // NT = 256: 4 waves in 2 x 2; NT = 512: 8 waves in 2 x 4 (each wave BM/2 x BN/4: four waves per
  // SIMD at two blocks per CU, so one wave's staging and barrier wait hide behind three others' MFMAs).
  // (A form with two in-block k groups for the 64 x 64 tile, summed through LDS, gave wrong input
  // gradients inside the fp32 engine chain while passing the isolated product tests: removed.)
  constexpr int NW = NT / 64, WCOLS = NW / 2;
  constexpr int WM = BM / 2, WN = BN / WCOLS, TM = WM / 32, TN = WN / 32;
  static_assert(TN >= 1 && TM >= 1, "fp32 GEMM wave tile below one 32x32 MFMA");
  constexpr int A_SZ = BM * BK, B_SZ = BN * BK;
  __shared__ __attribute__((aligned(16))) float lds[2][A_SZ + B_SZ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WCOLS, wn = wave % WCOLS;
  const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
  int tm, tn;
  tile_of(blockIdx.x, nbm, nbn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  // this slice's k range (whole K-tiles)
  const int ktiles = (a.K + BK - 1) / BK;
  const int per = (ktiles + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per, kt1 = min(ktiles, kt0 + per);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // P K-tiles of loads in flight in registers, two LDS stages, one barrier per K-tile (2 K-tiles in
  // flight for the 64x64 tile too: the fp32 engine MLP 2,551-2,562 iters/s against 2,410-2,465 with
  // 3; compiled for 4 blocks per CU instead, 2,530-2,558: r4_gemm_f32_occ4_ab.txt): iteration i
  // writes tile i + 1 into the stage tile i - 1 was read from, refills its registers with tile
  // i + 1 + P (clamped to the slice: re-reads of the last tile, never consumed), then consumes tile i.
  constexpr int P = 2;
  Tile<LA == 1, BM, VEC, MASKED, NT> ta[P];
  Tile<LB == 1, BN, VEC, false, NT> tb[P];
  const int nkt = kt1 - kt0;
  auto load = [&](int p, int i) {
    const int kt = kt0 + min(i, nkt - 1);
    ta[p].load(a.A, a.maskA, a.lda, m0, kt * BK, a.M, a.K, tid);
    tb[p].load(a.B, nullptr, a.ldb, n0, kt * BK, a.N, a.K, tid);
  };
  // fused row sums of the masked A (the bias gradient): the blocks of the first column tile add
  // every K-tile they stage (tiles staged past the slice's end are clamped re-reads: skipped)
  const bool rs_on = a.rowsum != nullptr && tn == 0;
  constexpr int APER = Tile<LA == 1, BM, VEC, MASKED, NT>::PER;
  f32x4 rsum[APER];
#pragma unroll
  for (int i = 0; i < APER; ++i) rsum[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int p, int buf, bool counted = false) {
    ta[p].store(lds[buf], tid, counted && rs_on ? rsum : nullptr);
    tb[p].store(lds[buf] + A_SZ, tid);
  };
  // the k groups' fragments are read one group ahead: group g + 1's LDS reads are in flight while
  // group g's MFMAs run (reading each group just before its MFMAs left the waves waiting on LDS
  // ~30x as long as hipBLASLt's: SQ_WAIT_INST_LDS, profiles/r4_gemm_f32_pmc.txt)
  auto consume = [&](int buf) {
    const float* la = lds[buf];
    const float* lb = lds[buf] + A_SZ;
    f32x4 fa[2][TM], fb[2][TN];
    auto read = [&](int g, int d) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[d][i] = frag<LA == 1, BM>(la, wm * WM + 32 * i, g, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[d][j] = frag<LB == 1, BN>(lb, wn * WN + 32 * j, g, lane);
    };
    constexpr int GPK = BK / 8;  // k groups of the K-tile
    read(0, 0);
#pragma unroll
    for (int gi = 0; gi < GPK; ++gi) {
      if (gi + 1 < GPK) read(gi + 1, (gi + 1) & 1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[gi & 1][i][s], fb[gi & 1][j][s], acc[i][j], 0, 0, 0);
    }
  };
  // (the loop sits inside the nkt > 0 branch: a path into the loop header that skipped the prologue
  // loads would make the compiler wait for every prefetched tile at the header)
  if (nkt > 0) {
    // the prologue's loads stay in tile order (sched_barrier): the loop header's wait counts assume
    // the oldest tile in flight is the one staged next
#pragma unroll
    for (int p = 0; p < P; ++p) {
      load(p, p);
      __builtin_amdgcn_sched_barrier(0);
    }
    stage(0, 0, true);
    load(0, P);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    // whole groups of P iterations: the ones past the slice stage and load (clamped) but consume
    // nothing -- a `break` would again give the header a path with fewer loads in flight
    for (int i0 = 0; i0 < nkt; i0 += P) {
#pragma unroll
      for (int d = 0; d < P; ++d) {
        const int i = i0 + d;
        const int nx = (d + 1) % P;  // static after the unroll
        stage(nx, (i + 1) & 1, i + 1 < nkt);
        load(nx, i + 1 + P);
        if (i < nkt) consume(i & 1);
        __syncthreads();
      }
    }
  }

  if (a.rowsum != nullptr && tn == 0) {
    // the block's row sums: each thread's per-chunk sums go to the chunk's own LDS slots (the staging
    // image: [k][rows] for KMAJ, [row][k] swizzled for MK), then one thread per row adds its BK (KMAJ)
    // or BK / 4 (MK) slots in k order; slice partials go to ws after the C partials
    if (nkt <= 0) __syncthreads();
    float* red = &lds[0][0];
    constexpr bool AK = LA == 1;
    using TA = Tile<AK, BM, VEC, MASKED, NT>;
#pragma unroll
    for (int i = 0; i < TA::PER; ++i) {
      const int c = tid + NT * i;
      if (AK) {
        *reinterpret_cast<f32x4*>(red + c * 4) = rsum[i];
      } else {
        red[c] = (rsum[i][0] + rsum[i][1]) + (rsum[i][2] + rsum[i][3]);
      }
    }
    __syncthreads();
    if (tid < BM && m0 + tid < a.M) {
      float t = 0.f;
      if (AK) {
        for (int k = 0; k < BK; ++k) t += red[k * BM + tid];
      } else {
        for (int q = 0; q < BK / 4; ++q) t += red[tid * (BK / 4) + q];
      }
      if (gridDim.y > 1) {
        a.ws[(long long)gridDim.y * a.M * a.N + (long long)blockIdx.y * a.M + m0 + tid] = t;
      } else {
        float* d = a.rowsum + m0 + tid;
        *d = a.accumulate ? *d + t : t;
      }
    }
    __syncthreads();  // the LDS is reused below
  }
  // epilogue: 32x32 accumulator layout col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  const bool split = gridDim.y > 1;
  float* out = split ? a.ws + (long long)blockIdx.y * a.M * a.N : a.C;
  const long long ldo = split ? a.N : a.ldc;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + 32 * j + (lane & 31);
    if (n >= a.N) continue;
    const float bias = (!split && a.bias) ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * WM + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m >= a.M) continue;
        float v = acc[i][j][e];
        float* dst = out + (long long)m * ldo + n;
        if (!split) {
          v += bias;
          if (a.relu) v = fmaxf(v, 0.f);
          if (a.maskC && !(a.maskC[(long long)m * a.N + n] > 0.f)) v = 0.f;
          if (a.accumulate) v += *dst;
        }
        *dst = v;
      }
    }
  }
}

// C = epi(sum over z of ws[z]) in slice order (deterministic), 4 consecutive elements of one row per
// thread with 16-byte accesses (N and ldc multiples of 4, C 16-byte aligned): every slice's load is in
// flight before the sum, one row / column split per thread instead of a 64-bit division per element
// (the scalar form below ran at ~2.5 TB/s, 13 launches = 105 us of the fp32 engine MLP step).
// Bitwise the scalar form: the same left-to-right slice order from 0.
// rowsum[m] (+)= the slices' row sums in slice order (the fused bias gradient, gemm_f32_kernel)
DGT_DEVICE void reduce_rowsum(const GemmF32Args& a, int splits) {
  const long long m = (long long)blockIdx.x * 256 + threadIdx.x;
  if (a.rowsum == nullptr || m >= a.M) return;
  const float* p = a.ws + (long long)splits * a.M * a.N + m;
  float t = 0.f;
  for (int z = 0; z < splits; ++z) t += p[(long long)z * a.M];
  a.rowsum[m] = a.accumulate ? a.rowsum[m] + t : t;
}

template <int SPLITS>
__global__ __launch_bounds__(256) void gemm_f32_splitk_reduce4(GemmF32Args a) {
  reduce_rowsum(a, SPLITS);
  const long long total = (long long)a.M * a.N;
  const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= total) return;
  const int m = (int)(i0 / a.N), n = (int)(i0 - (long long)m * a.N);
  f32x4 w[SPLITS];
#pragma unroll
  for (int z = 0; z < SPLITS; ++z) w[z] = *reinterpret_cast<const f32x4*>(a.ws + (long long)z * total + i0);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};  // from +0, as the scalar form (a -0 partial sums to +0 alike)
#pragma unroll
  for (int z = 0; z < SPLITS; ++z) v += w[z];
  if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + n);
  if (a.relu) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if (a.maskC) {
    const f32x4 mk = *reinterpret_cast<const f32x4*>(a.maskC + i0);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
  }
  f32x4* dst = reinterpret_cast<f32x4*>(a.C + (long long)m * a.ldc + n);
  if (a.accumulate) v += *dst;
  *dst = v;
}

// scalar form: any N / ldc / alignment
__global__ __launch_bounds__(256) void gemm_f32_splitk_reduce(GemmF32Args a, int splits) {
  reduce_rowsum(a, splits);
  const long long total = (long long)a.M * a.N;
  const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= total) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long i = i0 + e;
    if (i >= total) break;
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += a.ws[(long long)z * total + i];
    const int m = (int)(i / a.N), n = (int)(i % a.N);
    if (a.bias) v += a.bias[n];
    if (a.relu) v = fmaxf(v, 0.f);
    if (a.maskC && !(a.maskC[i] > 0.f)) v = 0.f;
    float* dst = a.C + (long long)m * a.ldc + n;
    if (a.accumulate) v += *dst;
    *dst = v;
  }
}

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

template <int LA, int LB, int BM, int BN, bool MASKED, int NT>
void launch_masked(const GemmF32Args& a, bool vec, const dim3& grid, hipStream_t stream) {
  if (vec)
    hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, BM, BN, true, MASKED, NT>), grid, dim3(NT), 0, stream, a);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, BM, BN, false, MASKED, NT>), grid, dim3(NT), 0, stream, a);
}

template <int LA, int LB, int BM, int BN, int NT>
hipError_t launch(const GemmF32Args& a, bool vec, int splits, hipStream_t stream) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  if (a.maskA)
    launch_masked<LA, LB, BM, BN, true, NT>(a, vec, grid, stream);
  else
    launch_masked<LA, LB, BM, BN, false, NT>(a, vec, grid, stream);
  return hipGetLastError();
}

template <int LA, int LB>
hipError_t dispatch(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream) {
  if (!p.big) return launch<LA, LB, 64, 64, 256>(a, vec, p.splits, stream);
  return p.threads == 512 ? launch<LA, LB, 128, 128, 512>(a, vec, p.splits, stream)
                          : launch<LA, LB, 128, 128, 256>(a, vec, p.splits, stream);
}

}  // namespace f32g

GemmF32Plan gemm_f32_plan(int M, int N, int K, int min_blocks) {
  GemmF32Plan p;
  const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128);
  const long long t64 = (long long)((M + 63) / 64) * ((N + 63) / 64);
  p.big = t128 >= 256;  // a full wave of 128x128 blocks; else 4x the blocks at 64x64
  const long long tiles = p.big ? t128 : t64;
  const int ktiles = (K + f32g::BK - 1) / f32g::BK;
  p.splits = 1;
  // small grid, long K (e.g. a wgrad whose reduction runs over a large batch): split K so the
  // launch covers the chip with 2 blocks per CU -- more blocks in flight measured faster in the fp32
  // engine step even where a hot repeat of one product is not, and 2 beat 1 and 4 for the 64x64
  // tiles once the reduce was vectorised (profiles/r4_gemm_f32_split_ab.txt); partial sums are
  // combined in slice order (deterministic)
  if (min_blocks <= 0) min_blocks = 512;
  p.threads = 512;
  while (tiles * p.splits < min_blocks && ktiles / (2 * p.splits) >= 8 && p.splits < 16) p.splits *= 2;
  return p;
}

hipError_t gemm_f32(const GemmF32Args& a, int la, int lb, const GemmF32Plan& p, hipStream_t stream) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || la < 0 || la > 1 || lb < 0 || lb > 1) return hipErrorInvalidValue;
  if (p.splits > 1 && a.ws == nullptr) return hipErrorInvalidValue;
  // 16-byte loads need the contiguous extent, the leading dims and the bases aligned to 4 floats
  const int ca = la == 0 ? a.K : a.M, cb = lb == 0 ? a.K : a.N;
  const bool vec = (ca % 4 == 0) && (cb % 4 == 0) && (a.lda % 4 == 0) && (a.ldb % 4 == 0) &&
                   ((uintptr_t)a.A % 16 == 0) && ((uintptr_t)a.B % 16 == 0) &&
                   (a.maskA == nullptr || (uintptr_t)a.maskA % 16 == 0);
  hipError_t e;
  const int code = la * 2 + lb;
  switch (code) {
    case 0: e = f32g::dispatch<0, 0>(a, p, vec, stream); break;
    case 1: e = f32g::dispatch<0, 1>(a, p, vec, stream); break;
    case 3: e = f32g::dispatch<1, 1>(a, p, vec, stream); break;
    default: e = f32g::dispatch<1, 0>(a, p, vec, stream); break;
  }
  if (e != hipSuccess || p.splits == 1) return e;
  const long long total = (long long)a.M * a.N;
  // (the row sums take one thread per row of C: enough blocks for M rows when N < 4)
  const dim3 grid((unsigned)std::max((total + 1023) / 1024, a.rowsum ? ((long long)a.M + 255) / 256 : 0LL));
  const bool v4 = a.N % 4 == 0 && a.ldc % 4 == 0 && (uintptr_t)a.C % 16 == 0 && (uintptr_t)a.ws % 16 == 0 &&
                  (a.bias == nullptr || (uintptr_t)a.bias % 16 == 0) &&
                  (a.maskC == nullptr || (uintptr_t)a.maskC % 16 == 0);
  switch (v4 ? p.splits : 0) {
    case 2: hipLaunchKernelGGL(f32g::gemm_f32_splitk_reduce4<2>, grid, dim3(256), 0, stream, a); break;
    case 4: hipLaunchKernelGGL(f32g::gemm_f32_splitk_reduce4<4>, grid, dim3(256), 0, stream, a); break;
    case 8: hipLaunchKernelGGL(f32g::gemm_f32_splitk_reduce4<8>, grid, dim3(256), 0, stream, a); break;
    case 16: hipLaunchKernelGGL(f32g::gemm_f32_splitk_reduce4<16>, grid, dim3(256), 0, stream, a); break;
    default: hipLaunchKernelGGL(f32g::gemm_f32_splitk_reduce, grid, dim3(256), 0, stream, a, p.splits);
  }
  return hipGetLastError();
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
