// Exact-fp32 MFMA GEMM kernel templates (see gemm_f32.hip for the design); instantiated per
// operand-layout pair in gemm_f32_l{LA}{LB}.hip so the four pairs compile in parallel.
#pragma once
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {
namespace f32g {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
constexpr int kF32MaxSplit = 8;  // gemm_f32_split's cap

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

// One operand's fragments for one KC = 16 H deep k chunk (H = 2: the K-split-4 64x64 tile of small
// grids keeps H = 1, twice the chunks per short K slice): f[h][t][s] = the value this lane feeds
// tile t at MFMA step s of the chunk's 16-deep half h.  T = 16-row tiles of the wave tile.
template <int T, int H>
struct Frag {
  f32x4v f[H][T];
};

// Loads one operand's fragments of the chunk starting at k = kc.
//   KROW = false (k-contiguous, MK / NK): tile t rows r0 + 16t + i; lane (i, q) loads
//          P[row * ld + kc + 16h + 4q .. + 3] -> f[h][t][s]; a row's two halves are issued back to
//          back, so each 128-byte line of it is fetched by two adjacent loads (one L2 request)
//   KROW = true (row-contiguous, KM / KN): group G rows r0 + 64G + 4i + e; lane (i, q) loads
//          P[(kc + 16h + 4q + s) * ld + r0 + 64G + 4i .. + 3] -> f[h][4G + e][s]
// VEC: 16-byte loads (contiguous extent, ld and base multiples of 4 floats); rows past `nr` are
// clamped to valid memory and only feed outputs that are never stored.  CHECK: the chunk may pass
// `nk` (the K tail): elements with k >= nk are zero.  !VEC: element loads with full bounds checks.
// MASK: the ReLU mask of a backward (same layout / ld as P): elements where mask <= 0 are zero.
template <bool KROW, int T, int H, bool VEC, bool CHECK, bool MASK>
DGT_DEVICE void load_frag(Frag<T, H>& fr, const float* __restrict__ P, const float* __restrict__ mask, long long ld,
                          int r0, int nr, int kc, int nk, int lane) {
  const int i = lane & 15, q = lane >> 4;
  if constexpr (!KROW) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = min(r0 + 16 * t + i, nr - 1);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int k = kc + 16 * h + 4 * q;
        if constexpr (VEC) {
          const long long off = (long long)row * ld + (CHECK ? min(k, nk - 4) : k);
          f32x4v v = *reinterpret_cast<const f32x4v*>(P + off);
          if constexpr (MASK) {
            const f32x4v mk = *reinterpret_cast<const f32x4v*>(mask + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
          }
          if constexpr (CHECK) {
            if (k >= nk) v = f32x4v{0.f, 0.f, 0.f, 0.f};
          }
          fr.f[h][t] = v;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const bool ok = k + s < nk;
            const long long off = ok ? (long long)row * ld + k + s : 0;
            float v = P[off];
            if constexpr (MASK) v = mask[off] > 0.f ? v : 0.f;
            fr.f[h][t][s] = ok ? v : 0.f;
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int G = 0; G < T / 4; ++G) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = kc + 16 * h + 4 * q + s;
          const int kk = CHECK ? min(k, nk - 1) : k;
          const int r = r0 + 64 * G + 4 * i;
          if constexpr (VEC) {
            const long long off = (long long)kk * ld + min(r, nr - 4);
            f32x4v v = *reinterpret_cast<const f32x4v*>(P + off);
            if constexpr (MASK) {
              const f32x4v mk = *reinterpret_cast<const f32x4v*>(mask + off);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
            }
            if constexpr (CHECK) {
              if (k >= nk) v = f32x4v{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) fr.f[h][4 * G + e][s] = v[e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool ok = k < nk && r + e < nr;
              const long long off = ok ? (long long)k * ld + r + e : 0;
              float v = P[off];
              if constexpr (MASK) v = mask[off] > 0.f ? v : 0.f;
              fr.f[h][4 * G + e][s] = ok ? v : 0.f;
            }
          }
        }
      }
    }
  }
}

// operand row of 16-row tile t, row x (0..15) within it
template <bool KROW>
DGT_DEVICE int row_of(int r0, int t, int x) {
  return KROW ? r0 + 64 * (t >> 2) + 4 * x + (t & 3) : r0 + 16 * t + x;
}

// The wave tile is WTM x WTN (16-row tiles TM x TN); the workgroup's 4 waves are WGM x WGN wave
// tiles x WGK K-slices.  acc[t][u] = the 16x16 output tile of A-tile t and B-tile u; its C/D layout
// (16x16x4 f32): register r of lane l is row 4 (l >> 4) + r, column l & 15 of the tile.
// SPK: a.split workgroups per tile (blocks tile * split + slice), K cut into split * WGK wave slices;
// after the in-workgroup sum each workgroup parks its 64x64 partial (16 KiB) in a.sk_slab with
// write-through (sc1) stores and bumps the tile's counter; the last to arrive sums the partials in
// slice order (the same bits whoever arrives last), re-arms the counter and runs the epilogue --
// the pattern of the bf16 small-grid split-K (gemm.hip gemm_nt_kernel SPK).
template <int LA, int LB, int WTM, int WTN, int WGM, int WGN, int WGK, int H, bool VEC, bool MASKED, bool ROWSUM,
          bool SPK = false>
__global__ __launch_bounds__(256, 1) void gemm_f32_kernel(GemmF32Args a) {
  constexpr int TM = WTM / 16, TN = WTN / 16, BM = WGM * WTM, BN = WGN * WTN;
  constexpr bool AK = LA == 1, BK = LB == 1;  // row-contiguous operands
  static_assert(WGM * WGN * WGK == 4, "4 waves per workgroup");
  static_assert((!AK || TM % 4 == 0) && (!BK || TN % 4 == 0), "row-contiguous tiles come in 64-row groups");
  static_assert(!SPK || (WTM == 64 && WTN == 64 && WGK == 4 && VEC && !ROWSUM), "split-K: the 64x64 K-split-4 tile");
  // (the wave index through readfirstlane: every per-wave quantity below is a scalar)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wk = wave % WGK, wmn = wave / WGK, wm = wmn / WGN, wn = wmn % WGN;
  const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
  const int split = SPK ? a.split : 1;
  const int tile = SPK ? (int)blockIdx.x / split : (int)blockIdx.x, slice = SPK ? (int)blockIdx.x % split : 0;
  int tm, tn;
  tile_of(tile, nbm, nbn, tm, tn);
  const int m0 = tm * BM + wm * WTM, n0 = tn * BN + wn * WTN;
  // this wave's K slice, in whole KC-deep chunks; a partial last chunk (K % KC) is peeled below
  constexpr int KC = 16 * H;
  const int nfull = a.K / KC, ntot = (a.K + KC - 1) / KC;
  const int per = (ntot + WGK * split - 1) / (WGK * split);
  const int c0 = (slice * WGK + wk) * per, c1 = min(ntot, c0 + per);
  const int f1 = max(c0, min(c1, nfull));  // [c0, f1): full chunks; [f1, c1): at most the partial chunk

  f32x4v acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[t][u] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const bool rs_on = ROWSUM && tn == 0 && wn == 0;
  // per-lane partial row sums of the (masked) A rows this lane loads: KM: rows 64G + 4i + e, MK:
  // rows 16t + i (summed over the lane's k values)
  f32x4v rs[ROWSUM ? TM : 1];
#pragma unroll
  for (int t = 0; t < (ROWSUM ? TM : 1); ++t) rs[t] = f32x4v{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const Frag<TM, H>& fa, const Frag<TN, H>& fb) {
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa.f[h][t][s], fb.f[h][u][s], acc[t][u], 0, 0, 0);
    if constexpr (ROWSUM) {
      if (rs_on) {
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
          for (int t = 0; t < TM; ++t) rs[t] += fa.f[h][t];
      }  // KM: (G, e) rows by step; MK: row t by k
    }
  };
  auto load = [&](Frag<TM, H>& fa, Frag<TN, H>& fb, int c) {
    load_frag<AK, TM, H, VEC, false, MASKED>(fa, a.A, a.maskA, a.lda, m0, a.M, KC * c, a.K, lane);
    load_frag<BK, TN, H, VEC, false, false>(fb, a.B, nullptr, a.ldb, n0, a.N, KC * c, a.K, lane);
  };

  if (c0 < f1) {
    // two register stages of KC-deep chunks: chunk c + 1 is in flight while chunk c's MFMAs run
    // (8,192 MFMA cycles per chunk for a 128x64 wave tile, 4,096 for 64x64); the loads past the
    // slice re-read its last chunk (clamped, never consumed), so every path issues the same loads
    // and the compiler's vmcnt accounting keeps the prefetch in flight.  Pairs of chunks with no
    // condition inside (a consumer under a branch lets the compiler sink the prefetch into that
    // branch, right in front of its MFMAs); sched_barrier keeps each load group in front of the
    // MFMAs it must overlap (left alone, the scheduler moves loads down next to their consumers to
    // shorten register lifetimes, exposing the load latency every chunk).  (Spreading the loads one
    // per R MFMAs instead, with sched_group_barrier, measured level: profiles/r5_gemm_f32_interleave_ab.txt)
    Frag<TM, H> fa0, fa1;
    Frag<TN, H> fb0, fb1;
    load(fa0, fb0, c0);
    int c = c0;
    for (; c + 1 < f1; c += 2) {
      load(fa1, fb1, c + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      load(fa0, fb0, min(c + 2, f1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      mma(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c < f1) mma(fa0, fb0);  // an odd chunk count: the last one is already in stage 0
  }
  if (f1 < c1) {  // the partial chunk of the K tail
    Frag<TM, H> fa;
    Frag<TN, H> fb;
    load_frag<AK, TM, H, VEC, true, MASKED>(fa, a.A, a.maskA, a.lda, m0, a.M, KC * f1, a.K, lane);
    load_frag<BK, TN, H, VEC, true, false>(fb, a.B, nullptr, a.ldb, n0, a.N, KC * f1, a.K, lane);
    mma(fa, fb);
  }

  // ---- K-slice partials: every wave parks its tile in LDS, then wave wk of each (wm, wn) sums the
  // WGK slices in slice order for the row tiles t = wk (mod WGK)
  constexpr int NACC = TM * TN * 4;
  // (static LDS: a workgroup may declare up to 160 KiB on gfx950)
  constexpr int RED_FLOATS = (WGK > 1 ? 4 * NACC * 64 : 0) + (ROWSUM ? 4 * TM * 4 * 64 : 0);
  __shared__ __attribute__((aligned(16))) float red[RED_FLOATS > 0 ? RED_FLOATS : 1];
  if constexpr (WGK > 1) {
    // one 16-byte LDS access per accumulator tile and lane ([wave][tile][lane] x float4)
    f32x4v* red4 = reinterpret_cast<f32x4v*>(red);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u) red4[((size_t)wave * TM * TN + t * TN + u) * 64 + lane] = acc[t][u];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (t % WGK != wk) continue;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        f32x4v v = {0.f, 0.f, 0.f, 0.f};  // slice order from +0 (deterministic)
#pragma unroll
        for (int k = 0; k < WGK; ++k) v += red4[((size_t)(wmn * WGK + k) * TM * TN + t * TN + u) * 64 + lane];
        acc[t][u] = v;
      }
    }
  }

  if constexpr (SPK) {
    // wave wk holds row tile t = wk of the workgroup's partial: [wave][u][lane] x float4 (picked out
    // with compile-time indices: acc[wk] would put the whole accumulator array in scratch)
    f32x4v own[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t)
      if (t == wk) {
#pragma unroll
        for (int u = 0; u < TN; ++u) own[u] = acc[t][u];
      }
    auto part = [&](int z) {
      return __builtin_amdgcn_make_buffer_rsrc(a.sk_slab + ((long long)tile * split + z) * (WTM * WTN), 0,
                                               WTM * WTN * 4, 0x00020000);
    };
    const auto mine = part(slice);
#pragma unroll
    for (int u = 0; u < TN; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, own[u]), mine,
                                             ((wave * TN + u) * 64 + lane) * 16, 0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();                                   // (and every wave is done reading `red`)
    int* word = reinterpret_cast<int*>(red);
    if (threadIdx.x == 0) *word = __hip_atomic_fetch_add(a.sk_flags + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*word != split - 1) return;  // not the last slice to arrive
    if (threadIdx.x == 0) __hip_atomic_store(a.sk_flags + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every load of a partial is an sc1 load behind the counter's add and the barrier above
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // every partial's loads are issued before the first add (own slot included: this workgroup's
    // stores drained above), so the cross-XCD round trips overlap instead of running one per slice
    f32x4v p[kF32MaxSplit][TN];
#pragma unroll
    for (int z = 0; z < kF32MaxSplit; ++z)
      if (z < split) {
        const auto rs = part(z);
#pragma unroll
        for (int u = 0; u < TN; ++u)
          p[z][u] = __builtin_bit_cast(
              f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rs, ((wave * TN + u) * 64 + lane) * 16, 0, 16));
      }
    f32x4v sum[TN];
#pragma unroll
    for (int u = 0; u < TN; ++u) sum[u] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < kF32MaxSplit; ++z)  // slice order: the same bits whoever arrived last
      if (z < split) {
#pragma unroll
        for (int u = 0; u < TN; ++u) sum[u] += p[z][u];
      }
#pragma unroll
    for (int t = 0; t < TM; ++t)
      if (t == wk) {
#pragma unroll
        for (int u = 0; u < TN; ++u) acc[t][u] = sum[u];
      }
  }

  // ---- row sums (the wgrad's bias gradient): lanes of one row sum over k quads q, then slices
  if (ROWSUM && tn == 0) {
    float* rsl = red + (WGK > 1 ? 4 * NACC * 64 : 0);  // [wave][TM * 4][64], after the K-slice partials
    if (wn == 0) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) rsl[((size_t)wave * TM * 4 + t * 4 + e) * 64 + lane] = rs[ROWSUM ? t : 0][e];
    }
    __syncthreads();
    if (wn == 0 && wk == 0) {
      // per lane (i, q): KM: rs[4G + e][s] summed the step-s values of row 64G + 4i + e; MK: rs[t][s]
      // the k = 4q + s values of row 16t + i.  Lane `lane` finishes rows lane, lane + 64, ... of the
      // wave tile, over k quads q and K slices in a fixed order.
      for (int x = lane; x < WTM; x += 64) {
        int t, i;
        if (AK) {
          t = 4 * (x >> 6) + (x & 3);
          i = (x & 63) >> 2;
        } else {
          t = x >> 4;
          i = x & 15;
        }
        float tot = 0.f;
        for (int k = 0; k < WGK; ++k)
          for (int q = 0; q < 4; ++q) {
            const float* p = rsl + ((size_t)(wmn * WGK + k) * TM * 4 + t * 4) * 64 + 16 * q + i;
            tot += ((p[0] + p[64]) + (p[128] + p[192]));
          }
        const int m = m0 + x;
        if (m < a.M) {
          float* d = a.rowsum + m;
          *d = a.accumulate ? *d + tot : tot;
        }
      }
    }
  }

  // ---- epilogue: bias, ReLU, output mask, accumulate, as float4s of 4 adjacent columns where C's
  // row stride allows: a KN product's interleaved column tiles already hold 4 adjacent columns per
  // lane; an NK product's 16x16 tile holds one column per lane, so each quad of lanes transposes
  // its 4x4 blocks first (two DPP butterflies: lane b of a quad then holds row 4q + b, the quad's 4
  // columns) -- a quarter of the store instructions of per-column stores
  const int q = lane >> 4, j = lane & 15;
  const bool c4 = VEC && (a.N & 3) == 0 && (a.ldc & 3) == 0 && (a.maskC == nullptr || ((uintptr_t)a.maskC & 15) == 0);
  auto store4 = [&](int m, int n, f32x4v v) {
    float* crow = a.C + (long long)m * a.ldc;
    if (a.bias) v += *reinterpret_cast<const f32x4v*>(a.bias + n);
    if (a.relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (a.maskC) {
      const f32x4v mk = *reinterpret_cast<const f32x4v*>(a.maskC + (long long)m * a.N + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
    }
    f32x4v* dst = reinterpret_cast<f32x4v*>(crow + n);
    if (a.accumulate) v += *dst;
    *dst = v;
  };
  auto store1 = [&](int m, int n, float x) {
    float* crow = a.C + (long long)m * a.ldc;
    if (a.bias) x += a.bias[n];
    if (a.relu) x = fmaxf(x, 0.f);
    if (a.maskC && !(a.maskC[(long long)m * a.N + n] > 0.f)) x = 0.f;
    if (a.accumulate) x += crow[n];
    crow[n] = x;
  };
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    if (WGK > 1 && t % WGK != wk) continue;
    if constexpr (BK) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row_of<AK>(m0, t, 4 * q + r);
        if (m >= a.M) continue;
#pragma unroll
        for (int G = 0; G < TN / 4; ++G) {
          const int n = n0 + 64 * G + 4 * j;
          const f32x4v v = {acc[t][4 * G][r], acc[t][4 * G + 1][r], acc[t][4 * G + 2][r], acc[t][4 * G + 3][r]};
          if (c4) {
            if (n < a.N) store4(m, n, v);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < a.N) store1(m, n + e, v[e]);
          }
        }
      }
    } else if (c4) {
      const int b = j & 3;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        f32x4v x = acc[t][u];
        // 4x4 transpose within the quad: M[lane b][reg r] = (row r, col b) -> T[lane b][c] = M[c][b]
        f32x4v y;
#pragma unroll
        for (int e = 0; e < 4; ++e)  // xor 2: quad_perm [2, 3, 0, 1]
          y[e] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x[e]), 0x4E, 0xF, 0xF, false));
        if (b & 2) {
          x[0] = y[2];
          x[1] = y[3];
        } else {
          x[2] = y[0];
          x[3] = y[1];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)  // xor 1: quad_perm [1, 0, 3, 2]
          y[e] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x[e]), 0xB1, 0xF, 0xF, false));
        if (b & 1) {
          x[0] = y[1];
          x[2] = y[3];
        } else {
          x[1] = y[0];
          x[3] = y[2];
        }
        const int m = row_of<AK>(m0, t, 4 * q + b);
        const int n = n0 + 16 * u + 4 * (j >> 2);
        if (m < a.M && n < a.N) store4(m, n, x);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row_of<AK>(m0, t, 4 * q + r);
        if (m >= a.M) continue;
#pragma unroll
        for (int u = 0; u < TN; ++u) {
          const int n = n0 + 16 * u + j;
          if (n < a.N) store1(m, n, acc[t][u][r]);
        }
      }
    }
  }
}

// VEC_OK / SCALAR_OK: which load paths this configuration is instantiated for (the scalar one only
// for the K-split-4 64x64 configuration: compile time)
// PLAIN: only the unmasked, row-sum-free instantiations (the 128x64 wave tile: its masked and
// row-sum forms spill; dispatch routes those products to the 64x64 tile)
template <int LA, int LB, int WTM, int WTN, int WGM, int WGN, int WGK, int H, bool PLAIN = false>
hipError_t launch(const GemmF32Args& a, bool vec, hipStream_t stream) {
  constexpr bool VEC_OK = true, SCALAR_OK = WTM == 64 && WTN == 64 && WGK == 4 && !PLAIN;
  constexpr int BM = WGM * WTM, BN = WGN * WTN;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const dim3 grid((unsigned)tiles), block(256);
#define DGT_F32_LAUNCH(V, MK, RS)                                                                          \
  {                                                                                                    \
    hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, WTM, WTN, WGM, WGN, WGK, H, V, MK, RS>), grid, block, 0, stream, a); \
  }
  if constexpr (SCALAR_OK) {  // the small-grid split-K (gemm_f32_split)
    if (vec && a.split > 1 && a.rowsum == nullptr) {
      const dim3 sgrid((unsigned)(tiles * a.split));
      if (a.maskA)
        hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, WTM, WTN, WGM, WGN, WGK, H, true, true, false, true>), sgrid, block,
                           0, stream, a);
      else
        hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, WTM, WTN, WGM, WGN, WGK, H, true, false, false, true>), sgrid, block,
                           0, stream, a);
      return hipGetLastError();
    }
  }
  // (the ReLU-masked A and the fused row sums come together in a wgrad: MASKED and ROWSUM share
  // one instantiation pair)
  const bool rs = a.rowsum != nullptr;
  if constexpr (PLAIN) {
    if (!vec || a.maskA || rs) return hipErrorInvalidValue;  // (dispatch never sends these here)
    DGT_F32_LAUNCH(true, false, false)
    return hipGetLastError();
  } else if constexpr (VEC_OK) {
    if (vec) {
      if (a.maskA && rs) DGT_F32_LAUNCH(true, true, true)
      else if (a.maskA) DGT_F32_LAUNCH(true, true, false)
      else if (rs) DGT_F32_LAUNCH(true, false, true)
      else DGT_F32_LAUNCH(true, false, false)
      return hipGetLastError();
    }
  }
  if constexpr (SCALAR_OK) {
    if (a.maskA && rs) DGT_F32_LAUNCH(false, true, true)
    else if (a.maskA) DGT_F32_LAUNCH(false, true, false)
    else if (rs) DGT_F32_LAUNCH(false, false, true)
    else DGT_F32_LAUNCH(false, false, false)
  }
#undef DGT_F32_LAUNCH
  return hipGetLastError();
}

template <int LA, int LB>
hipError_t dispatch(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream) {
  // ragged operands (scalar loads) are rare: one configuration serves them all (it takes any grid)
  if (!vec) return launch<LA, LB, 64, 64, 1, 1, 4, 1>(a, false, stream);
  switch (p.cfg) {
    case kF32Wave128:
      if (a.maskA || a.rowsum) return launch<LA, LB, 64, 64, 2, 2, 1, 2>(a, vec, stream);
      return launch<LA, LB, 128, 64, 2, 2, 1, 2, true>(a, vec, stream);
    case kF32Wave64: return launch<LA, LB, 64, 64, 2, 2, 1, 2>(a, vec, stream);
    case kF32Wave64Split2: return launch<LA, LB, 64, 64, 1, 2, 2, 2>(a, vec, stream);
    default: return launch<LA, LB, 64, 64, 1, 1, 4, 1>(a, vec, stream);
  }
}

}  // namespace f32g
}  // namespace dgt
