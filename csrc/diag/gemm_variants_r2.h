// Round-2 GEMM variants, kept for re-measurement only (NOT in the shipped extension): each was
// measured slower than, or no better than, the default kernels inside the MLP step, and the A/B
// records stay in profiles/:
//   v3 128x128 4-stage 4 waves; v5 256x128 split-K 2 (profiles/r2_gemm_m1024.jsonl);
//   v6 wgrad+Adam wave-specialised (profiles/r2_wgrad_adam_ws_ab.txt);
//   v7 BK=128 / v8 two K-tiles per barrier (profiles/r2_gemm_bk128_ab.txt);
//   v9 256x256 one barrier per K-tile (profiles/r2_gemm_wgrad_k1024.jsonl).
// Include AFTER ../gemm.hip (it reuses the staging, fragment and epilogue helpers) and call
// dgt::diag_gemm_nt(g, epi, stream, variant) instead of dgt::gemm_nt for variants 3 and 5-9.
#pragma once

namespace dgt {

// S = 2: two stages (64 KiB), two blocks per CU, plain vmcnt(0) + barrier per K-step.
// S > 2: S stages (S x 32 KiB), one block per CU, S-1 K-tiles in flight: the wait before K-tile kt
// is a counted vmcnt (every glds but the newest (S-2) tiles' 8 per thread) and the barrier is a raw
// s_barrier, so the prefetches stay in flight across it (a __syncthreads would drain them).  For
// grids that fit the chip in one wave of blocks this hides HBM latency the 2-stage loop exposes.

// NW = 4: waves 2 (M) x 2 (N), 64 x 64 each (4 x 4 accumulators).  NW = 8: waves 2 x 4, 64 x 32
// each: two waves per SIMD, so one wave's LDS fragment reads overlap the other's MFMAs (the
// 4-wave block leaves the matrix core idle while its only wave waits on LDS).
// BK = 128 (S = 2 only, 128 KiB of LDS, one block per CU): hipBLASLt's macro-tile depth -- half the
// barriers and vmcnt drains per FLOP of BK = 64, and 4 MFMA k-steps between them instead of 2.
// G = 2 (S = 5, 160 KiB): the same halved barrier count at BK = 64 granularity -- one barrier per
// two K-tiles, three K-tiles (96 KiB) in flight behind the pair being computed, as deep as the
// 4-stage loop, where BK = 128 x 2 stages keeps only one 64 KiB tile ahead (cold operands stall it).
template <int EPI, int S, int NW = 4, int BK = GBK, int G = 1>
__global__ __launch_bounds__(64 * NW, (S == 2 && BK == GBK) ? 2 : 1) void gemm_nt_kernel_r2(GemmArgs g) {
  static_assert(BK == GBK || (BK == 2 * GBK && S == 2), "BK = 128 only with the 2-stage loop");
  static_assert(G == 1 || (S > 2 && S >= 2 * G + 1 && BK == GBK), "G tiles per barrier need S >= 2G + 1 stages");
  constexpr bool KN = (EPI & kEpiBKN) != 0;      // B is [K, N]: staged as is, transposed reads
  constexpr int WN = NW == 8 ? 32 : 64;          // wave tile columns
  constexpr int WCOLS = GBN / WN;                // waves across N
  constexpr int NJ = WN / 16;                    // accumulator columns per wave
  __shared__ __attribute__((aligned(16))) u16 lds[S][2][GBM * BK];  // [stage][A|B], 32 KiB per stage at BK 64
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int tm, tn;
  tile_of_block(blockIdx.x, g.M / GBM, g.N / GBN, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int wr = w / WCOLS, wc = w % WCOLS;
  const u16* A = static_cast<const u16*>(g.A);
  const u16* B = static_cast<const u16*>(g.B);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  auto compute = [&](int buf) {
    const u16* As = lds[buf][0];
    const u16* Bs = lds[buf][1];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<BK>(As, wr * 64 + i * 16 + (l & 15), chunk);
      if constexpr (KN) {
        i16x4 blo[NJ], bhi[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) read_frag_kn(Bs, kk * 32, wc * WN + j * 16, l, blo[j], bhi[j]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = tr_wait(blo[j], bhi[j]);
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = read_frag<BK>(Bs, wc * WN + j * 16 + (l & 15), chunk);
      }
#if defined(DGT_GEMM_ABLATE) && DGT_GEMM_ABLATE == 2  // diag: 2 = LDS reads, no MFMA
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j][0] += (float)af[i][0] + (float)bfr[j][0];
#else
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
#endif
    }
  };
  if constexpr (S == 2) {
    stage_tile<NW, BK>(A, g.lda, m0, 0, lds[0][0], w, l);
    stage_b<KN, NW, BK>(B, g.ldb, n0, 0, lds[0][1], w, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        stage_tile<NW, BK>(A, g.lda, m0, (kt + 1) * BK, lds[cur ^ 1][0], w, l);
        stage_b<KN, NW, BK>(B, g.ldb, n0, (kt + 1) * BK, lds[cur ^ 1][1], w, l);
      }
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    constexpr int PER_TILE = 2 * (16 / NW);  // glds per thread per K-tile (A and B)
    constexpr int AHEAD = S - 2 * G;         // K-tiles left in flight past the G being retired
    Stager<NW, false> sa(A, g.lda, m0, w, l);
    Stager<NW, KN> sb(B, g.ldb, n0, w, l);
#pragma unroll
    for (int p = 0; p < S - G; ++p) {
      if (p < nk) {
        sa.issue(lds[p][0]);
        sb.issue(lds[p][1]);
      }
    }
    int buf = 0, nb = S - G;  // buffer of tile kt, buffer the next staged tile lands in (tile % S)
    for (int kt = 0; kt < nk; kt += G) {
      // tiles kt .. min(kt + S - G - 1, nk - 1) are in flight; retire tiles kt .. kt + G - 1
      const int ahead = min(AHEAD, nk - kt - G);
      if (ahead >= AHEAD) wait_vmcnt<AHEAD * PER_TILE>();
      else if (AHEAD > 1 && ahead == 1) wait_vmcnt<PER_TILE>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // tiles kt.. visible to all waves; buffers of kt-G .. kt-1 free for reuse
      __builtin_amdgcn_sched_barrier(0);
#if !(defined(DGT_GEMM_ABLATE) && DGT_GEMM_ABLATE == 1)  // diag: 1 = no staging inside the loop
#pragma unroll
      for (int i = 0; i < G; ++i) {
        if (kt + S - G + i < nk) {
          sa.issue(lds[nb][0]);
          sb.issue(lds[nb][1]);
        }
        nb = (nb + 1 == S) ? 0 : nb + 1;
      }
#endif
#pragma unroll
      for (int i = 0; i < G; ++i) {
        compute(buf);
        buf = (buf + 1 == S) ? 0 : buf + 1;
      }
    }
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: D col = l&15 (n), row = 4*(l>>4) + r (m)
  if constexpr ((EPI & kEpiAdam) != 0) {
    // fp32 128 x 128 tile = 64 KiB: one pass fits the 2-stage (64 KiB) and 4-stage LDS
    epilogue_adam<GBM, GBN, 64, WN, 64 * NW, GBM>(g, acc, reinterpret_cast<float*>(&lds[0][0][0]), m0, n0, wr, wc, l,
                                                  tid);
  } else if constexpr (!(EPI & kEpiOutF32)) {
    epilogue_staged<EPI, GBM, GBN, 64, WN, 64 * NW>(g, acc, &lds[0][0][0], m0, n0, wr, wc, l, tid);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + wr * 64 + i * 16 + 4 * (l >> 4), n0 + wc * WN + j * 16 + (l & 15));
  }
}

// ------------------------------------------------------------------ 256 x 128 tile, split-K 2
// For the MLP's M = 1024 products (forward a . W^T and dgrad g . W at N = K = 4096): a 128 x 128
// tile per CU (the only way 256 tiles fill 256 CUs without splitting K) re-reads 64 B of operand per
// 2 x 64 x 64 x 2 FLOP, and those reads - global -> LDS staging and LDS fragment reads - bound the
// loop (profiles/r1_gemm128_ablation.txt).  Here a block owns a 256 x 128 tile over HALF of K:
// 25 % fewer staged bytes per FLOP and 64 x 64 wave tiles (4 (M) x 2 (N) waves of 4 x 4
// accumulators: 33 % fewer LDS fragment bytes per FLOP than the 64 x 32 wave tiles of the 8-wave
// 128 kernel), and M = 1024 still gives 4 x 32 tiles x 2 halves = 256 blocks.
// The halves meet through a per-tile arrival counter: the first to finish writes its fp32 partial
// tile (128 KiB) to the slab and publishes it (agent-scope release, flag); the second waits for
// the flag (acquire), adds the slab to its accumulators (fp32 a + b == b + a: the result does not
// depend on which half came first) and runs the fused epilogue.  Only the FIRST block ever waits
// on nothing and the waiting block's partner has already arrived, so no co-residency is assumed.
// Blocks 8 apart share an XCD: both halves of a tile get ids 8 apart (same XCD, slab in that
// XCD's L2), and each XCD takes a contiguous range of tiles, M-tiles fastest (T1).
namespace sk {
constexpr int BM = 256, BN = 128, BK = 64, S = 3, NW = 8;
constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK, STAGE = A_ELEMS + B_ELEMS;  // u16 per stage (48 KiB)
constexpr int PW_A = (BM / 8) / NW;  // A: 1 KiB wave-instructions (8 rows x 128 B) per wave = 4
constexpr int PW_B = 16 / NW;        // B: [N,K] 8 rows x 128 B, or [K,N] 4 k-rows x 256 B = 2
constexpr int PER_TILE = PW_A + PW_B;

template <bool KN>
struct Stage {
  const u16* pa[PW_A];
  const u16* pb[PW_B];
  int la[PW_A], lb[PW_B];
  long long stepb;
  DGT_DEVICE Stage(const u16* A, int lda, int m0, const u16* B, int ldb, int n0, int k0, int w, int l) {
#pragma unroll
    for (int i = 0; i < PW_A; ++i) {
      const int rblk = (w * PW_A + i) * 8, row = rblk + (l >> 3);
      const int c = (l & 7) ^ (row & 7);
      pa[i] = A + (long long)(m0 + row) * lda + k0 + c * 8;
      la[i] = rblk * BK;
    }
#pragma unroll
    for (int i = 0; i < PW_B; ++i) {
      if constexpr (KN) {
        const int rblk = (w * PW_B + i) * 4, row = rblk + (l >> 4);
        const int c = (l & 15) ^ kn_swz(row);
        pb[i] = B + (long long)(k0 + row) * ldb + n0 + c * 8;
        lb[i] = rblk * BN;
      } else {
        const int rblk = (w * PW_B + i) * 8, row = rblk + (l >> 3);
        const int c = (l & 7) ^ (row & 7);
        pb[i] = B + (long long)(n0 + row) * ldb + k0 + c * 8;
        lb[i] = rblk * BK;
      }
    }
    stepb = KN ? (long long)BK * ldb : BK;
  }
  DGT_DEVICE void issue(u16* st) {
#pragma unroll
    for (int i = 0; i < PW_A; ++i) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pa[i]), reinterpret_cast<int*>(st + la[i]), 16, 0,
                                       0);
      pa[i] += BK;
    }
#pragma unroll
    for (int i = 0; i < PW_B; ++i) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pb[i]),
                                       reinterpret_cast<int*>(st + A_ELEMS + lb[i]), 16, 0, 0);
      pb[i] += stepb;
    }
  }
};
}  // namespace sk

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_nt_sk_kernel(GemmArgs g) {
  using namespace sk;
  constexpr bool KN = (EPI & kEpiBKN) != 0;
  __shared__ __attribute__((aligned(16))) u16 lds[S * STAGE];  // ONE array: 144 KiB
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;  // 4 (M) x 2 (N) waves of 64 x 64
  const int MT = g.M / BM, T = MT * (g.N / BN);
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, half = slot & 1;
  const int t = xcd * (T / 8) + (slot >> 1);
  const int m0 = (t % MT) * BM, n0 = (t / MT) * BN;
  const int kh = g.K / 2, nk = kh / BK;
  const u16* A = static_cast<const u16*>(g.A);
  const u16* B = static_cast<const u16*>(g.B);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<KN> st(A, g.lda, m0, B, g.ldb, n0, half * kh, w, l);
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) st.issue(lds + p * STAGE);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tiles kt .. min(kt + S - 2, nk - 1) are in flight; retire tile kt
    if (kt + S - 2 < nk) wait_vmcnt<(S - 2) * PER_TILE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // tile kt visible to every wave; the buffer of kt - 1 is free
    __builtin_amdgcn_sched_barrier(0);
    if (kt + S - 1 < nk) st.issue(lds + ((buf + S - 1) % S) * STAGE);
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag(As, wr * 64 + i * 16 + (l & 15), chunk);
      if constexpr (KN) {
        i16x4 blo[4], bhi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) read_frag_kn(Bs, kk * 32, wc * 64 + j * 16, l, blo[j], bhi[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = tr_wait(blo[j], bhi[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = read_frag(Bs, wc * 64 + j * 16 + (l & 15), chunk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    buf = (buf + 1 == S) ? 0 : buf + 1;
  }
  __builtin_amdgcn_s_barrier();  // every wave is done with the operand stages

  // ---- split-K meeting point (cdna_hip_programming.md, projection GEMM item 2 / Guideline 16)
  int* arrive = g.sk_flags + 2 * t;
  int* ready = arrive + 1;
  float* slab = g.sk_slab + (long long)t * BM * BN;
  int* order = reinterpret_cast<int*>(lds);  // in the one LDS array (operands are dead)
  if (tid == 0) *order = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool first = *order == 0;
  if (first) {
    // publish (Guideline 16 R1): write-through (sc1) stores of the partial tile, drained by EVERY
    // storing wave, barrier, ONE relaxed agent-scope flag store: no release fence (no L2 writeback)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          __hip_atomic_store(slab + (wr * 64 + i * 16 + 4 * (l >> 4) + rr) * BN + wc * 64 + j * 16 + (l & 15),
                             acc[i][j][rr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (tid == 0) {
    // the partner has arrived (the counter said so): it is writing the slab.  Bounded all the same
    // (~0.5 s), so a corrupted flag can only produce a wrong tile, never a hung GPU
    for (int spin = 0; spin < (1 << 24) && __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
         ++spin)
      __builtin_amdgcn_s_sleep(1);
    // both halves are past their last use of the flags: re-arm them for the next launch
    __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ready, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // every load of the slab is an sc1 (agent-scope) load: it bypasses this CU's L1, so no acquire
  // fence is needed (Guideline 16: all payload stores sc1 + drained, flag atomic, all loads sc1)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        acc[i][j][rr] += __hip_atomic_load(slab + (wr * 64 + i * 16 + 4 * (l >> 4) + rr) * BN + wc * 64 + j * 16 + (l & 15),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  epilogue_staged<EPI, BM, BN, 64, 64, 512>(g, acc, lds, m0, n0, wr, wc, l, tid);
}

// ------------------------------------------------------------------ 256 x 256 tile, one barrier per K-tile
// The 8-phase kernel above meets at two barriers per 16 MFMAs per wave (16 per BK = 64 K-tile); at
// K = 1024 (the MLP's weight gradient) those meetings, not the matrix cores, set the pace.  Here the
// same 8 waves (2 (M) x 4 (N), 128 x 64 each, 8 x 4 accumulators) run the plain two-stage loop of the
// 128 x 128 kernel: the whole next K-tile (256 + 256 rows x 64, 64 KiB) is staged by LDS-DMA while
// the current one is consumed by 64 MFMAs per wave, then ONE vmcnt(0) + barrier.  The two waves on a
// SIMD overlap each other's fragment reads with MFMAs.  Same MFMAs in the same k order as the other
// kernels (bit-identical results).  B as [N, K] only.
template <int EPI>
__global__ __launch_bounds__(512) void gemm_nt_256s_kernel(GemmArgs g) {
  static_assert(!(EPI & kEpiBKN), "the 256 x 256 single-barrier kernel reads B as [N, K]");
  constexpr int BM = 256, BN = 256, BK = GBK, NW = 8;
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][BM * BK];  // [stage][A|B], 64 KiB per stage
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int tm, tn;
  tile_of_block(blockIdx.x, g.M / BM, g.N / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN, wr = w >> 2, wc = w & 3;
  const u16* A = static_cast<const u16*>(g.A);
  const u16* B = static_cast<const u16*>(g.B);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int kt, int buf) {  // 128-row halves: stage_tile's swizzle depends on row & 7 only
    stage_tile<NW>(A, g.lda, m0, kt * BK, lds[buf][0], w, l);
    stage_tile<NW>(A, g.lda, m0 + 128, kt * BK, lds[buf][0] + 128 * BK, w, l);
    stage_tile<NW>(B, g.ldb, n0, kt * BK, lds[buf][1], w, l);
    stage_tile<NW>(B, g.ldb, n0 + 128, kt * BK, lds[buf][1] + 128 * BK, w, l);
  };
  const int nk = g.K / BK;
  stage(0, 0);
  wait_vmcnt<0>();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const u16* As = lds[cur][0];
    const u16* Bs = lds[cur][1];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = read_frag(As, wr * 128 + i * 16 + (l & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag(Bs, wc * 64 + j * 16 + (l & 15), chunk);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    wait_vmcnt<0>();
    __syncthreads();
  }
  if constexpr ((EPI & kEpiAdam) != 0) {
    // fp32 256 x 256 tile = 256 KiB: two passes of 128 rows through the 128 KiB of operand LDS
    epilogue_adam<BM, BN, 128, 64, 512, 128>(g, acc, reinterpret_cast<float*>(&lds[0][0][0]), m0, n0, wr, wc, l, tid);
  } else if constexpr (!(EPI & kEpiOutF32)) {
    epilogue_staged<EPI, BM, BN, 128, 64, 512>(g, acc, &lds[0][0][0], m0, n0, wr, wc, l, tid);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + wr * 128 + i * 16 + 4 * (l >> 4), n0 + wc * 64 + j * 16 + (l & 15));
  }
}

// ------------------------------------------------------------------ wgrad + Adam, wave-specialised
// The MLP's weight-gradient GEMM dW = g^T . a (M = N = 4096, K = batch = 1024) with Adam applied to
// each 128 x 128 gradient tile in place (kEpiAdam).  In the one-tile-per-block kernels every CU runs
// its K loop (MFMA-bound) and THEN its tile's update (HBM-bound: 26 B/param), so the chip alternates
// between the two limits (profiles/r2_mlp_fused_adam_ab.txt).  Here a persistent block walks
// T / gridDim tiles with two wave groups sharing one LDS:
//   * 8 MFMA waves (2 x 4 of 64 x 32) stream the operands through a 3-slot LDS-DMA ring across tile
//     boundaries and, at the end of each tile, hand the fp32 tile to a 64 KiB LDS buffer;
//   * 4 Adam waves update the PREVIOUS tile from that buffer, one 1/16 chunk (one float4 per lane)
//     per K step, with master / m / v loads R-1 chunks ahead in registers,
// so the update of tile i streams from HBM while the matrix cores compute tile i+1.  All 12 waves
// meet at every K step's ring barrier (raw s_barrier: the wave groups run different code, one
// barrier sequence); at a tile boundary two more barriers fence the hand-off buffer.  The last
// tile's update runs after the loop.  Per element the update is epilogue_adam's: the same fp32
// gradient (alpha * acc) and the same adam_update, so results are bit-identical to variant 0.
// Measured (csrc/diag/wsa_ablate.hip, profiles/r2_wgrad_adam_ws_ab.txt): the GEMM alone runs 33 us
// in this structure and the update alone 72 us, but together 103-110 us -- the sum, no overlap: the
// 128 x 128 tiles re-read ~0.5 GB of operands through L2 per layer, and that traffic and the
// update's HBM stream contend in the memory system rather than in the CU.  Opt-in only (variant 6).
namespace wsa {
constexpr int BM = 128, BN = 128, BK = 64, S = 3, NMW = 8, NAW = 4, NT = 64 * (NMW + NAW);
constexpr int NK = 16;         // K steps per tile: K = 1024 (one float4 per Adam lane per step)
constexpr int R = 8;           // Adam register ring: chunks R-1 ahead
constexpr int WN = 32, NJ = WN / 16, WCOLS = BN / WN;
constexpr int PER_TILE = 2 * (16 / NMW);  // LDS-DMA instructions per MFMA thread per K step
static_assert(NK % R == 0 && BM * BN / 4 == NK * 64 * NAW, "one float4 per Adam lane per K step");

struct AdamIn {
  f32x4 p, m, v;
};

DGT_DEVICE void tile_origin(int vid, int tiles_m, int tiles_n, int& m0, int& n0) {
  int tm, tn;
  tile_of_block(vid, tiles_m, tiles_n, tm, tn);
  m0 = tm * BM;
  n0 = tn * BN;
}
}  // namespace wsa

__global__ __launch_bounds__(wsa::NT, 1) void gemm_wgrad_adam_ws_kernel(GemmArgs g) {
  using namespace wsa;
  __shared__ __attribute__((aligned(16))) u16 ring[S][2][BM * BK];  // 96 KiB operand ring
  __shared__ __attribute__((aligned(16))) float hand[BM * BN];      // 64 KiB gradient hand-off
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = g.M / BM, tiles_n = g.N / BN, T = tiles_m * tiles_n, G = gridDim.x;
  const int ntb = (T - (int)blockIdx.x + G - 1) / G;  // this block's tiles: blockIdx.x + i * G
  const int Q = ntb * NK;                             // K steps of this block
  if (w < NMW) {
    // ---------------- MFMA waves
    const int wr = w / WCOLS, wc = w % WCOLS;
    const u16* A = static_cast<const u16*>(g.A);
    const u16* B = static_cast<const u16*>(g.B);
    auto issue = [&](int q) {
      const int i = q / NK, kt = q - i * NK;
      int m0, n0;
      tile_origin((int)blockIdx.x + i * G, tiles_m, tiles_n, m0, n0);
      stage_tile<NMW>(A, g.lda, m0, kt * BK, ring[q % S][0], w, l);
      stage_tile<NMW>(B, g.ldb, n0, kt * BK, ring[q % S][1], w, l);
    };
    f32x4 acc[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (p < Q) issue(p);
    for (int q = 0; q < Q; ++q) {
      if (q + 1 < Q) wait_vmcnt<(S - 2) * PER_TILE>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // B1: step q's operands visible; slot of step q-1 free
      __builtin_amdgcn_sched_barrier(0);
#if !(defined(DGT_WSA_ABLATE) && DGT_WSA_ABLATE == 2)  // diag: 2 = MFMA waves idle (barriers only)
      if (q + S - 1 < Q) issue(q + S - 1);
      const u16* As = ring[q % S][0];
      const u16* Bs = ring[q % S][1];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (l >> 4);
        bf16x8 af[4], bfr[NJ];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = read_frag(As, wr * 64 + i * 16 + (l & 15), chunk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = read_frag(Bs, wc * WN + j * 16 + (l & 15), chunk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
#endif
      if (q % NK == NK - 1) {
        __builtin_amdgcn_s_barrier();  // B2: the Adam waves are done with the previous tile's hand-off
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
              hand[adam_slot<BN>(wr * 64 + i * 16 + 4 * (l >> 4) + rr, wc * WN + j * 16 + (l & 15))] =
                  acc[i][j][rr] * g.alpha;
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the hand-off stores are in LDS
        __builtin_amdgcn_s_barrier();        // B3: hand-off complete
      }
    }
    return;
  }
  // ---------------- Adam waves.  Chunk c of tile ti is the float4 at row 8c + at / 32, column
  // 4 (at % 32) of the tile, updated during K step (ti + 1) * NK + c (the MFMA waves' next tile);
  // the last tile's chunks after the loop.  Straight-line per tile (16 chunks unrolled, loads R-1
  // chunks ahead in a register ring, no per-lane branches) so the compiler's vmcnt waits are counted,
  // not drains.
  const GemmAdam& ad = g.adam;
  __hip_bfloat16* lp = static_cast<__hip_bfloat16*>(ad.lp);
  const int at = (w - NMW) * 64 + l;
  const int r0 = at / (BN / 4), c0 = (at % (BN / 4)) * 4;
  const long long lane_off = (long long)r0 * g.ldc + c0, step_off = 8LL * g.ldc;
  auto tile_base = [&](int ti) -> long long {
    int m0, n0;
    tile_origin((int)blockIdx.x + min(ti, ntb - 1) * G, tiles_m, tiles_n, m0, n0);
    return (long long)m0 * g.ldc + n0;
  };
  auto load = [&](long long o, AdamIn& in) {
#if defined(DGT_WSA_ABLATE) && DGT_WSA_ABLATE == 1  // diag: 1 = Adam waves idle (barriers only)
    return;
#endif
    in.p = *reinterpret_cast<const f32x4*>(ad.master + o);
    in.m = *reinterpret_cast<const f32x4*>(ad.m + o);
    in.v = *reinterpret_cast<const f32x4*>(ad.v + o);
  };
  auto update = [&](long long o, int c, AdamIn& in) {
#if defined(DGT_WSA_ABLATE) && DGT_WSA_ABLATE == 1
    return;
#endif
    const f32x4 gr = *reinterpret_cast<const f32x4*>(hand + adam_slot<BN>(r0 + 8 * c, c0));
    __hip_bfloat16 b[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mm = in.m[e], vv = in.v[e];
      in.p[e] = adam_update(in.p[e], gr[e], mm, vv, ad.hp, ad.step_size_neg, ad.bc2_sqrt);
      in.m[e] = mm;
      in.v[e] = vv;
      b[e] = __float2bfloat16(in.p[e]);
    }
    *reinterpret_cast<f32x4*>(ad.master + o) = in.p;
    *reinterpret_cast<f32x4*>(ad.m + o) = in.m;
    *reinterpret_cast<f32x4*>(ad.v + o) = in.v;
    *reinterpret_cast<uint2*>(lp + o) = *reinterpret_cast<const uint2*>(b);
  };
  AdamIn buf[R];
  {
    const long long b0 = tile_base(0) + lane_off;
#pragma unroll
    for (int u = 0; u < R - 1; ++u) load(b0 + u * step_off, buf[u]);
  }
  // the MFMA waves' first tile: barriers only
  for (int q = 0; q < NK; ++q) __builtin_amdgcn_s_barrier();  // B1
  __builtin_amdgcn_s_barrier();                                // B2
  __builtin_amdgcn_s_barrier();                                // B3
  for (int ti = 0; ti < ntb; ++ti) {
    const bool overlapped = ti < ntb - 1;  // the MFMA waves are computing tile ti + 1
    const long long cur = tile_base(ti) + lane_off, nxt = tile_base(ti + 1) + lane_off;
#pragma unroll
    for (int c = 0; c < NK; ++c) {
      if (overlapped) __builtin_amdgcn_s_barrier();  // B1 of K step (ti + 1) * NK + c
      const int cp = c + R - 1;                      // chunk prefetched now (this tile or the next)
      load(cp < NK ? cur + cp * step_off : nxt + (cp - NK) * step_off, buf[cp % R]);
      update(cur + c * step_off, c, buf[c % R]);
      if (overlapped && c == NK - 1) {
        __builtin_amdgcn_s_barrier();  // B2: done with this tile's hand-off
        __builtin_amdgcn_s_barrier();  // B3: the next tile's gradient is in the hand-off buffer
      }
    }
  }
}

// variant: 0 = pick by shape, 1 = 128x128 2-stage, 2 = 256x256 8-phase, 3 = 128x128 4-stage,
// 4 = 128x128 4-stage with 8 waves, 5 = 256x128 split-K 2 (needs the sk workspace),
// 6 = wgrad + Adam with wave-specialised update overlap (kEpiAdam, K = 1024 only),
// 7 = 128x128 2-stage with 8 waves at BK = 128 (K % 128 == 0),
// 8 = 128x128 5-stage with 8 waves, one barrier per two K-tiles (K % 128 == 0),
// 9 = 256x256 2-stage with 8 waves of 128x64, one barrier per K-tile (B as [N, K])
static int diag_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
static bool diag_sk_fits(const GemmArgs& g) {
  const int T = (g.M % 256 == 0 && g.N % 128 == 0) ? (g.M / 256) * (g.N / 128) : 0;
  return T > 0 && T % 8 == 0 && g.K % 128 == 0 && g.sk_slab && g.sk_flags;
}

hipError_t diag_gemm_nt(const GemmArgs& g, int epi, hipStream_t stream, int variant) {
  if (g.M % GBM || g.N % GBN || g.K % GBK || g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  // split-K 256 x 128 (variant 5) on request only: on the M = 1024 MLP products it ties the 8-wave
  // 128 x 128 kernel (fwd 46.2 vs 48.1 us hot, 53.9 vs 53.4 cold; dgrad 50.7 vs 49.5 hot,
  // profiles/r2_gemm_m1024.jsonl), so the shape-picked default stays the 128 x 128 kernel
  if (variant == 6) {
    if (epi != kEpiAdam || g.K != wsa::NK * wsa::BK || g.M % wsa::BM || g.N % wsa::BN) return hipErrorInvalidValue;
    const int T = (g.M / wsa::BM) * (g.N / wsa::BN);
    hipLaunchKernelGGL(gemm_wgrad_adam_ws_kernel, dim3(std::min(T, diag_cu_count())), dim3(wsa::NT), 0, stream, g);
    return hipGetLastError();
  }
  const bool sk_epi = !(epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam));
  if (variant == 5 && (!diag_sk_fits(g) || !sk_epi)) return hipErrorInvalidValue;
  const bool use_sk = variant == 5;
  if (use_sk) {
    const int grid = (g.M / 256) * (g.N / 128) * 2;
    switch (epi) {
#define DGT_SK_CASE(E) \
  case E: hipLaunchKernelGGL((gemm_nt_sk_kernel<E>), dim3(grid), dim3(512), 0, stream, g); return hipGetLastError();
      DGT_SK_CASE(0)
      DGT_SK_CASE(kEpiBias | kEpiRelu | kEpiStoreT)
      DGT_SK_CASE(kEpiBias | kEpiRelu)
      DGT_SK_CASE(kEpiMask | kEpiStoreT)
      DGT_SK_CASE(kEpiMask | kEpiStoreT | kEpiBKN)
      DGT_SK_CASE(kEpiBKN)
#undef DGT_SK_CASE
      default:
        if (variant == 5) return hipErrorInvalidValue;  // no split-K instance: fall through to the others
    }
  }
  const bool fits256 = g.M % 256 == 0 && g.N % 256 == 0 && g.K % 128 == 0;
  // the big tile needs most of the 256 CUs busy: below ~200 tiles the 128 kernel (4x the blocks,
  // 2 blocks per CU) wins
  bool big = fits256 && (g.M / 256) * (g.N / 256) >= 200;
  if (variant == 1 || variant == 3 || variant == 4 || variant == 7 || variant == 8) big = false;
  if ((variant == 7 || variant == 8) && g.K % (2 * GBK)) return hipErrorInvalidValue;
  const bool bk128 = variant == 7, pair = variant == 8;
  if (variant == 2 || variant == 9) {
    if (!fits256) return hipErrorInvalidValue;
    big = true;
  }
  if (epi & kEpiBKN) {  // only the 128x128 kernel reads a [K, N] B operand
    if (variant == 2 || variant == 9) return hipErrorInvalidValue;
    big = false;
  }
  const bool single = big && variant == 9;
  const int grid = big ? (g.M / 256) * (g.N / 256) : (g.M / GBM) * (g.N / GBN);
  // a grid that fits the chip at one block per CU gains nothing from 2 blocks/CU: spend the LDS on
  // a deep (4-stage) pipeline instead
  const bool deep = !big && (variant == 3 || variant == 4 || (variant == 0 && grid <= 256));
  const bool eight = deep && variant != 3;  // measured: 8 waves beat 4 on one-wave grids (817 vs 759 TF)
#define DGT_EPI_CASE_KN(E)                                                                        \
  case E:                                                                                         \
    if (bk128) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 2, 8, 2 * GBK>), dim3(grid), dim3(512), 0, stream, g); \
    else if (pair) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 5, 8, GBK, 2>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else if (deep) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 4>), dim3(grid), dim3(256), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
#define DGT_EPI_CASE(E)                                                                           \
  case E:                                                                                         \
    if (single) hipLaunchKernelGGL((gemm_nt_256s_kernel<E>), dim3(grid), dim3(512), 0, stream, g); \
    else if (big) hipLaunchKernelGGL((gemm_nt_256_kernel<E>), dim3(grid), dim3(512), 0, stream, g); \
    else if (bk128) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 2, 8, 2 * GBK>), dim3(grid), dim3(512), 0, stream, g); \
    else if (pair) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 5, 8, GBK, 2>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else if (deep) hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 4>), dim3(grid), dim3(256), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel_r2<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
  switch (epi) {
    DGT_EPI_CASE(0)
    DGT_EPI_CASE(kEpiBias | kEpiRelu | kEpiStoreT)                 // hidden-layer forward
    DGT_EPI_CASE(kEpiBias | kEpiRelu)                              // forward, no transposed copy
    DGT_EPI_CASE(kEpiMask | kEpiStoreT)                            // dgrad through ReLU
    DGT_EPI_CASE(kEpiOutF32)                                       // wgrad into fp32 grads
    DGT_EPI_CASE(kEpiOutF32 | kEpiAccumulate)                      // wgrad, gradient accumulation
    DGT_EPI_CASE(kEpiOutF32 | kEpiBias)                            // generic fp32 out
    DGT_EPI_CASE(kEpiAdam)                                         // wgrad consumed by Adam in place
    DGT_EPI_CASE_KN(kEpiMask | kEpiStoreT | kEpiBKN)               // dgrad straight from W[out, in]
    DGT_EPI_CASE_KN(kEpiBKN)                                       // plain A . B
    DGT_EPI_CASE_KN(kEpiOutF32 | kEpiBKN)
    default:
      return hipErrorInvalidValue;
  }
#undef DGT_EPI_CASE
#undef DGT_EPI_CASE_KN
  return hipGetLastError();
}


}  // namespace dgt
