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
// Reference: Linear(20,64) / Linear(64,1) of train.py:29-33, forward train.py:107, backward train.py:113.
#include <hip/hip_bf16.h>

#include <algorithm>
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

// one 128 x BK bf16 operand tile: rows of BK/8 16-byte chunks, the chunk XOR-swizzled by the low
// bits of the row (BK = 64: 128-B rows, row & 7; BK = 128: 256-B rows, row & 15), so the 16 lanes
// of a ds_read_b128 group reading one chunk index of 16 consecutive rows hit distinct bank groups.
// 128 * BK * 2 / 1 KiB LDS-DMA wave-instructions per tile, 64 / (BK/8) rows each.
template <int NWAVE = 4, int BK = GBK>
DGT_DEVICE void stage_tile(const u16* __restrict__ src, int ld, int row0, int k0, u16* lds, int w, int l) {
  constexpr int CH = BK / 8, RPI = 64 / CH;    // chunks per row, rows per wave-instruction
  constexpr int PER_WAVE = GBM / RPI / NWAVE;  // 1 KiB wave-instructions per wave
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int rblk = (w * PER_WAVE + i) * RPI; // first of the rows this wave-instruction writes
    const int row = rblk + l / CH;
    const int p = l % CH;                      // LDS 16-B chunk this lane lands in
    const int c = p ^ (row & (CH - 1));        // logical chunk fetched (source-side swizzle)
    const u16* g = src + (long long)(row0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(g), reinterpret_cast<int*>(lds + rblk * BK), 16, 0,
                                     0);
  }
}

template <int BK = GBK>
DGT_DEVICE bf16x8 read_frag(const u16* lds, int row, int chunk) {
  const int p = chunk ^ (row & (BK / 8 - 1));
  return *reinterpret_cast<const bf16x8*>(lds + row * BK + p * 8);
}

// ---- B given as [K, N] (N contiguous, e.g. the weight W[out, in] as the dgrad's B operand): the
// K-tile is staged as it lies in memory, [64 k][128 n] with 256-byte rows, and the MFMA B fragment
// (8 consecutive k of one n per lane) is read with two gfx950 ds_read_b64_tr_b16 transposed reads
// (cdna_hip_programming.md T10), so no transposed copy of W is ever materialised.  The 16 16-byte
// chunks of row r are XOR-swizzled by ((r & 3) << 2) | ((r >> 2) & 3) (the guide's 256-byte-row
// image): conflict-free for the two 4-row blocks 8 rows apart that a 32-lane half reads.
DGT_DEVICE int kn_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

template <int NWAVE = 4, int BK = GBK>
DGT_DEVICE void stage_tile_kn(const u16* __restrict__ src, int ld, int k0, int n0, u16* lds, int w, int l) {
  constexpr int PER_WAVE = BK / 4 / NWAVE;     // 1 KiB wave-instructions per wave (4 k-rows each)
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int rblk = (w * PER_WAVE + i) * 4;   // first of the 4 k-rows this wave-instruction writes
    const int row = rblk + (l >> 4);
    const int c = (l & 15) ^ kn_swz(row);      // logical chunk fetched into physical chunk l & 15
    const u16* g = src + (long long)(k0 + row) * ld + n0 + c * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(g), reinterpret_cast<int*>(lds + rblk * GBN), 16, 0,
                                     0);
  }
}

// B operand staging of the 128x128 kernel: [N, K] rows (stage_tile) or [K, N] rows (stage_tile_kn)
template <bool KN, int NWAVE, int BK = GBK>
DGT_DEVICE void stage_b(const u16* __restrict__ src, int ld, int n0, int k0, u16* lds, int w, int l) {
  if constexpr (KN) stage_tile_kn<NWAVE, BK>(src, ld, k0, n0, lds, w, l);
  else stage_tile<NWAVE, BK>(src, ld, n0, k0, lds, w, l);
}

// Per-thread staging state of one operand of the 128x128 kernel: the global source of each of the
// thread's LDS-DMA pieces is computed ONCE and advanced by one K-tile per issue (K-tiles are staged
// strictly in order), instead of recomputing 64-bit row addresses and swizzles for every piece of
// every K-tile inside the main loop.
template <int NWAVE, bool KN>
struct Stager {
  static constexpr int PER_WAVE = 16 / NWAVE;
  const u16* p[PER_WAVE];
  int lds_off[PER_WAVE];  // element offset of the piece in the LDS operand tile (wave-uniform)
  long long step;         // elements per K-tile
  // NT operand [rows, K]: rc0 = first row of the block; KN operand [K, N]: rc0 = first column
  DGT_DEVICE Stager(const u16* __restrict__ src, int ld, int rc0, int w, int l) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      if constexpr (KN) {
        const int rblk = (w * PER_WAVE + i) * 4, row = rblk + (l >> 4);
        const int c = (l & 15) ^ kn_swz(row);
        p[i] = src + (long long)row * ld + rc0 + c * 8;
        lds_off[i] = rblk * GBN;
      } else {
        const int rblk = (w * PER_WAVE + i) * 8, row = rblk + (l >> 3);
        const int c = (l & 7) ^ (row & 7);
        p[i] = src + (long long)(rc0 + row) * ld + c * 8;
        lds_off[i] = rblk * GBK;
      }
    }
    step = KN ? (long long)GBK * ld : GBK;
  }
  DGT_DEVICE void issue(u16* lds) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(p[i]), reinterpret_cast<int*>(lds + lds_off[i]),
                                       16, 0, 0);
      p[i] += step;
    }
  }
};

typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

// lane (n = l & 15, kg = l >> 4) receives B[kb + 8kg + e][nb + n], e = 0..7: lane 4q + p of its
// 16-lane group supplies the address of row kb + 8kg + q (+4), columns nb + 4p .. nb + 4p + 3.
// Inline asm: the builtin's memory operand makes the compiler drain every in-flight LDS-DMA
// (vmcnt(0)) before each read, which serialises the staging pipeline; the caller waits lgkmcnt
// itself (tr_wait) before the fragments are used.
DGT_DEVICE void read_frag_kn(const u16* lds, int kb, int nb, int l, i16x4& lo, i16x4& hi) {
  const int q = (l >> 2) & 3, col = nb + 4 * (l & 3);
  const int r0 = kb + 8 * (l >> 4) + q, r1 = r0 + 4;
  const u16* a0 = lds + r0 * GBN + (((col >> 3) ^ kn_swz(r0)) << 3) + (col & 4);
  const u16* a1 = lds + r1 * GBN + (((col >> 3) ^ kn_swz(r1)) << 3) + (col & 4);
  const unsigned o0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) const u16*)(a0));
  const unsigned o1 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) const u16*)(a1));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(o0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(o1));
}

// wait for the asm transposed reads; the operands tie the wait to the registers it guards
DGT_DEVICE bf16x8 tr_wait(i16x4& lo, i16x4& hi) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo), "+v"(hi));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// One MFMA accumulator (rows mb..mb+3 of column n) through the fused epilogue.
template <int EPI>
DGT_DEVICE void epi_store(const GemmArgs& g, const f32x4& acc, int mb, int n) {
  const float bn = (EPI & kEpiBias) ? g.bias[n] : 0.f;
  const u16* mask = static_cast<const u16*>(g.mask);
  float v[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    float x = acc[rr] * g.alpha + bn;
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

// XCD-aware bijective block remap (T1): blocks b and b+8 share an XCD; give each XCD a contiguous
// range of tile ids, then group GROUP block-rows so consecutive ids reuse the same B panel in L2.
DGT_DEVICE void tile_of_block(int bid, int nbm, int nbn, int& tm, int& tn) {
  const int nwg = nbm * nbn, xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  const int GROUP = 8;
  const int group = wgid / (GROUP * nbn), first_m = group * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  tm = first_m + (wgid % (GROUP * nbn)) % gsize;
  tn = (wgid % (GROUP * nbn)) / gsize;
}

// bf16-output epilogue staged through the (then idle) operand LDS, for a TM x TN block tile of NT
// threads whose waves own WM x WN sub-tiles: the MFMA layout gives each lane 4 rows of ONE column,
// so direct stores are 2-byte scatters; staged, every global access (C rows, C^T rows, mask rows)
// is a 16-byte vector and 16 lanes cover one 256-byte row piece.  The low 4 bits of a row's
// 16-byte chunk index are XOR-swizzled by row / 8, so both the row reads (C) and the column reads
// (C^T: 16 lanes at rows 8k + e of one column) hit 16 distinct bank groups.  Values are rounded to
// bf16 once (after bias / ReLU) and masked after rounding (identical results: the mask only zeroes).
template <int TN>
DGT_DEVICE int etile(int r, int n) {
  const int c = n >> 3;
  return r * TN + ((((c ^ (r >> 3)) & 15) | (c & ~15)) << 3) + (n & 7);
}

// kEpiAdam epilogue: the block's fp32 gradient tile goes through LDS (the operand stages are idle)
// so that every global access of the optimizer update is a 16-byte vector: per float4 of the weight,
// 16-B loads of master / exp_avg / exp_avg_sq, torch's Adam in fp32 (the same per-element op order
// as adam_flat), 16-B stores of the three and an 8-B store of the bf16 compute copy.  The gradient
// never reaches memory: this replaces the wgrad's gradient store (2-4 B/param), the optimizer's
// gradient read (2-4 B/param) and the separate Adam launch, and overlaps the update's HBM traffic
// with the MFMA work of the blocks still in their K loop.
// LDS image: [RP rows][TN] fp32 per pass, the 16-float column group XOR-swizzled by (row >> 2) & 3:
// the MFMA layout writes 4 rows 4 apart x 16 consecutive columns per instruction (conflict-free),
// the update reads 16-B row pieces.  Waves whose WM-row band lies in pass h write in that pass.
template <int TN>
DGT_DEVICE int adam_slot(int r, int c) { return r * TN + (c ^ (((r >> 2) & 3) << 4)); }

template <int TM, int TN, int WM, int WN, int NT, int RP>
DGT_DEVICE void epilogue_adam(const GemmArgs& g, const f32x4 (&acc)[WM / 16][WN / 16], float* tile, int m0, int n0,
                              int wr, int wc, int l, int tid) {
  static_assert(TM % RP == 0 && RP % WM == 0 && TN >= 64 && (RP * TN / 4) % NT == 0, "adam epilogue geometry");
  const GemmAdam& a = g.adam;
  __hip_bfloat16* lp = static_cast<__hip_bfloat16*>(a.lp);
#pragma unroll 1
  for (int h = 0; h < TM / RP; ++h) {
    __syncthreads();  // operand stages (h = 0) or the previous pass's tile (h = 1) fully read
    if (wr * WM / RP == h) {
#pragma unroll
      for (int i = 0; i < WM / 16; ++i)
#pragma unroll
        for (int j = 0; j < WN / 16; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            tile[adam_slot<TN>(wr * WM - h * RP + i * 16 + 4 * (l >> 4) + rr, wc * WN + j * 16 + (l & 15))] =
                acc[i][j][rr] * g.alpha;
    }
    __syncthreads();
#pragma unroll 4
    for (int it = 0; it < RP * TN / 4 / NT; ++it) {
      const int idx = tid + NT * it, r = idx / (TN / 4), c = (idx % (TN / 4)) * 4;
      const f32x4 gr = *reinterpret_cast<const f32x4*>(tile + adam_slot<TN>(r, c));
      const long long o = (long long)(m0 + h * RP + r) * g.ldc + n0 + c;
      f32x4 p = *reinterpret_cast<const f32x4*>(a.master + o);
      f32x4 m = *reinterpret_cast<const f32x4*>(a.m + o);
      f32x4 v = *reinterpret_cast<const f32x4*>(a.v + o);
      __hip_bfloat16 b[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float mm = m[e], vv = v[e];
        p[e] = adam_update(p[e], gr[e], mm, vv, a.hp, a.step_size_neg, a.bc2_sqrt);
        m[e] = mm;
        v[e] = vv;
        b[e] = __float2bfloat16(p[e]);
      }
      *reinterpret_cast<f32x4*>(a.master + o) = p;
      *reinterpret_cast<f32x4*>(a.m + o) = m;
      *reinterpret_cast<f32x4*>(a.v + o) = v;
      *reinterpret_cast<uint2*>(lp + o) = *reinterpret_cast<const uint2*>(b);
    }
  }
}

template <int EPI, int TM, int TN, int WM, int WN, int NT>
DGT_DEVICE void epilogue_staged(const GemmArgs& g, const f32x4 (&acc)[WM / 16][WN / 16], u16* tile, int m0, int n0,
                                int wr, int wc, int l, int tid) {
  __syncthreads();  // every wave has finished reading the operand stages
#pragma unroll
  for (int j = 0; j < WN / 16; ++j) {
    const int nl = wc * WN + j * 16 + (l & 15);
    const float bn = (EPI & kEpiBias) ? g.bias[n0 + nl] : 0.f;
#pragma unroll
    for (int i = 0; i < WM / 16; ++i) {
      const int ml = wr * WM + i * 16 + 4 * (l >> 4);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float x = acc[i][j][rr] * g.alpha + bn;
        if (EPI & kEpiRelu) x = fmaxf(x, 0.f);
        tile[etile<TN>(ml + rr, nl)] = f2bf(x);
      }
    }
  }
  __syncthreads();
  const u16* mask = static_cast<const u16*>(g.mask);
  u16* C = static_cast<u16*>(g.C);
  constexpr int CPR = TN / 8;  // 16-byte chunks per row
  if ((EPI & kEpiMask) || C) {
#pragma unroll
    for (int it = 0; it < TM * CPR / NT; ++it) {
      const int idx = tid + NT * it, r = idx / CPR, c = (idx % CPR) * 8;
      uint4 v = *reinterpret_cast<const uint4*>(tile + etile<TN>(r, c));
      if (EPI & kEpiMask) {
        const uint4 mk = *reinterpret_cast<const uint4*>(mask + (long long)(m0 + r) * g.ldmask + n0 + c);
        unsigned* vw = reinterpret_cast<unsigned*>(&v);
        const unsigned* mw = reinterpret_cast<const unsigned*>(&mk);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned lo = bf2f(mw[e] & 0xffff) > 0.f ? 0x0000ffffu : 0u;
          const unsigned hi = __uint_as_float(mw[e] & 0xffff0000u) > 0.f ? 0xffff0000u : 0u;
          vw[e] &= lo | hi;
        }
        if (EPI & kEpiStoreT) *reinterpret_cast<uint4*>(tile + etile<TN>(r, c)) = v;
      }
      if (C) *reinterpret_cast<uint4*>(C + (long long)(m0 + r) * g.ldc + n0 + c) = v;
    }
  }
  if (EPI & kEpiStoreT) {
    if (EPI & kEpiMask) __syncthreads();
    u16* CT = static_cast<u16*>(g.CT);
    constexpr int CPC = TM / 8;  // 8-row chunks per column
#pragma unroll
    for (int it = 0; it < TN * CPC / NT; ++it) {
      const int idx = tid + NT * it, n = idx / CPC, mc = (idx % CPC) * 8;
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)tile[etile<TN>(mc + 2 * e, n)] | ((unsigned)tile[etile<TN>(mc + 2 * e + 1, n)] << 16);
      *reinterpret_cast<uint4*>(CT + (long long)(n0 + n) * g.ldct + m0 + mc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// S = 2: two stages (64 KiB), two blocks per CU, plain vmcnt(0) + barrier per K-step.
// S > 2: S stages (S x 32 KiB), one block per CU, S-1 K-tiles in flight: the wait before K-tile kt
// is a counted vmcnt (every glds but the newest (S-2) tiles' 8 per thread) and the barrier is a raw
// s_barrier, so the prefetches stay in flight across it (a __syncthreads would drain them).  For
// grids that fit the chip in one wave of blocks this hides HBM latency the 2-stage loop exposes.
template <int N>
DGT_DEVICE void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// NW = 4: waves 2 (M) x 2 (N), 64 x 64 each (4 x 4 accumulators).  NW = 8: waves 2 x 4, 64 x 32
// each: two waves per SIMD, so one wave's LDS fragment reads overlap the other's MFMAs (the
// 4-wave block leaves the matrix core idle while its only wave waits on LDS).
// BK = 128 (S = 2 only, 128 KiB of LDS, one block per CU): hipBLASLt's macro-tile depth -- half the
// barriers and vmcnt drains per FLOP of BK = 64, and 4 MFMA k-steps between them instead of 2.
// G = 2 (S = 5, 160 KiB): the same halved barrier count at BK = 64 granularity -- one barrier per
// two K-tiles, three K-tiles (96 KiB) in flight behind the pair being computed, as deep as the
// 4-stage loop, where BK = 128 x 2 stages keeps only one 64 KiB tile ahead (cold operands stall it).
template <int EPI, int S, int NW = 4, int BK = GBK, int G = 1>
__global__ __launch_bounds__(64 * NW, (S == 2 && BK == GBK) ? 2 : 1) void gemm_nt_kernel(GemmArgs g) {
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

// ------------------------------------------------------------------ 256 x 256 tile, 8-phase pipeline
// For large M x N (>= ~200 tiles): 512 threads = 8 waves in 2 (M) x 4 (N), each wave 128 x 64 =
// 8 x 4 accumulators of 16x16 (128 VGPRs).  A K-tile (BK = 64) of A and of B is staged as four
// 16 KiB "units" of 128 rows, split so that each unit is read in exactly ONE phase:
//   A_lo: block rows with (row % 128) < 64    read in phase q0 (rows 0..63 of every wave)
//   A_hi: block rows with (row % 128) >= 64   read in phase q2
//   B_lo: block cols with (col % 64) < 32     read in phase q0
//   B_hi: block cols with (col % 64) >= 32    read in phase q1
// A K-tile is consumed in four phases, one output quadrant (64 x 32 per wave, 16 MFMAs) each:
//   q0: A_lo x B_lo (reads A_lo, B_lo)   q1: A_lo x B_hi (reads B_hi)
//   q2: A_hi x B_hi (reads A_hi)         q3: A_hi x B_lo (no reads)
// Two LDS buffers (even / odd K-tile) = 128 KiB; one loop iteration = 8 phases = 2 K-tiles.  Each
// phase issues ONE unit of staging (2 global_load_lds per thread), its LDS reads, then
// `s_waitcnt vmcnt(10)` (every unit but the 5 newest has landed), barrier, MFMAs, barrier.  The
// unit order below restages a unit at least one phase after its last read (WAR) and reads it at
// least one phase after the wait that retires it (RAW), so loads stay in flight across 5 phases
// and never drain in the main loop (cdna_hip_programming.md §5, "8-phase template").
namespace g256 {
constexpr int BM = 256, BN = 256, BK = 64, UNIT = 128 * BK;  // elements per unit
enum Unit { kALo = 0, kAHi = 1, kBLo = 2, kBHi = 3 };

// LDS row u of a unit holds global chunk c at slot c ^ ((u >> 1) & 7): a 16-lane group reading 16
// consecutive rows at one chunk then touches 16 distinct 16-byte bank slots (conflict-free).
DGT_DEVICE int swz(int u, int c) { return c ^ ((u >> 1) & 7); }

// Per-lane staging offsets (elements, 32-bit) for the two glds of a unit; the unit/tile part of
// the address is wave-uniform and added to the base pointer, so each glds needs one VGPR.
//   A units: unit row u -> block row (u >> 6) * 128 + (u & 63) (+64 for A_hi)
//   B units: unit row u -> block col (u >> 5) * 64 + (u & 31)  (+32 for B_hi)
DGT_DEVICE int lane_off(bool is_a, int ld, int w, int i, int l) {
  const int u = (w * 2 + i) * 8 + (l >> 3);
  const int row = is_a ? (u >> 6) * 128 + (u & 63) : (u >> 5) * 64 + (u & 31);
  return row * ld + swz(u, l & 7) * 8;
}

DGT_DEVICE void stage(const u16* ubase, const int (&off)[2], u16* unit_lds, int w) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(ubase + off[i]),
                                     reinterpret_cast<int*>(unit_lds + (w * 2 + i) * 8 * BK), 16, 0, 0);
}

DGT_DEVICE bf16x8 frag(const u16* unit_lds, int u, int c) {
  return *reinterpret_cast<const bf16x8*>(unit_lds + u * BK + swz(u, c) * 8);
}

// s_waitcnt with only the vector-memory count constrained (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4]
// << 14, expcnt[6:4] = 7 and lgkmcnt[11:8] = 15 mean "don't wait")
template <int N>
DGT_DEVICE void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
DGT_DEVICE void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }

struct Frags {
  bf16x8 a[4][2];    // the wave's current 64 A rows x K 64 (lo or hi half)
  bf16x8 blo[2][2];  // 32 B columns x K 64
  bf16x8 bhi[2][2];
};

struct Ctx {
  const u16* A;      // block's A panel: A + m0 * lda
  const u16* B;      // block's B panel: B + n0 * ldb
  int lda, ldb, w, l, wr, wc;
  int offa[2], offb[2];
  u16* lds;
};

template <int U>
DGT_DEVICE void stage_unit(const Ctx& c, int kt, int buf) {
  const bool is_a = (U == kALo || U == kAHi);
  const u16* ubase = is_a ? c.A + (U == kAHi ? 64 * c.lda : 0) + kt * BK
                          : c.B + (U == kBHi ? 32 * c.ldb : 0) + kt * BK;
  stage(ubase, is_a ? c.offa : c.offb, c.lds + (buf * 4 + U) * UNIT, c.w);
}

// unit staged in phase P (1..8) of an iteration: ph1 -> the odd tile's A_hi; ph2..5 -> the next
// even tile; ph6..8 -> the next odd tile's A_lo, B_lo, B_hi
template <int P>
DGT_DEVICE void stage_phase(const Ctx& c, int it) {
  constexpr int unit = P == 1 ? kAHi : P == 2 ? kALo : P == 3 ? kBLo : P == 4 ? kBHi : P == 5 ? kAHi
                     : P == 6 ? kALo : P == 7 ? kBLo : kBHi;
  constexpr int buf = (P == 1 || P >= 6) ? 1 : 0;
  const int kt = P == 1 ? 2 * it + 1 : (P <= 5 ? 2 * it + 2 : 2 * it + 3);
  stage_unit<unit>(c, kt, buf);
}

template <int P, bool LAST>
DGT_DEVICE void phase(const Ctx& c, int it, Frags& f, f32x4 (&acc)[8][4]) {
  constexpr int buf = P <= 4 ? 0 : 1;
  constexpr int q = (P - 1) & 3;
  const u16* base = c.lds + buf * 4 * UNIT;
  const int lr = c.l & 15, lc = c.l >> 4;
  if (!LAST || P == 1) stage_phase<P>(c, it);
  if (q == 0 || q == 2) {
    const u16* ul = base + (q == 0 ? kALo : kAHi) * UNIT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f.a[i][kk] = frag(ul, c.wr * 64 + i * 16 + lr, kk * 4 + lc);
  }
  if (q == 0 || q == 1) {
    const u16* ul = base + (q == 0 ? kBLo : kBHi) * UNIT;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 v = frag(ul, c.wc * 32 + j * 16 + lr, kk * 4 + lc);
        if (q == 0) f.blo[j][kk] = v;
        else f.bhi[j][kk] = v;
      }
  }
  // retire the unit read next phase (see the schedule above); the last iteration stages nothing
  // after phase 1, so its counts shrink as the pipeline drains
  if (!LAST) wait_vm<10>();
  else wait_vm<P == 1 ? 10 : P == 2 ? 8 : P == 3 ? 6 : P == 4 ? 4 : P == 5 ? 2 : 0>();
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  wait_lgkm0();
  __builtin_amdgcn_s_setprio(1);
  constexpr int i0 = (q == 0 || q == 1) ? 0 : 4;
  constexpr bool hi_b = (q == 1 || q == 2);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i0 + i][(hi_b ? 2 : 0) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            f.a[i][kk], hi_b ? f.bhi[j][kk] : f.blo[j][kk], acc[i0 + i][(hi_b ? 2 : 0) + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool LAST>
DGT_DEVICE void iteration(const Ctx& c, int it, Frags& f, f32x4 (&acc)[8][4]) {
  phase<1, LAST>(c, it, f, acc);
  phase<2, LAST>(c, it, f, acc);
  phase<3, LAST>(c, it, f, acc);
  phase<4, LAST>(c, it, f, acc);
  phase<5, LAST>(c, it, f, acc);
  phase<6, LAST>(c, it, f, acc);
  phase<7, LAST>(c, it, f, acc);
  phase<8, LAST>(c, it, f, acc);
}
}  // namespace g256

template <int EPI>
__global__ __launch_bounds__(512) void gemm_nt_256_kernel(GemmArgs g) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) u16 lds[2 * 4 * UNIT];  // ONE array (no extra vmcnt(0) waits)
  const int tid = threadIdx.x;
  int tm, tn;
  tile_of_block(blockIdx.x, g.M / BM, g.N / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  Ctx c;
  c.A = static_cast<const u16*>(g.A) + (long long)m0 * g.lda;
  c.B = static_cast<const u16*>(g.B) + (long long)n0 * g.ldb;
  c.lda = g.lda;
  c.ldb = g.ldb;
  c.w = tid >> 6;
  c.l = tid & 63;
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    c.offa[i] = lane_off(true, g.lda, c.w, i, c.l);
    c.offb[i] = lane_off(false, g.ldb, c.w, i, c.l);
  }
  c.lds = lds;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frags f;

  // prologue: the 7 units phases 2..8 of iteration "-1" would have staged (tile 0 whole, tile 1
  // without A_hi), then the wait phase 8 would have done
  stage_unit<kALo>(c, 0, 0);
  stage_unit<kBLo>(c, 0, 0);
  stage_unit<kBHi>(c, 0, 0);
  stage_unit<kAHi>(c, 0, 0);
  stage_unit<kALo>(c, 1, 1);
  stage_unit<kBLo>(c, 1, 1);
  stage_unit<kBHi>(c, 1, 1);
  wait_vm<10>();
  __builtin_amdgcn_s_barrier();

  const int nit = g.K / (2 * BK);
  for (int it = 0; it + 1 < nit; ++it) iteration<false>(c, it, f, acc);
  iteration<true>(c, nit - 1, f, acc);

  if constexpr ((EPI & kEpiAdam) != 0) {
    // fp32 256 x 256 tile = 256 KiB: two passes of 128 rows through the 128 KiB of operand LDS
    epilogue_adam<BM, BN, 128, 64, 512, 128>(g, acc, reinterpret_cast<float*>(lds), m0, n0, c.wr, c.wc, c.l, tid);
  } else if constexpr (!(EPI & kEpiOutF32)) {
    epilogue_staged<EPI, BM, BN, 128, 64, 512>(g, acc, lds, m0, n0, c.wr, c.wc, c.l, tid);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + c.wr * 128 + i * 16 + 4 * (c.l >> 4), n0 + c.wc * 64 + j * 16 + (c.l & 15));
  }
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
static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
static bool sk_fits(const GemmArgs& g) {
  const int T = (g.M % 256 == 0 && g.N % 128 == 0) ? (g.M / 256) * (g.N / 128) : 0;
  return T > 0 && T % 8 == 0 && g.K % 128 == 0 && g.sk_slab && g.sk_flags;
}

hipError_t gemm_nt(const GemmArgs& g, int epi, hipStream_t stream, int variant) {
  if (g.M % GBM || g.N % GBN || g.K % GBK || g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  // split-K 256 x 128 (variant 5) on request only: on the M = 1024 MLP products it ties the 8-wave
  // 128 x 128 kernel (fwd 46.2 vs 48.1 us hot, 53.9 vs 53.4 cold; dgrad 50.7 vs 49.5 hot,
  // profiles/r2_gemm_m1024.jsonl), so the shape-picked default stays the 128 x 128 kernel
  if (variant == 6) {
    if (epi != kEpiAdam || g.K != wsa::NK * wsa::BK || g.M % wsa::BM || g.N % wsa::BN) return hipErrorInvalidValue;
    const int T = (g.M / wsa::BM) * (g.N / wsa::BN);
    hipLaunchKernelGGL(gemm_wgrad_adam_ws_kernel, dim3(std::min(T, cu_count())), dim3(wsa::NT), 0, stream, g);
    return hipGetLastError();
  }
  const bool sk_epi = !(epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam));
  if (variant == 5 && (!sk_fits(g) || !sk_epi)) return hipErrorInvalidValue;
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
    if (bk128) hipLaunchKernelGGL((gemm_nt_kernel<E, 2, 8, 2 * GBK>), dim3(grid), dim3(512), 0, stream, g); \
    else if (pair) hipLaunchKernelGGL((gemm_nt_kernel<E, 5, 8, GBK, 2>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else if (deep) hipLaunchKernelGGL((gemm_nt_kernel<E, 4>), dim3(grid), dim3(256), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
#define DGT_EPI_CASE(E)                                                                           \
  case E:                                                                                         \
    if (single) hipLaunchKernelGGL((gemm_nt_256s_kernel<E>), dim3(grid), dim3(512), 0, stream, g); \
    else if (big) hipLaunchKernelGGL((gemm_nt_256_kernel<E>), dim3(grid), dim3(512), 0, stream, g); \
    else if (bk128) hipLaunchKernelGGL((gemm_nt_kernel<E, 2, 8, 2 * GBK>), dim3(grid), dim3(512), 0, stream, g); \
    else if (pair) hipLaunchKernelGGL((gemm_nt_kernel<E, 5, 8, GBK, 2>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else if (deep) hipLaunchKernelGGL((gemm_nt_kernel<E, 4>), dim3(grid), dim3(256), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
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

// Full 64 x 64 tiles: one wave per tile, lane (rb, cg) moves the 8 x 8 block rows 8rb.., cols 8cg..
// entirely in registers: eight 16-byte row loads, eight 16-byte transposed row stores (8 lanes
// cover one 128-byte line on both sides), no LDS and no barrier.
__global__ __launch_bounds__(256) void transpose_bf16_tile_kernel(const u16* __restrict__ in, u16* __restrict__ out,
                                                                  int rows, int cols) {
  const int l = threadIdx.x & 63, cg = l & 7, rb = l >> 3;
  const int r = blockIdx.y * 64 + rb * 8, c = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64 + cg * 8;
  uint4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const uint4*>(in + (long long)(r + k) * cols + c);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned lo = (&v[2 * q].x)[e >> 1], hi = (&v[2 * q + 1].x)[e >> 1];
      o[q] = (e & 1) ? ((lo >> 16) | (hi & 0xffff0000u)) : ((lo & 0xffffu) | (hi << 16));
    }
    *reinterpret_cast<uint4*>(out + (long long)(c + e) * rows + r) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

hipError_t transpose_bf16(const void* in, void* out, int rows, int cols, hipStream_t stream) {
  if (rows % 64 == 0 && cols % 64 == 0) {  // 4 tiles per block side by side when the width allows
    const int wpb = cols % 256 == 0 ? 4 : 1;
    hipLaunchKernelGGL(transpose_bf16_tile_kernel, dim3(cols / (64 * wpb), rows / 64), dim3(64 * wpb), 0, stream,
                       static_cast<const u16*>(in), static_cast<u16*>(out), rows, cols);
    return hipGetLastError();
  }
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
#pragma unroll 4  // the row's 16-byte loads in flight together (same summation order)
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
// g[b,:] = dz[b] * w * 1[a[b,:] > 0] (bf16, and g^T); dw = sum_b dz[b] a[b,:]; db = sum_b dz[b].
// Kernel 1: one row per wave (every 16-byte load of the row in flight together) computes
// z, dz and the row's loss term into a scratch vector, and zeroes dw.  No atomics: 1024 float /
// double atomics on ONE address serialised at the L2 and made this kernel 19 us.
// Kernel 2: one wave per 64 x 64 tile, 16-byte rows of a in, 16-byte rows of g and g^T out, dw
// accumulated with one atomic per column per tile; tile (0, 0) also reduces dz -> db and the row
// losses -> loss_acc in a fixed order (one atomic).
__global__ __launch_bounds__(256) void head_fwd_kernel(const u16* __restrict__ a, const float* __restrict__ w,
                                                       const float* __restrict__ b0, const float* __restrict__ y,
                                                       int B, int D, float* __restrict__ dz,
                                                       float* __restrict__ lrow, float* __restrict__ dw) {
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < D; i += gridDim.x * 256) dw[i] = 0.f;
  constexpr int R = 1;
  const int row0 = blockIdx.x * 4 + wv * R;
  float s[R] = {0.f};
#pragma unroll 8
  for (int c = l * 8; c < D; c += 64 * 8) {  // unrolled: a row's loads are in flight together
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + c), w1 = *reinterpret_cast<const f32x4*>(w + c + 4);
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = *reinterpret_cast<const uint4*>(a + (long long)(row0 + r) * D + c);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      s[r] += bf2f(v[r].x & 0xffff) * w0[0] + bf2f(v[r].x >> 16) * w0[1] + bf2f(v[r].y & 0xffff) * w0[2] +
              bf2f(v[r].y >> 16) * w0[3] + bf2f(v[r].z & 0xffff) * w1[0] + bf2f(v[r].z >> 16) * w1[1] +
              bf2f(v[r].w & 0xffff) * w1[2] + bf2f(v[r].w >> 16) * w1[3];
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) s[r] = wave_sum(s[r]);
  if (l < R) {
    float sr = s[0];
#pragma unroll
    for (int r = 1; r < R; ++r) sr = l == r ? s[r] : sr;
    const int row = row0 + l;
    const float z = sr + *b0, yy = y[row];
    const float e = __expf(-fabsf(z));
    const float sig = z >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
    dz[row] = (sig - yy) / (float)B;
    lrow[row] = ((1.f - yy) * z - (fminf(z, 0.f) - log1pf(e))) / (float)B;
  }
}

__global__ __launch_bounds__(256) void head_bwd_kernel(const u16* __restrict__ a, const float* __restrict__ w,
                                                      const float* __restrict__ dz,
                                                      const float* __restrict__ lrow, int B, int D,
                                                      u16* __restrict__ g, u16* __restrict__ gT,
                                                      float* __restrict__ dw, float* __restrict__ db,
                                                      double* __restrict__ loss_acc) {
  // one wave per 64 x 64 tile; lane (rb, cg) owns the 8 x 8 block rows r0 + 8rb.., cols c0 + 8cg..:
  // eight 16-byte row loads of a, eight 16-byte g row stores (8 lanes = one 128-byte line) and
  // eight 16-byte g^T row stores (8 consecutive rows of one column): no LDS
  const int l = threadIdx.x & 63, cg = l & 7, rb = l >> 3, wv = threadIdx.x >> 6;
  const int r = blockIdx.y * 64 + rb * 8, c = (blockIdx.x * (blockDim.x >> 6) + wv) * 64 + cg * 8;
  const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + c), w1 = *reinterpret_cast<const f32x4*>(w + c + 4);
  const float wc[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
  uint4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const uint4*>(a + (long long)(r + k) * D + c);
  float part[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  u16 gb[8][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float d = dz[r + k];
    const unsigned u[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    unsigned o[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float av = bf2f((u16)(e & 1 ? u[e >> 1] >> 16 : u[e >> 1] & 0xffff));
      part[e] += d * av;
      gb[k][e] = f2bf(av > 0.f ? d * wc[e] : 0.f);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (unsigned)gb[k][2 * q] | ((unsigned)gb[k][2 * q + 1] << 16);
    *reinterpret_cast<uint4*>(g + (long long)(r + k) * D + c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (unsigned)gb[2 * q][e] | ((unsigned)gb[2 * q + 1][e] << 16);
    *reinterpret_cast<uint4*>(gT + (long long)(c + e) * B + r) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  // dw: sum the 8 row-blocks (lanes cg, cg + 8, ..., cg + 56), one atomic per column per tile
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float x = part[e];
    x += __shfl_xor(x, 8);
    x += __shfl_xor(x, 16);
    x += __shfl_xor(x, 32);
    part[e] = x;
  }
  if (rb == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(&dw[c + e], part[e]);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && wv == 0) {  // db and the step's loss, in a fixed order
    float sd = 0.f, sl = 0.f;
    for (int i = l; i < B; i += 64) {
      sd += dz[i];
      sl += lrow[i];
    }
    sd = wave_sum(sd);
    sl = wave_sum(sl);
    if (l == 0) {
      *db = sd;
      atomicAdd(loss_acc, (double)sl);
    }
  }
}

hipError_t mlp_head(const HeadArgs& h, hipStream_t stream) {
  if (h.B % 64 || h.D % 64 || !h.scratch) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(h.B / 4), dim3(256), 0, stream, static_cast<const u16*>(h.a), h.w,
                     h.b0, h.y, h.B, h.D, h.dz, h.scratch, h.dw);
  const int wpb = h.D % 256 == 0 ? 4 : 1;  // 4 tiles per block side by side when the width allows
  hipLaunchKernelGGL(head_bwd_kernel, dim3(h.D / (64 * wpb), h.B / 64), dim3(64 * wpb), 0, stream,
                     static_cast<const u16*>(h.a),
                     h.w, h.dz, h.scratch, h.B, h.D, static_cast<u16*>(h.g), static_cast<u16*>(h.gT), h.dw, h.db,
                     h.loss_acc);
  return hipGetLastError();
}

}  // namespace dgt
