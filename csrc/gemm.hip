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
#include <cstdlib>
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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
// LDS-DMA issued from inline asm (FR kernel): the compiler's waitcnt insertion treats a
// global_load_lds it can see as an LDS event and then drains every ds_read with lgkmcnt(0) before
// the first MFMA that uses one; hidden in asm it counts the reads (lgkmcnt(N)).  The caller owns
// the DMA's vmcnt accounting (wait_vmcnt) and its ordering against LDS reads (s_barrier).  M0 is
// saved and restored around the DMA's use of it.
DGT_DEVICE unsigned lds_byte_addr(const void* p) {
  return (unsigned)(uintptr_t)((__attribute__((address_space(3))) const char*)(p));
}
DGT_DEVICE void glds_asm(const u16* gptr, unsigned la) {  // la: wave-uniform LDS byte address
  unsigned saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(gptr), "s"(la)
      : "memory");
}

template <int NWAVE, bool KN, bool ASM = false>
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
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) lds_b[i] = __builtin_amdgcn_readfirstlane((unsigned)lds_off[i] * 2u);
  }
  unsigned lds_b[PER_WAVE];  // ASM: byte offsets of the pieces, in SGPRs
  DGT_DEVICE void issue(u16* lds) {
    if constexpr (ASM) {  // one address-space cast per tile; the pieces are scalar adds
      issue_at(__builtin_amdgcn_readfirstlane(lds_byte_addr(lds)));
      return;
    }
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(p[i]), reinterpret_cast<int*>(lds + lds_off[i]),
                                       16, 0, 0);
      p[i] += step;
    }
  }
  DGT_DEVICE void issue_at(unsigned tile_base) {  // ASM only: LDS byte address of the operand tile
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      glds_asm(p[i], tile_base + lds_b[i]);
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

// read_frag_kn through the compiler builtin (FR kernel: with the LDS-DMA hidden in asm the compiler
// counts these reads like any ds_read instead of draining the staging pipeline before each one)
DGT_DEVICE bf16x8 read_frag_kn_fr(const u16* lds, int kb, int nb, int l) {
  const int q = (l >> 2) & 3, col = nb + 4 * (l & 3);
  const int r0 = kb + 8 * (l >> 4) + q, r1 = r0 + 4;
  const u16* a0 = lds + r0 * GBN + (((col >> 3) ^ kn_swz(r0)) << 3) + (col & 4);
  const u16* a1 = lds + r1 * GBN + (((col >> 3) ^ kn_swz(r1)) << 3) + (col & 4);
  typedef short __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) * p4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((p4)((__attribute__((address_space(3))) const u16*)(a0)));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((p4)((__attribute__((address_space(3))) const u16*)(a1)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

DGT_DEVICE float bias_at(const GemmArgs& g, int n) {
  return g.bias_bf16 ? bf2f(static_cast<const u16*>(g.bias)[n]) : static_cast<const float*>(g.bias)[n];
}

// One MFMA accumulator (rows mb..mb+3 of column n) through the fused epilogue.
template <int EPI>
DGT_DEVICE void epi_store(const GemmArgs& g, const f32x4& acc, int mb, int n) {
  const float bn = (EPI & kEpiBias) ? bias_at(g, n) : 0.f;
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
// is a 16-byte vector.  Tile rows are whole multiples of 32 banks, so only the 16-byte chunk index
// can separate rows: its low 4 bits are XOR-swizzled by (row / 8) ^ (bit 2 of the row << 1).
//   MFMA-layout writes (2-byte, banks mod 32): a 32-lane half writes 16 columns (chunks {x, x^1}) of
//     rows r and r + 4; bit 2 moves row r + 4 to chunks {x^2, x^3}: disjoint banks.
//   C row reads (16 B, banks mod 64): 16 lanes per row, 2 rows per 16-lane group with equal swizzle.
//   C^T column reads (2-byte, banks mod 32): a 32-lane half reads 4 adjacent columns (one chunk) of 8
//     row blocks 8k + e, k = 8 consecutive values: 8 distinct chunk residues mod 8.
// Values are rounded to bf16 once (after bias / ReLU) and masked after rounding (identical results:
// the mask only zeroes).
template <int TN>
DGT_DEVICE int etile(int r, int n) {
  const int c = n >> 3;
  return r * TN + ((((c ^ (r >> 3) ^ (((r >> 2) & 1) << 1)) & 15) | (c & ~15)) << 3) + (n & 7);
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
      // the optimizer state streams through once per step: nontemporal loads and stores keep it
      // from evicting the GEMM operands other blocks are still reading (DGT_ADAM_EPI_NT=0: plain)
      f32x4 p, m, v;
      if (g.adam_nt) {
        p = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.master + o));
        m = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.m + o));
        v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.v + o));
      } else {
        p = *reinterpret_cast<const f32x4*>(a.master + o);
        m = *reinterpret_cast<const f32x4*>(a.m + o);
        v = *reinterpret_cast<const f32x4*>(a.v + o);
      }
      __hip_bfloat16 b[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float mm = m[e], vv = v[e];
        p[e] = adam_update(p[e], gr[e], mm, vv, a.hp, a.step_size_neg, a.bc2_sqrt);
        m[e] = mm;
        v[e] = vv;
        b[e] = __float2bfloat16(p[e]);
      }
      if (g.adam_nt) {
        __builtin_nontemporal_store(p, reinterpret_cast<f32x4*>(a.master + o));
        __builtin_nontemporal_store(m, reinterpret_cast<f32x4*>(a.m + o));
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.v + o));
      } else {
        *reinterpret_cast<f32x4*>(a.master + o) = p;
        *reinterpret_cast<f32x4*>(a.m + o) = m;
        *reinterpret_cast<f32x4*>(a.v + o) = v;
      }
      *reinterpret_cast<uint2*>(lp + o) = *reinterpret_cast<const uint2*>(b);  // read by the next forward
    }
  }
}

// What the staged epilogue reads from memory, loadable ahead: the bias of a wave's WN / 16
// accumulator columns (nb + 16 j + (l & 15)) and the ReLU-mask chunks of the thread's C-row passes.
// Read where they are used, each load's latency is exposed in turn (a vmcnt(0) after each: the
// compiler cannot move a mask load above the previous pass's C store).
template <int EPI, int TM, int TN, int WN, int NT>
struct EpiPre {
  static constexpr int NB = WN / 16, CPR = TN / 8;
  static constexpr int NMK = (EPI & kEpiMask) ? TM * CPR / NT : 1;
  float bn[NB];
  uint4 mk[NMK];
  DGT_DEVICE void load_bias(const GemmArgs& g, int nb, int l) {
    if constexpr ((EPI & kEpiBias) != 0) {
      if (g.bias_bf16) {
        const u16* b = static_cast<const u16*>(g.bias) + nb + (l & 15);
#pragma unroll
        for (int j = 0; j < NB; ++j) bn[j] = bf2f(b[16 * j]);
      } else {
        const float* b = static_cast<const float*>(g.bias) + nb + (l & 15);
#pragma unroll
        for (int j = 0; j < NB; ++j) bn[j] = b[16 * j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) bn[j] = 0.f;
    }
  }
  DGT_DEVICE void load_mask(const GemmArgs& g, int m0, int n0, int tid) {
    if constexpr ((EPI & kEpiMask) != 0) {
      const u16* mask = static_cast<const u16*>(g.mask);
#pragma unroll
      for (int it = 0; it < NMK; ++it) {
        const int idx = tid + NT * it, r = idx / CPR, c = (idx % CPR) * 8;
        mk[it] = *reinterpret_cast<const uint4*>(mask + (long long)(m0 + r) * g.ldmask + n0 + c);
      }
    }
  }
};

// PRE: the bias and mask come from `pre` (loaded ahead by the split-K kernel); otherwise they are
// read here, where used (the 128 x 128 / 256 x 256 kernels: issuing them ahead of the K loop, or
// batched at the epilogue, measured no faster in the MLP step -- 1,406-1,413 vs 1,411-1,417 iters/s,
// scripts/sessions/gpu_r6_epi.sh)
template <int EPI, int TM, int TN, int WM, int WN, int NT, bool PRE = false>
DGT_DEVICE void epilogue_staged(const GemmArgs& g, const f32x4 (&acc)[WM / 16][WN / 16], u16* tile, int m0, int n0,
                                int wr, int wc, int l, int tid, const EpiPre<EPI, TM, TN, WN, NT>& pre,
                                bool own = true) {
  __syncthreads();  // every wave has finished reading the operand stages
  // (own = false: this wave holds none of the tile's accumulators -- the split-K kernel's half
  // epilogue -- and only joins the store passes)
#pragma unroll
  for (int j = 0; j < WN / 16 && own; ++j) {
    const int nl = wc * WN + j * 16 + (l & 15);
    float bnj;
    if constexpr (PRE) bnj = pre.bn[j];
    else bnj = (EPI & kEpiBias) ? bias_at(g, n0 + nl) : 0.f;
#pragma unroll
    for (int i = 0; i < WM / 16; ++i) {
      const int ml = wr * WM + i * 16 + 4 * (l >> 4);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float x = acc[i][j][rr] * g.alpha + bnj;
        if (EPI & kEpiRelu) x = fmaxf(x, 0.f);
        tile[etile<TN>(ml + rr, nl)] = f2bf(x);
      }
    }
  }
  __syncthreads();
  u16* C = static_cast<u16*>(g.C);
  constexpr int CPR = TN / 8;  // 16-byte chunks per row
  if ((EPI & kEpiMask) || C) {
#pragma unroll
    for (int it = 0; it < TM * CPR / NT; ++it) {
      const int idx = tid + NT * it, r = idx / CPR, c = (idx % CPR) * 8;
      uint4 v = *reinterpret_cast<const uint4*>(tile + etile<TN>(r, c));
      if constexpr ((EPI & kEpiMask) != 0) {
        uint4 mk;
        if constexpr (PRE) mk = pre.mk[it];
        else mk = *reinterpret_cast<const uint4*>(static_cast<const u16*>(g.mask) + (long long)(m0 + r) * g.ldmask + n0 + c);
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
      if (C) {
        uint4* dst = reinterpret_cast<uint4*>(C + (long long)(m0 + r) * g.ldc + n0 + c);
        if (EPI & kEpiAccumulate) {  // bf16 C += result: the sum in fp32, rounded once
          const uint4 o = *dst;
          unsigned* vw = reinterpret_cast<unsigned*>(&v);
          const unsigned* ow = reinterpret_cast<const unsigned*>(&o);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = bf2f(vw[e] & 0xffff) + bf2f(ow[e] & 0xffff);
            const float hi = __uint_as_float(vw[e] & 0xffff0000u) + __uint_as_float(ow[e] & 0xffff0000u);
            vw[e] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
          }
        }
        *dst = v;
      }
    }
  }
  if (EPI & kEpiStoreT) {
    if (EPI & kEpiMask) __syncthreads();
    u16* CT = static_cast<u16*>(g.CT);
    constexpr int CPC = TM / 8;  // 8-row chunks per column
    static_assert(CPC % 16 == 0 && NT % 64 == 0, "C^T read mapping: 16-chunk blocks per wave");
    static_assert(!(EPI & kEpiColSum) || CPC == 16 || CPC == 32, "column sums: per 128-row block of the tile");
#pragma unroll
    for (int it = 0; it < TN * CPC / NT; ++it) {
      // a wave reads 4 columns x 16 row chunks; each 32-lane half 4 columns x 8 row chunks
      const int idx = tid + NT * it, sub = idx % (4 * CPC), q = sub & 63;
      const int n = (idx / (4 * CPC)) * 4 + ((q & 31) >> 3);
      const int mc = ((q & 7) + 8 * (q >> 5) + 16 * (sub >> 6)) * 8;
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)tile[etile<TN>(mc + 2 * e, n)] | ((unsigned)tile[etile<TN>(mc + 2 * e + 1, n)] << 16);
      *reinterpret_cast<uint4*>(CT + (long long)(n0 + n) * g.ldct + m0 + mc) = make_uint4(w[0], w[1], w[2], w[3]);
      if constexpr ((EPI & kEpiColSum) != 0) {
        // the column's 16 chunks sit in the 16 lanes that differ in lane bits 0-2 and 5: sum the
        // lane's 8 values, then a fixed xor tree over those bits (the same order on every call)
        float cs = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) cs += bf2f((u16)(w[e] & 0xffff)) + __uint_as_float(w[e] & 0xffff0000u);
        cs += __shfl_xor(cs, 1);
        cs += __shfl_xor(cs, 2);
        cs += __shfl_xor(cs, 4);
        cs += __shfl_xor(cs, 32);
        // (a 256-row tile: sub >> 6 picks the 128-row half, one partial row each)
        if ((q & 0x27) == 0) g.colsum[(long long)(m0 / 128 + (sub >> 6)) * g.N + n0 + n] = cs;
      }
    }
  }
}

// S = 2: two stages (64 KiB), two blocks per CU, plain vmcnt(0) + barrier per K-step.
// S = 4: four stages (128 KiB), one block per CU, two K-tiles in flight: the wait before K-tile kt
// is a counted vmcnt (every glds but the newest 2 tiles' per thread) and the barrier is a raw
// s_barrier, so the prefetches stay in flight across it (a __syncthreads would drain them).  For
// grids that fit the chip in one wave of blocks this hides HBM latency the 2-stage loop exposes.
template <int N>
DGT_DEVICE void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// NW = 4: waves 2 (M) x 2 (N), 64 x 64 each (4 x 4 accumulators).  NW = 8: waves 2 x 4, 64 x 32
// each: two waves per SIMD, so one wave's LDS fragment reads overlap the other's MFMAs (the
// 4-wave block leaves the matrix core idle while its only wave waits on LDS).
// (Round-2 BK = 128 / two-K-tiles-per-barrier forms of this loop: git history, commit c0371a5.)
// FR (front-loaded fragment reads): each wave issues ALL its ds_reads of a K-tile
// (both 32-deep halves) before its first MFMA and lets counted lgkmcnt waits release the MFMAs as
// fragments land.  After the per-K-tile barrier all waves otherwise move in lockstep through
// read -> lgkmcnt(0) -> 4 MFMAs phases, so the LDS and the matrix cores take turns instead of
// overlapping.
// (Round-3 forms measured and removed, records in profiles/r3_gemm_m1024.jsonl: one barrier per two
// K-tiles -- fastest hot, loses cold and in the MLP step; five stages, three K-tiles in flight -- no
// gain in the step.  Source: git history, commits fd01625 and 45106c5.)
// FR = 3 (SP, software-pipelined reads; S = 5, all 160 KiB of LDS): K-tile kt+1's fragments are read
// into a second register set while tile kt's MFMAs run, so no MFMA waits on an LDS round trip of
// its own K-tile; the barrier of step kt publishes tile kt+1 (one K-tile earlier than FR = 1), and
// five stages keep the same two to three K-tiles of staging in flight.
// SPK (split-K, small grids): g.skn_split blocks per tile, block s taking K-slice s; the slices meet
// in-launch -- each block writes its fp32 partial (64 KiB, write-through sc1 stores), drains and
// adds to the tile's counter; the block whose add comes last sums every partial in slice order
// (fixed, so the bits do not depend on arrival order), re-arms the counter and runs the epilogue
// (MI355X_MICROARCH.md visibility, valid forms, first row: the last adder is told by its add).
template <int EPI, int S, int NW = 4, int FR = 0, bool SPK = false>
__global__ __launch_bounds__(64 * NW, S == 2 ? 2 : 1) void gemm_nt_kernel(GemmArgs g) {
  static_assert(S == 2 || S == 4 || (S == 5 && FR == 3), "two stages (2 blocks / CU), four (1 block / CU), or SP");
  static_assert(!SPK || (S == 4 && NW == 8 && FR == 1), "split-K: the FR kernel");
  constexpr int BK = GBK;
  constexpr bool KN = (EPI & kEpiBKN) != 0;      // B is [K, N]: staged as is, transposed reads
  constexpr int WN = NW == 8 ? 32 : 64;          // wave tile columns
  constexpr int WCOLS = GBN / WN;                // waves across N
  constexpr int NJ = WN / 16;                    // accumulator columns per wave
  __shared__ __attribute__((aligned(16))) u16 lds[S][2][GBM * BK];  // [stage][A|B], 32 KiB per stage
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int split = SPK ? g.skn_split : 1;
  const int tile = SPK ? (int)blockIdx.x / split : (int)blockIdx.x, slice = SPK ? (int)blockIdx.x % split : 0;
  int tm, tn;
  tile_of_block(tile, g.M / GBM, g.N / GBN, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int wr = w / WCOLS, wc = w % WCOLS;
  const long long kbase = (long long)slice * (g.K / split);
  const u16* A = static_cast<const u16*>(g.A) + kbase;
  const u16* B = static_cast<const u16*>(g.B) + kbase * (KN ? g.ldb : 1);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK / split;
  auto compute = [&](int buf) {
    const u16* As = lds[buf][0];
    const u16* Bs = lds[buf][1];
    if constexpr (FR) {
      // all 12 reads of the K-tile (per 32-deep half: A0..A3, B0, B1) ahead of the 16 MFMAs; the
      // compiler's counted lgkmcnt waits release each MFMA as its two fragments land
      bf16x8 af[BK / 32][4], bfr[BK / 32][NJ];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (l >> 4);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (KN) bfr[kk][j] = read_frag_kn_fr(Bs, kk * 32, wc * WN + j * 16, l);
          else bfr[kk][j] = read_frag<BK>(Bs, wc * WN + j * 16 + (l & 15), chunk);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) af[kk][i] = read_frag<BK>(As, wr * 64 + i * 16 + (l & 15), chunk);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
      // every DS read first, the first half's before the second's (at most 16 in flight, and the
      // first MFMAs wait on the first half only), then the MFMAs
      if constexpr (KN) {  // 16 reads: the second half's go out after the first MFMAs (lgkmcnt <= 15)
        __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ - 2, 0);
      } else {
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) __builtin_amdgcn_sched_group_barrier(0x100, 4 + NJ, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ, 0);
      }
      return;
    }
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
  } else if constexpr (FR == 3) {
    static_assert(S == 5 && NW == 8, "SP: five stages, eight waves");
    constexpr int PER_TILE = 2 * (16 / NW);
    Stager<NW, false, true> sa(A, g.lda, m0, w, l);
    Stager<NW, KN, true> sb(B, g.ldb, n0, w, l);
    const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_byte_addr(&lds[0][0][0]));
    auto tile_at = [&](int b, int o) { return lds0 + (unsigned)((b * 2 + o) * GBM * BK * 2); };
    struct Fr {
      bf16x8 a[BK / 32][4];
      bf16x8 b[BK / 32][NJ];
    };
    auto read_frags = [&](int buf, Fr& fr) {
      const u16* As = lds[buf][0];
      const u16* Bs = lds[buf][1];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int chunk = kk * 4 + (l >> 4);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (KN) fr.b[kk][j] = read_frag_kn_fr(Bs, kk * 32, wc * WN + j * 16, l);
          else fr.b[kk][j] = read_frag<BK>(Bs, wc * WN + j * 16 + (l & 15), chunk);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) fr.a[kk][i] = read_frag<BK>(As, wr * 64 + i * 16 + (l & 15), chunk);
      }
    };
    auto mfmas = [&](const Fr& fr) {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr.a[kk][i], fr.b[kk][j], acc[i][j], 0, 0, 0);
    };
    // prologue: tiles 0..3 staged, tile 0 retired and published, its fragments read
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p < nk) {
        sa.issue_at(tile_at(p, 0));
        sb.issue_at(tile_at(p, 1));
      }
    }
    {
      const int newer = min(3, nk - 1);  // tiles staged after tile 0
      if (newer >= 3) wait_vmcnt<3 * PER_TILE>();
      else if (newer == 2) wait_vmcnt<2 * PER_TILE>();
      else if (newer == 1) wait_vmcnt<PER_TILE>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    Fr f0, f1;
    read_frags(0, f0);
    int rb = 1, nb = 4;  // stage of tile kt + 1, stage the next staged tile lands in (tile % 5)
    // one step: publish tile kt + 1 (its own wait + the barrier), stage tile kt + 4 into the stage
    // tile kt - 1 left (its fragments were consumed by step kt - 1, which every wave has finished),
    // read tile kt + 1 into `nxt`, then tile kt's MFMAs from `cur`
    auto step = [&](int kt, const Fr& cur, Fr& nxt) {
      if (kt + 1 < nk) {
        const int newer = min(2, nk - kt - 2);  // tiles staged after tile kt + 1
        if (newer >= 2) wait_vmcnt<2 * PER_TILE>();
        else if (newer == 1) wait_vmcnt<PER_TILE>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 4 < nk) {
          sa.issue_at(tile_at(nb, 0));
          sb.issue_at(tile_at(nb, 1));
        }
        nb = (nb + 1 == S) ? 0 : nb + 1;
        read_frags(rb, nxt);
        rb = (rb + 1 == S) ? 0 : rb + 1;
        // (the MFMAs inside each branch: after a join the compiler could only wait lgkmcnt(0))
        mfmas(cur);
      } else {
        mfmas(cur);
      }
    };
    for (int kt = 0; kt < nk; kt += 2) {  // nk even (the dispatcher's condition): static register sets
      step(kt, f0, f1);
      step(kt + 1, f1, f0);
    }
    __builtin_amdgcn_s_barrier();
  } else {
    constexpr int PER_TILE = 2 * (16 / NW);  // glds per thread per K-tile (A and B)
    constexpr int AHEAD = S - 2;             // K-tiles left in flight past the one being retired
    Stager<NW, false, FR != 0> sa(A, g.lda, m0, w, l);
    Stager<NW, KN, FR != 0> sb(B, g.ldb, n0, w, l);
    // LDS byte address of operand tile (stage b, operand o): integer arithmetic on one base
    const unsigned lds0 = FR ? __builtin_amdgcn_readfirstlane(lds_byte_addr(&lds[0][0][0])) : 0u;
    auto tile_at = [&](int b, int o) { return lds0 + (unsigned)((b * 2 + o) * GBM * BK * 2); };
#pragma unroll
    for (int p = 0; p < S - 1; ++p) {
      if (p < nk) {
        if constexpr (FR != 0) {
          sa.issue_at(tile_at(p, 0));
          sb.issue_at(tile_at(p, 1));
        } else {
          sa.issue(lds[p][0]);
          sb.issue(lds[p][1]);
        }
      }
    }
    int buf = 0, nb = S - 1;  // buffer of tile kt, buffer the next staged tile lands in (tile % S)
    for (int kt = 0; kt < nk; ++kt) {
      // tiles kt .. min(kt + S - 2, nk - 1) are in flight; retire tile kt
      const int ahead = min(AHEAD, nk - kt - 1);
      if (ahead >= AHEAD) wait_vmcnt<AHEAD * PER_TILE>();
      else if (ahead == 1) wait_vmcnt<PER_TILE>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // tile kt visible to all waves; the buffer of kt - 1 is free for reuse
      __builtin_amdgcn_sched_barrier(0);
#if !(defined(DGT_GEMM_ABLATE) && DGT_GEMM_ABLATE == 1)  // diag: 1 = no staging inside the loop
      if (kt + S - 1 < nk) {
        if constexpr (FR != 0) {
          sa.issue_at(tile_at(nb, 0));
          sb.issue_at(tile_at(nb, 1));
        } else {
          sa.issue(lds[nb][0]);
          sb.issue(lds[nb][1]);
        }
      }
      nb = (nb + 1 == S) ? 0 : nb + 1;
#endif
      compute(buf);
      buf = (buf + 1 == S) ? 0 : buf + 1;
    }
    __builtin_amdgcn_s_barrier();
  }

  if constexpr (SPK) {
    const int t = blockIdx.x / split;  // the tile's index for its partials and counter
    auto part = [&](int q) {
      return __builtin_amdgcn_make_buffer_rsrc(g.sk_slab + ((long long)t * split + q) * (GBM * GBN), 0, GBM * GBN * 4,
                                               0x00020000);
    };
    const auto mine = part(slice);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), mine,
                                               ((i * NJ + j) * 512 + tid) * 16, 0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    int* word = reinterpret_cast<int*>(&lds[0][0][0]);  // the stages are idle
    if (tid == 0) *word = __hip_atomic_fetch_add(g.sk_flags + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*word != split - 1) return;  // not the last slice to arrive
    if (tid == 0) __hip_atomic_store(g.sk_flags + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    // every load of a partial is an sc1 load behind the counter's add and the barrier above
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f32x4 sum[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) sum[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int q = 0; q < split; ++q) {  // slice order: the same sum whoever arrived last
      f32x4 p[4][NJ];
      if (q == slice) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) p[i][j] = acc[i][j];
      } else {
        const auto rs = part(q);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            p[i][j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * NJ + j) * 512 + tid) * 16, 0, 16));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) sum[i][j] += p[i][j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = sum[i][j];
  }

  // ---- epilogue: D col = l&15 (n), row = 4*(l>>4) + r (m)
  if constexpr ((EPI & kEpiAdam) != 0) {
    // fp32 128 x 128 tile = 64 KiB: one pass fits the 2-stage (64 KiB) and 4-stage LDS
    epilogue_adam<GBM, GBN, 64, WN, 64 * NW, GBM>(g, acc, reinterpret_cast<float*>(&lds[0][0][0]), m0, n0, wr, wc, l,
                                                  tid);
  } else if constexpr (!(EPI & kEpiOutF32)) {
    epilogue_staged<EPI, GBM, GBN, 64, WN, 64 * NW>(g, acc, &lds[0][0][0], m0, n0, wr, wc, l, tid,
                                                    EpiPre<EPI, GBM, GBN, WN, 64 * NW>{});
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + wr * 64 + i * 16 + 4 * (l >> 4), n0 + wc * WN + j * 16 + (l & 15));
  }
}

// ------------------------------------------------------------------ 256 x 128 tile, split-K 2 (SK)
// For products whose 128 x 128 grid is one block per CU (the MLP's M = 1024 forward and dgrad at
// N = K = 4096): each CU there streams 2 MiB of operands at the chip's ~13 TB/s L2 -> CU rate
// (profiles/r4_panel_stream.jsonl; the stage depth does not move it), so only fewer bytes per CU
// help.  Here a block owns a 256 x 128 tile over HALF of K: 1.5 MiB per CU for the same FLOPs, and
// 64 x 64 wave tiles (4 (M) x 2 (N) waves of 4 x 4 accumulators: 16 fragment reads per 32 MFMAs,
// against 12 per 16 in the 128 x 128 kernel's 64 x 32 wave tiles).  M = 1024 gives 4 x 32 tiles x
// 2 halves = 256 blocks.  The loop is the FR kernel's (asm LDS-DMA, front-loaded fragment reads,
// counted vmcnt + raw barrier), three 48 KiB stages.
// The halves meet in-launch (cdna_hip_programming.md §5 projection GEMM item 2, §6 Guideline 16)
// per 128-row half of the tile, with static roles: each block publishes its fp32 partial of one row
// half (64 KiB, write-through sc1 16-byte stores, drained, then a compare-and-swap of that half's
// state word) and finishes the other (polls its state word, adds the partner's partial with sc1
// loads -- fp32 a + b == b + a: the sum does not depend on arrival order -- and runs the staged
// epilogue of those 128 rows).  A finisher whose partner has not published within ~20 us hands its
// own partial over instead and leaves the row half to the publisher, so no block waits on a partner
// that is not running (no co-residency is assumed).  Every state word is back at zero after a launch.
// sk_xs = 1 puts a tile's halves on neighbouring XCDs (each XCD's L2 then holds half of K for a
// 4 x 8-tile region: 8 MiB of unique operands per XCD instead of 12), 0 on one XCD.
// agent-scope compare-and-swap (relaxed), returning the value found
DGT_DEVICE int cas_agent(int* p, int expected, int desired) {
  __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return expected;
}

namespace sk {
constexpr int TM = 256, TN = 128, S = 3, NW = 8;
constexpr int A_ELEMS = TM * GBK, STAGE = (TM + TN) * GBK;  // u16 per stage (48 KiB)
constexpr int PER_TILE = 3 * (16 / NW);                      // LDS-DMAs per thread per K-tile (A 4, B 2)
}  // namespace sk

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_nt_sk_kernel(GemmArgs g) {
  using namespace sk;
  constexpr int BK = GBK, NJ = 4;
  constexpr bool KN = (EPI & kEpiBKN) != 0;
  static_assert(!(EPI & (kEpiOutF32 | kEpiAccumulate | kEpiAdam)), "SK: staged bf16 epilogues only");
  // ONE __shared__ array: a second LDS object (even the ticket word) can make the compiler drain
  // the DMAs before every fragment read
  __shared__ __attribute__((aligned(16))) u16 lds[S * STAGE];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const int MT = g.M / TM, T = MT * (g.N / TN);
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  int half, t;
  if (g.sk_xs & 1) {
    half = xcd & 1;
    t = (xcd >> 1) * (T / 4) + slot;
  } else {
    half = slot & 1;
    t = xcd * (T / 8) + (slot >> 1);
  }
  const int m0 = (t % MT) * TM, n0 = (t / MT) * TN;
  const int kh = g.K / 2, nk = kh / BK;
  const u16* A = static_cast<const u16*>(g.A) + (long long)half * kh;
  const u16* B = static_cast<const u16*>(g.B) + (long long)half * kh * (KN ? g.ldb : 1);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  EpiPre<EPI, 128, TN, 64, 512> pre;  // the epilogue's bias, in flight during the K loop (the mask:
  pre.load_bias(g, n0 + wc * 64, l);   // per row half, when that half's epilogue starts)

  Stager<NW, false, true> sa0(A, g.lda, m0, w, l);
  Stager<NW, false, true> sa1(A, g.lda, m0 + 128, w, l);
  Stager<NW, KN, true> sb(B, g.ldb, n0, w, l);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_byte_addr(lds));
  auto issue = [&](int b) {
    const unsigned base = lds0 + (unsigned)(b * STAGE * 2);
    sa0.issue_at(base);
    sa1.issue_at(base + 128 * BK * 2);
    sb.issue_at(base + A_ELEMS * 2);
  };
  auto compute = [&](int buf) {
    const u16* As = lds + buf * STAGE;
    const u16* Bs = As + A_ELEMS;
    bf16x8 af[BK / 32][4], bfr[BK / 32][NJ];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (KN) bfr[kk][j] = read_frag_kn_fr(Bs, kk * 32, wc * 64 + j * 16, l);
        else bfr[kk][j] = read_frag<BK>(Bs, wc * 64 + j * 16 + (l & 15), chunk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = read_frag<BK>(As, wr * 64 + i * 16 + (l & 15), chunk);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    if constexpr (KN) {
      __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ - 2, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) __builtin_amdgcn_sched_group_barrier(0x100, 4 + NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ, 0);
    }
  };
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p);
  int buf = 0, nb = S - 1;
  for (int kt = 0; kt < nk; ++kt) {
    // tiles kt and (if any) kt + 1 are in flight: retire tile kt
    if (kt + 1 < nk) wait_vmcnt<PER_TILE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // tile kt visible to every wave; the stage of tile kt - 1 is free
    __builtin_amdgcn_sched_barrier(0);
    if (kt + S - 1 < nk) issue(nb);
    nb = (nb + 1 == S) ? 0 : nb + 1;
    compute(buf);
    buf = (buf + 1 == S) ? 0 : buf + 1;
  }
  __builtin_amdgcn_s_barrier();  // every wave is done with the operand stages
  const int own_half = w >> 2;     // waves 4r .. 4r + 3 hold rows [128 r, 128 r + 128) of the tile
  if (g.sk_xs & 6) {  // diag (DGT_GEMM_SK_XS bits, timing only, WRONG results): 2 = the K loop alone,
    if (g.sk_xs & 2) return;  // 4 = each block runs the epilogue of one row half on its own partial
    pre.load_mask(g, m0 + 128 * half, n0, tid);
    epilogue_staged<EPI, 128, TN, 64, 64, 512, true>(g, acc, lds, m0 + 128 * half, n0, wr - 2 * half, wc, l, tid,
                                                     pre, own_half == half);
    return;
  }

  // ---- the halves meet.  Roles are static: the block of K half h FINISHES row half h (adds the
  // partner's partial, runs its epilogue) and PUBLISHES its partial of row half 1 - h.  Publishing
  // never waits; finishing waits for the partner's publish only up to a time limit, after which the
  // finisher hands its own partial over and leaves the row half to the publisher (a per-row-half
  // state word, compare-and-swap: 0 -> kPub by the publisher, 0 -> kGaveUp by a finisher that timed
  // out; exactly one of the two succeeds).  So no block waits on a partner that is not running,
  // and arriving together each block finishes half the tile.
  // (v2, tickets per row half taken in order: the ticket round trips sat on the critical path,
  // 42.4 vs 35.7 us without the meeting; v2b, both tickets at once: the first arriver won both.)
  constexpr int kPub = 1, kGaveUp = 2;
  int* words = reinterpret_cast<int*>(lds + 64 * 1024);  // LDS broadcast words, past the epilogue tile
  const int pr = half ^ 1;                                 // the row half this block publishes
  int* st_pub = g.sk_flags + 4 * t + pr;
  int* st_fin = g.sk_flags + 4 * t + half;
  // 4 partials of 64 KiB per tile: [row half][0 = the publisher's, 1 = a finisher's that gave up]
  auto slab_of = [&](int r, int which) {
    return __builtin_amdgcn_make_buffer_rsrc(g.sk_slab + (long long)(4 * t + 2 * r + which) * (128 * TN), 0,
                                             128 * TN * 4, 0x00020000);
  };
  auto store_rows = [&](int r, int which) {  // the owning waves' accumulators of row half r, sc1
    if (own_half == r) {
      const auto rsrc = slab_of(r, which);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsrc,
                                                 ((i * NJ + j) * 256 + (tid & 255)) * 16, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
  };
  auto finish_rows = [&](int r, int which) {  // add the other block's partial of row half r, epilogue
    // every load of a partial is an sc1 load (L1 bypassed) behind the state word's sc1 poll or
    // compare-and-swap and a barrier: no acquire fence (MI355X_MICROARCH.md, visibility: valid forms)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (own_half == r) {
      const auto rsrc = slab_of(r, which);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] += __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((i * NJ + j) * 256 + (tid & 255)) * 16, 0, 16));
    }
    pre.load_mask(g, m0 + 128 * r, n0, tid);
    epilogue_staged<EPI, 128, TN, 64, 64, 512, true>(g, acc, lds, m0 + 128 * r, n0, wr - 2 * r, wc, l, tid, pre,
                                                     own_half == r);
  };
  // 1. publish row half pr (the compare-and-swap's answer is only needed at step 3)
  store_rows(pr, 0);
  int pub_old = 0;
  if (tid == 0) pub_old = cas_agent(st_pub, 0, kPub);
  // 2. finish row half `half`: wait for the partner's publish, at most ~20 us (sk_xs bit 3, a test
  // knob: not at all, so the hand-over paths run)
  if (tid == 0) {
    const unsigned long long t0 = wall_clock64(), limit = (g.sk_xs & 8) ? 0 : 2000;  // 100 MHz: 20 us
    int st;
    while ((st = __hip_atomic_load(st_fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 &&
           wall_clock64() - t0 < limit)
      __builtin_amdgcn_s_sleep(1);
    words[0] = st;
  }
  __syncthreads();
  int fin = words[0];
  if (fin != kPub) {
    // the partner has not published: hand this block's partial over and give the row half up,
    // unless the partner's publish lands first
    store_rows(half, 1);
    if (tid == 0) words[1] = cas_agent(st_fin, 0, kGaveUp);
    __syncthreads();
    fin = words[1] == kPub ? kPub : kGaveUp;
  }
  if (fin == kPub) {
    if (tid == 0) __hip_atomic_store(st_fin, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    finish_rows(half, 0);
  }
  // 3. the finisher of row half pr gave up: finish it here from its handed-over partial
  if (tid == 0) words[2] = pub_old;
  __syncthreads();
  if (words[2] == kGaveUp) {
    if (tid == 0) __hip_atomic_store(st_pub, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    finish_rows(pr, 1);
  }
}

bool gemm_nt_sk_fits(const GemmArgs& g, int epi) {
  if (epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam)) return false;
  if (g.M <= 0 || g.N <= 0 || g.M % sk::TM || g.N % sk::TN || g.K % (2 * GBK)) return false;
  return ((g.M / sk::TM) * (g.N / sk::TN)) % 8 == 0;
}

// ------------------------------------------------------------------ 128 x 128, register prefetch (RP)
// Variant 6 (NT operands): the K-tiles in flight live in VGPRs instead of LDS.  Each thread loads its
// four 16-byte pieces of a K-tile (A rows tid/8 and tid/8 + 64, B likewise, chunk tid % 8) with
// plain global loads D K-tiles ahead, and writes them into one of two LDS stages (ds_write_b128, the
// same XOR-swizzled image the LDS-DMA produces) just before the tile is consumed: LDS holds 64 KiB,
// the registers another D x 32 KiB per block, so D + 1 K-tiles are in flight against the 4-stage
// kernel's two -- the per-CU operand stream of the one-wave M = 1024 grids is latency x bytes in
// flight bound (profiles/r3_gemm_pmc.txt: MFMA ~40 % busy in ours and hipBLASLt's alike).  The
// fragment reads and MFMA order are the FR kernel's (variant 3): results are bit-identical to it.
// One barrier per K-tile: the write of tile kt + 1 goes into the stage tile kt - 1 was read from,
// which every wave finished before the previous barrier.
// A [K, N] B operand (the dgrad's W, kEpiBKN) is loaded as it lies -- thread tid fetches chunk tid % 16
// of k-rows tid / 16 and tid / 16 + 32 -- into stage_tile_kn's image, and read with the FR kernel's
// transposed ds_read_b64_tr_b16 fragments.
template <int EPI, int D>
__global__ __launch_bounds__(512, 1) void gemm_nt_rp_kernel(GemmArgs g) {
  constexpr int BK = GBK, NW = 8, WN = 32, WCOLS = GBN / WN, NJ = WN / 16;
  constexpr bool KN = (EPI & kEpiBKN) != 0;
  static_assert(!(EPI & kEpiAdam), "RP: no in-epilogue Adam");
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][GBM * BK];  // [stage][A|B], 32 KiB per stage
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int tm, tn;
  tile_of_block(blockIdx.x, g.M / GBM, g.N / GBN, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int wr = w / WCOLS, wc = w % WCOLS;
  const int prow = tid >> 3, pch = tid & 7;
  const u16* ga[2];
  const u16* gb[2];
  int loff[2], lboff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = prow + 64 * i;
    ga[i] = static_cast<const u16*>(g.A) + (long long)(m0 + row) * g.lda + pch * 8;
    loff[i] = row * BK + ((pch ^ (row & 7)) << 3);  // read_frag<BK>'s image
    if constexpr (KN) {
      const int kr = (tid >> 4) + 32 * i, c = tid & 15;  // k-row, 16-byte chunk of the 128 n
      gb[i] = static_cast<const u16*>(g.B) + (long long)kr * g.ldb + n0 + c * 8;
      lboff[i] = kr * GBN + ((c ^ kn_swz(kr)) << 3);  // stage_tile_kn's image
    } else {
      gb[i] = static_cast<const u16*>(g.B) + (long long)(n0 + row) * g.ldb + pch * 8;
      lboff[i] = loff[i];
    }
  }
  const long long bstep = KN ? (long long)BK * g.ldb : BK;  // elements per K-tile of B
  u32x4 rg[D][4];
  auto gload = [&](int kt, u32x4 (&r)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      r[i] = *reinterpret_cast<const u32x4*>(ga[i] + (long long)kt * BK);
      r[2 + i] = *reinterpret_cast<const u32x4*>(gb[i] + kt * bstep);
    }
  };
  auto lwrite = [&](int st, const u32x4 (&r)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u32x4*>(&lds[st][0][loff[i]]) = r[i];
      *reinterpret_cast<u32x4*>(&lds[st][1][lboff[i]]) = r[2 + i];
    }
  };
  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {  // the FR kernel's K-tile (gemm_nt_kernel, FR != 0)
    const u16* As = lds[buf][0];
    const u16* Bs = lds[buf][1];
    bf16x8 af[BK / 32][4], bfr[BK / 32][NJ];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (KN) bfr[kk][j] = read_frag_kn_fr(Bs, kk * 32, wc * WN + j * 16, l);
        else bfr[kk][j] = read_frag<BK>(Bs, wc * WN + j * 16 + (l & 15), chunk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = read_frag<BK>(As, wr * 64 + i * 16 + (l & 15), chunk);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    if constexpr (KN) {  // as the FR kernel: the second half's reads go out after the first MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4 + 2 * NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ - 2, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) __builtin_amdgcn_sched_group_barrier(0x100, 4 + NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, (BK / 32) * 4 * NJ, 0);
    }
  };

  // nk % D == 0 (the dispatcher's condition).  Every iteration issues exactly four loads and four
  // LDS writes, past the end on clamped tile indices (re-reads of the last tile, never consumed):
  // with a conditional load the compiler's vmcnt accounting takes the shorter path's count at the
  // loop header and waits for every load in flight, leaving one K-tile of prefetch instead of D.
  const int nk = g.K / BK;
#pragma unroll
  for (int d = 0; d < D; ++d) gload(min(d, nk - 1), rg[d]);
  lwrite(0, rg[0]);
  gload(min(D, nk - 1), rg[0]);
  __syncthreads();
  // iteration kt: tile kt + 1 (in rg[(kt + 1) % D]) -> LDS stage (kt + 1) & 1, its registers refilled
  // with tile kt + 1 + D, then tile kt's MFMAs; unrolled by D so every register index is static
  for (int kt0 = 0; kt0 < nk; kt0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int kt = kt0 + d;
      const int nx = (d + 1) % D;  // static after the unroll
      lwrite((kt + 1) & 1, rg[nx]);
      gload(min(kt + 1 + D, nk - 1), rg[nx]);
      compute(kt & 1);
      __syncthreads();
    }
  }

  if constexpr (!(EPI & kEpiOutF32)) {
    epilogue_staged<EPI, GBM, GBN, 64, WN, 64 * NW>(g, acc, &lds[0][0][0], m0, n0, wr, wc, l, tid,
                                                    EpiPre<EPI, GBM, GBN, WN, 64 * NW>{});
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + wr * 64 + i * 16 + 4 * (l >> 4), n0 + wc * WN + j * 16 + (l & 15));
  }
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
// phase issues ONE unit of staging (2 LDS-DMAs per thread), its LDS reads, then `s_waitcnt
// vmcnt(8)` (every unit but the 4 newest has landed), ONE barrier, MFMAs.  The unit order below
// restages a unit at least two phases after its last read (WAR, so no second barrier) and reads it
// at least one phase after the wait that retires it (RAW), so loads stay in flight across 4 phases
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

// One unit's two LDS-DMAs per thread, issued from asm in the saddr form: the unit's base in SGPRs,
// the lane's 32-bit byte offset in a VGPR, so the register-full loop (128 accumulator VGPRs + 64 of
// fragments) holds no 64-bit address temporaries.  Through the compiler builtin every 256x256
// kernel spilled 1-3 VGPRs to scratch; from asm none does, 4-6 % faster at every size
// (profiles/r3_gemm256_asm_ab.jsonl).  With every DMA of the loop in asm, the compiler tracks none
// of them; the phase's explicit vmcnt waits and barriers order them (as in the 128x128 FR kernel).
// unit_la: the unit's LDS byte address, wave-uniform (kept in SGPRs: a generic LDS pointer per unit
// costs two VGPRs each, and the cross-phase variant below has none to spare)
DGT_DEVICE void stage(const u16* ubase, const int (&off)[2], unsigned unit_la, int w) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(ubase);
  // (readfirstlane returns int: each half goes through unsigned, or the low half would be
  // sign-extended into the high one)
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b), hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const unsigned long long sb = ((unsigned long long)hi << 32) | lo;
  const unsigned l0 = __builtin_amdgcn_readfirstlane(unit_la + (unsigned)(w * 2 * 8 * BK * 2));
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    unsigned saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"((unsigned)off[i] * 2u), "s"(sb), "s"(l0 + (unsigned)(i * 8 * BK * 2))
        : "memory");
  }
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
  unsigned lds0;     // lds's LDS byte address (wave-uniform)
};

template <int U>
DGT_DEVICE void stage_unit(const Ctx& c, int kt, int buf) {
  const bool is_a = (U == kALo || U == kAHi);
  const u16* ubase = is_a ? c.A + (U == kAHi ? 64 * c.lda : 0) + kt * BK
                          : c.B + (U == kBHi ? 32 * c.ldb : 0) + kt * BK;
  stage(ubase, is_a ? c.offa : c.offb, c.lds0 + (unsigned)((buf * 4 + U) * UNIT * 2), c.w);
}

// unit staged in phase P (1..8) of an iteration: ph1, ph2 -> the odd tile's B_hi, A_hi; ph3..6 ->
// the next even tile's A_lo, B_lo, B_hi, A_hi; ph7, ph8 -> the next odd tile's A_lo, B_lo.  Every
// unit is restaged at least TWO phases after its last read and read at least five phases after it
// is staged (four units in flight: vmcnt(8)).  A wave staging in phase S has passed barrier S-1,
// which every wave reaches only after its reads of phase S-2 have landed (lgkmcnt(0) before its
// MFMAs), so no WAR barrier after the MFMAs is needed: ONE barrier per 16 MFMAs.  (Round 2's order
// -- one phase between a unit's last read and its restaging, five units in flight -- needed a
// second barrier per phase and was 10-13 % slower at every size: profiles/r3_gemm256_asm_ab.jsonl.)
template <int P>
DGT_DEVICE void stage_phase(const Ctx& c, int it) {
  constexpr int unit = P == 1 ? kBHi : P == 2 ? kAHi : P == 3 ? kALo : P == 4 ? kBLo : P == 5 ? kBHi
                     : P == 6 ? kAHi : P == 7 ? kALo : kBLo;
  constexpr int buf = (P <= 2 || P >= 7) ? 1 : 0;
  const int kt = P <= 2 ? 2 * it + 1 : (P <= 6 ? 2 * it + 2 : 2 * it + 3);
  stage_unit<unit>(c, kt, buf);
}

template <int P, bool LAST>
DGT_DEVICE void phase(const Ctx& c, int it, Frags& f, f32x4 (&acc)[8][4]) {
  constexpr int buf = P <= 4 ? 0 : 1;
  constexpr int q = (P - 1) & 3;
  const u16* base = c.lds + buf * 4 * UNIT;
  const int lr = c.l & 15, lc = c.l >> 4;
  // the last iteration stages only its own odd tile's remaining two units
  if (!LAST || P <= 2) stage_phase<P>(c, it);
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
  // after phase 2, so its counts shrink as the pipeline drains
  if (!LAST) wait_vm<8>();
  else wait_vm<P <= 3 ? 8 : P == 4 ? 4 : P == 5 ? 2 : 0>();
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

// ---- cross-phase fragment prefetch (variant 8).  Above, every phase reads its fragments and then
// waits for them before its MFMAs; the barrier lines all 8 waves up, so the CU's LDS reads (up to 96
// KiB in q0) and its MFMAs take turns instead of overlapping.  Here phase P issues the reads of phase
// P + 1 right after its barrier, interleaved with its own 16 MFMAs, and waits for them (lgkmcnt(0))
// only before the next barrier.  The staging order and vmcnt waits are unchanged: the unit phase P+1
// reads is exactly the one phase P's wait retires, and a read issued after barrier P has completed
// before barrier P+1, so a unit may be restaged from phase P+2 on (every restage above is >= 2 phases
// after the old last read, so >= 3 after the new one).  Each operand half keeps one register set:
// q0 reads B_hi (free since the last tile's q2), q1 A_hi (free since q3), q2 the next tile's A_lo
// (free since q1); B_lo is still being multiplied in q3 when the next tile's is read, so q3 issues
// its kk = 0 MFMAs, then the reads that overwrite B_lo's kk = 0 fragments, then the kk = 1 MFMAs and
// the remaining reads.  Same MFMAs in the same order per accumulator: bit-identical to phase<>.
struct FragsX {
  bf16x8 alo[4][2], ahi[4][2];
  bf16x8 blo[2][2], bhi[2][2];
};

template <int U>
DGT_DEVICE void read_a(const Ctx& c, int buf, bf16x8 (&dst)[4][2]) {  // A unit: the wave's 64 rows
  const u16* ul = c.lds + (buf * 4 + U) * UNIT;
  const int lr = c.l & 15, lc = c.l >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) dst[i][kk] = frag(ul, c.wr * 64 + i * 16 + lr, kk * 4 + lc);
}
template <int U>
DGT_DEVICE void read_b(const Ctx& c, int buf, int kk, bf16x8 (&dst)[2][2]) {  // B unit: 32 cols, one kk
  const u16* ul = c.lds + (buf * 4 + U) * UNIT;
  const int lr = c.l & 15, lc = c.l >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) dst[j][kk] = frag(ul, c.wc * 32 + j * 16 + lr, kk * 4 + lc);
}

template <int Q>
DGT_DEVICE void mfma_half(FragsX& f, f32x4 (&acc)[8][4], int kk) {  // quadrant Q's 8 MFMAs of one kk
  constexpr int i0 = (Q == 0 || Q == 1) ? 0 : 4;
  constexpr bool hi_b = (Q == 1 || Q == 2);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[i0 + i][(hi_b ? 2 : 0) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
          i0 == 0 ? f.alo[i][kk] : f.ahi[i][kk], hi_b ? f.bhi[j][kk] : f.blo[j][kk],
          acc[i0 + i][(hi_b ? 2 : 0) + j], 0, 0, 0);
}

template <int P, bool LAST>
DGT_DEVICE void phase_x(const Ctx& c, int it, FragsX& f, f32x4 (&acc)[8][4]) {
  constexpr int q = (P - 1) & 3;
  constexpr int buf = P <= 4 ? 0 : 1;
  if (!LAST || P <= 2) stage_phase<P>(c, it);
  if (!LAST) wait_vm<8>();
  else wait_vm<P <= 3 ? 8 : P == 4 ? 4 : P == 5 ? 2 : 0>();
  wait_lgkm0();  // this phase's fragments (read during the previous phase) have landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  constexpr bool reads = !(LAST && P >= 7);  // the last tile's q2 / q3 have no next tile to read
  __builtin_amdgcn_s_setprio(1);
  if constexpr (q == 3) {
    mfma_half<3>(f, acc, 0);
    if constexpr (reads) read_b<kBLo>(c, buf ^ 1, 0, f.blo);
    mfma_half<3>(f, acc, 1);
    if constexpr (reads) {
      read_b<kBLo>(c, buf ^ 1, 1, f.blo);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
  } else {
    // q0: B_hi (4 reads), q1: A_hi (8), q2: the next tile's A_lo (8)
    constexpr int nreads = q == 0 ? 4 : 8;
    if constexpr (reads) {
      if constexpr (q == 0) {
        read_b<kBHi>(c, buf, 0, f.bhi);
        read_b<kBHi>(c, buf, 1, f.bhi);
      } else if constexpr (q == 1) {
        read_a<kAHi>(c, buf, f.ahi);
      } else {
        read_a<kALo>(c, buf ^ 1, f.alo);
      }
    }
    mfma_half<q>(f, acc, 0);
    mfma_half<q>(f, acc, 1);
    if constexpr (reads) {
#pragma unroll
      for (int r = 0; r < nreads; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16 - nreads, 0);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

template <bool LAST>
DGT_DEVICE void iteration_x(const Ctx& c, int it, FragsX& f, f32x4 (&acc)[8][4]) {
  phase_x<1, LAST>(c, it, f, acc);
  phase_x<2, LAST>(c, it, f, acc);
  phase_x<3, LAST>(c, it, f, acc);
  phase_x<4, LAST>(c, it, f, acc);
  phase_x<5, LAST>(c, it, f, acc);
  phase_x<6, LAST>(c, it, f, acc);
  phase_x<7, LAST>(c, it, f, acc);
  phase_x<8, LAST>(c, it, f, acc);
}
}  // namespace g256

// SPK (split-K 2, grids of 100-128 tiles, e.g. M = 1024 x N = 8192): two blocks per tile, each over
// half of K -- half the operand bytes per CU of the 128 x 128 kernel's two waves of blocks.  Each
// writes its fp32 partial (256 KiB, write-through sc1), drains and adds to the tile's counter; the
// second to add sums the other's partial into its accumulators (fp32 a + b == b + a: the bits do not
// depend on the order), re-arms the counter and runs the epilogue.
template <int EPI, bool XP = false, bool SPK = false>
__global__ __launch_bounds__(512) void gemm_nt_256_kernel(GemmArgs g) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) u16 lds[2 * 4 * UNIT];
  const int tid = threadIdx.x;
  const int tile = SPK ? (int)blockIdx.x >> 1 : (int)blockIdx.x, slice = SPK ? (int)blockIdx.x & 1 : 0;
  int tm, tn;
  tile_of_block(tile, g.M / BM, g.N / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kslice = SPK ? g.K / 2 : g.K;
  Ctx c;
  c.A = static_cast<const u16*>(g.A) + (long long)m0 * g.lda + (long long)slice * kslice;
  c.B = static_cast<const u16*>(g.B) + (long long)n0 * g.ldb + (long long)slice * kslice;
  c.lda = g.lda;
  c.ldb = g.ldb;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.l = tid & 63;
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    c.offa[i] = lane_off(true, g.lda, c.w, i, c.l);
    c.offb[i] = lane_off(false, g.ldb, c.w, i, c.l);
  }
  c.lds = lds;
  c.lds0 = __builtin_amdgcn_readfirstlane(lds_byte_addr(lds));

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
  wait_vm<8>();
  __builtin_amdgcn_s_barrier();

  const int nit = kslice / (2 * BK);
  if constexpr (XP) {
    // phase 1's fragments (tile 0's A_lo and B_lo, retired by the wait above)
    FragsX fx;
    read_a<kALo>(c, 0, fx.alo);
    read_b<kBLo>(c, 0, 0, fx.blo);
    read_b<kBLo>(c, 0, 1, fx.blo);
    for (int it = 0; it + 1 < nit; ++it) iteration_x<false>(c, it, fx, acc);
    iteration_x<true>(c, nit - 1, fx, acc);
  } else {
    for (int it = 0; it + 1 < nit; ++it) iteration<false>(c, it, f, acc);
    iteration<true>(c, nit - 1, f, acc);
  }

  if constexpr (SPK) {
    auto part = [&](int q) {
      return __builtin_amdgcn_make_buffer_rsrc(g.sk_slab + ((long long)tile * 2 + q) * (BM * BN), 0, BM * BN * 4,
                                               0x00020000);
    };
    const auto mine = part(slice);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), mine,
                                               ((i * 4 + j) * 512 + tid) * 16, 0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();                                  // (and every wave is past its last LDS read)
    int* word = reinterpret_cast<int*>(lds);
    if (tid == 0) *word = __hip_atomic_fetch_add(g.sk_flags + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*word == 0) return;  // the other half finishes the tile
    if (tid == 0) __hip_atomic_store(g.sk_flags + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // sc1 loads behind the counter's add + barrier
    const auto other = part(slice ^ 1);
    // one accumulator row at a time: the accumulators hold 128 VGPRs, so all 32 loads in flight at
    // once would spill
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f32x4 p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        p[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(other, ((i * 4 + j) * 512 + tid) * 16, 0, 16));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += p[j];
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  if constexpr ((EPI & kEpiAdam) != 0) {
    // fp32 256 x 256 tile = 256 KiB: two passes of 128 rows through the 128 KiB of operand LDS
    epilogue_adam<BM, BN, 128, 64, 512, 128>(g, acc, reinterpret_cast<float*>(lds), m0, n0, c.wr, c.wc, c.l, tid);
  } else if constexpr (!(EPI & kEpiOutF32)) {
    // (bias and mask loaded together ahead of the epilogue (EpiPre, PRE = true): 1.5-2 % on the
    // large transposed dgrads, with 4-13 more spilled VGPRs -- not kept)
    epilogue_staged<EPI, BM, BN, 128, 64, 512>(g, acc, lds, m0, n0, c.wr, c.wc, c.l, tid, EpiPre<EPI, BM, BN, 64, 512>{});
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        epi_store<EPI>(g, acc[i][j], m0 + c.wr * 128 + i * 16 + 4 * (c.l >> 4), n0 + c.wc * 64 + j * 16 + (c.l & 15));
  }
}

// variant: 0 = pick by shape (256x256 for >= 200 tiles, else for one-wave grids the 128x128 variant
// 5 for a [K, N] B operand with K % 128 == 0 and variant 3 otherwise, else variant 1), 1 = 128x128
// 2-stage (4 waves, 2 blocks / CU), 2 = 256x256 8-phase (the bitwise oracle of 8), 3 = variant 4 with
// front-loaded fragment reads (FR), 4 = 128x128 4-stage with 8 waves (1 block / CU; the FR kernels'
// bitwise oracle), 5 = software-pipelined fragment reads (SP, five stages; K % 128 == 0, else 3),
// 6 / 7 = register prefetch, 8 = 256x256 with cross-phase fragment prefetch (the shape rule's
// 256x256 kernel).  The round-2 variants measured slower or no better inside the MLP step live in
// git history (commit c0371a5).
// the RP kernel for the forward-type epilogues (others: false, the dispatcher reports it)
template <int E>
bool launch_rp(int grid, const GemmArgs& g, hipStream_t stream, int depth) {
  if constexpr (!(E & kEpiAdam)) {
    // depth 4 for the forward-type epilogues only (the others: 2)
    if constexpr ((E & ~(kEpiBias | kEpiRelu | kEpiStoreT | kEpiOutF32)) == 0) {
      if (depth == 4) {
        hipLaunchKernelGGL((gemm_nt_rp_kernel<E, 4>), dim3(grid), dim3(512), 0, stream, g);
        return true;
      }
    }
    hipLaunchKernelGGL((gemm_nt_rp_kernel<E, 2>), dim3(grid), dim3(512), 0, stream, g);
    return true;
  } else {
    return false;
  }
}

// the shape rule's use of the split-K kernel: DGT_GEMM_SK=1 for one-wave 128 x 128 grids with
// K >= 2048 and a [N, K] B (the MLP's M = 1024 forwards); the default (0) keeps the 128 x 128
// kernels: hot the split-K forward is level with them (45.3-45.7 vs 45.4-46.9 us with C^T), in the
// bf16 MLP step it times the same (41.5 vs 41.5 us) (profiles/r6_gemm_m1024_splitk.jsonl: its K loop
// alone takes 32-33 us, a 128-row half epilogue ~4 us, the halves' meeting ~5 us)
static bool sk_auto() {
  static const int on = [] {
    const char* e = std::getenv("DGT_GEMM_SK");
    return (e && *e) ? std::atoi(e) : 0;
  }();
  return on != 0;
}

bool gemm_nt_uses_sk(const GemmArgs& g, int epi, int variant) {
  if (variant == 9) return true;
  // (the [K, N] dgrad stays on the software-pipelined 128 x 128 kernel: 41.9 vs 46.5-47.8 us)
  if (variant != 0 || !sk_auto() || (epi & kEpiBKN) || !gemm_nt_sk_fits(g, epi)) return false;
  return (g.M / GBM) * (g.N / GBN) <= 256 && g.K >= 2048;
}

// The split of the 128 x 128 split-K mode (variant 10) for a grid that leaves CUs idle: the largest
// of 8 / 4 / 2 with tiles x split <= 256 blocks and at least 8 K-tiles per slice (0: none fits).
// DGT_GEMM_SKN (default 1) lets the shape rule use it for grids of at most 128 tiles.
int gemm_nt_skn_split(const GemmArgs& g, int epi) {
  if (epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam)) return 0;
  const int tiles = (g.M / GBM) * (g.N / GBN), nk = g.K / GBK;
  for (int sp = 8; sp >= 2; sp /= 2)
    if (tiles * sp <= 256 && nk % sp == 0 && nk / sp >= 8) return sp;
  return 0;
}

static bool skn_auto() {
  static const int on = [] {
    const char* e = std::getenv("DGT_GEMM_SKN");
    return (e && *e) ? std::atoi(e) : 1;
  }();
  return on != 0;
}

// The 256 x 256 kernel's split-K 2 mode (variant 11; the shape rule's choice, DGT_GEMM_SKN=1, for
// 100-128 tiles of 256 x 256 with an [N, K] B, a staged bf16 epilogue and K / 2 a multiple of 128, at
// least 1024): M = 1024 x N = 8192 or M = 2048 x N = 4096.
int gemm_nt_uses_spk256(const GemmArgs& g, int epi, int variant) {
  if (variant != 11 && (variant != 0 || !skn_auto())) return 0;
  if (epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam | kEpiBKN | kEpiColSum)) return 0;
  if (g.M % 256 || g.N % 256 || g.K % 256 || g.lda > (1 << 22) || g.ldb > (1 << 22)) return 0;
  const int tiles = (g.M / 256) * (g.N / 256);
  if (variant == 11) return tiles * 2 <= 1024 ? 1 : 0;
  return (tiles >= 100 && tiles <= 128 && g.K / 2 >= 1024) ? 1 : 0;
}

// A [K, N] B operand on a grid of at least 200 tiles of 256 x 256 (batch 4096 on 4096-wide layers,
// 2048 on 8192-wide ones) is transposed once (transpose_bf16, into the caller's workspace) and the product
// runs as NT on the 256 x 256 kernels: 4096^3 dgrad 167-172 -> ~110 us (hipBLASLt 107), 2048 x 8192
// 279-283 -> ~235.  DGT_GEMM_KN_T=0 keeps the 128 x 128 [K, N] kernels.  (variant 0, B contiguous.)
bool gemm_nt_kn_transposes(const GemmArgs& g, int epi, int variant) {
  static const int on = [] {
    const char* e = std::getenv("DGT_GEMM_KN_T");
    return (e && *e) ? std::atoi(e) : 1;
  }();
  if (!on || variant != 0 || !(epi & kEpiBKN) || (epi & (kEpiOutF32 | kEpiAccumulate | kEpiAdam))) return false;
  if (g.M % 256 || g.N % 256 || g.K % 256 || g.ldb != g.N || g.K > (1 << 22)) return false;
  // the NT product must land on the 256 x 256 kernel's full grid (>= 200 tiles); at 100-128 tiles
  // (2048 x 4096) transpose + split-K 2 measured level with the [K, N] 128 x 128 kernel
  return (g.M / 256) * (g.N / 256) >= 200;
}

int gemm_nt_uses_skn(const GemmArgs& g, int epi, int variant) {
  if (variant == 10) return gemm_nt_skn_split(g, epi);
  if (variant != 0 || !skn_auto() || (g.M / GBM) * (g.N / GBN) > 128) return 0;
  return gemm_nt_skn_split(g, epi);
}

hipError_t gemm_nt(const GemmArgs& g, int epi, hipStream_t stream, int variant) {
  if (g.M % GBM || g.N % GBN || g.K % GBK || g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  if (variant < 0 || variant > 11) return hipErrorInvalidValue;
  if (gemm_nt_uses_spk256(g, epi, variant)) {
    if (!g.sk_slab || !g.sk_flags) return hipErrorInvalidValue;
    const int grid = (g.M / 256) * (g.N / 256) * 2;
    switch (epi) {
#define DGT_SPK256_CASE(E)                                                                             \
  case E:                                                                                              \
    hipLaunchKernelGGL((gemm_nt_256_kernel<E, true, true>), dim3(grid), dim3(512), 0, stream, g);      \
    return hipGetLastError();
      DGT_SPK256_CASE(0)
      DGT_SPK256_CASE(kEpiBias | kEpiRelu | kEpiStoreT)
      DGT_SPK256_CASE(kEpiBias | kEpiRelu)
      DGT_SPK256_CASE(kEpiBias | kEpiStoreT)
      DGT_SPK256_CASE(kEpiBias)
      DGT_SPK256_CASE(kEpiMask | kEpiStoreT)
#undef DGT_SPK256_CASE
      default:
        return hipErrorInvalidValue;
    }
  }
  if (variant == 11) return hipErrorInvalidValue;
  if (variant == 10 || (variant == 0 && gemm_nt_uses_skn(g, epi, 0))) {
    const int split = gemm_nt_skn_split(g, epi);
    if (!split || g.skn_split != split || !g.sk_slab || !g.sk_flags) return hipErrorInvalidValue;
    const int grid = (g.M / GBM) * (g.N / GBN) * split;
    switch (epi) {
#define DGT_SKN_CASE(E)                                                                         \
  case E:                                                                                       \
    hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8, 1, true>), dim3(grid), dim3(512), 0, stream, g); \
    return hipGetLastError();
      DGT_SKN_CASE(0)
      DGT_SKN_CASE(kEpiBias | kEpiRelu | kEpiStoreT)
      DGT_SKN_CASE(kEpiBias | kEpiRelu)
      DGT_SKN_CASE(kEpiBias | kEpiStoreT)
      DGT_SKN_CASE(kEpiBias)
      DGT_SKN_CASE(kEpiMask | kEpiStoreT)
      DGT_SKN_CASE(kEpiMask | kEpiStoreT | kEpiBKN)
      DGT_SKN_CASE(kEpiMask | kEpiStoreT | kEpiBKN | kEpiColSum)
      DGT_SKN_CASE(kEpiBKN)
      DGT_SKN_CASE(kEpiStoreT | kEpiBKN)
#undef DGT_SKN_CASE
      default:
        return hipErrorInvalidValue;
    }
  }
  if (gemm_nt_uses_sk(g, epi, variant)) {
    if (!gemm_nt_sk_fits(g, epi) || !g.sk_slab || !g.sk_flags) return hipErrorInvalidValue;
    const int grid = 2 * (g.M / sk::TM) * (g.N / sk::TN);
    switch (epi) {
#define DGT_SK_CASE(E)                                                                          \
  case E:                                                                                       \
    hipLaunchKernelGGL((gemm_nt_sk_kernel<E>), dim3(grid), dim3(512), 0, stream, g);            \
    return hipGetLastError();
      DGT_SK_CASE(0)
      DGT_SK_CASE(kEpiBias | kEpiRelu | kEpiStoreT)
      DGT_SK_CASE(kEpiBias | kEpiRelu)
      DGT_SK_CASE(kEpiBias | kEpiStoreT)
      DGT_SK_CASE(kEpiBias)
      DGT_SK_CASE(kEpiMask | kEpiStoreT)
      DGT_SK_CASE(kEpiMask | kEpiStoreT | kEpiBKN)
      DGT_SK_CASE(kEpiMask | kEpiStoreT | kEpiBKN | kEpiColSum)
      DGT_SK_CASE(kEpiBKN)
      DGT_SK_CASE(kEpiStoreT | kEpiBKN)
#undef DGT_SK_CASE
      default:
        return hipErrorInvalidValue;
    }
  }
  // the 256x256 kernel runs the cross-phase fragment prefetch (g256::phase_x) unless variant 2 asks
  // for the 8-phase pipeline it is bitwise-checked against: 8192^3 1.51-1.52 vs 1.39-1.47 PF, the
  // MLP's wgrad 31.6-31.9 vs 33.0-33.7 us (profiles/r4_gemm256_xp.jsonl)
  const bool xp = variant != 2;
  if (variant == 8) variant = 2;
  // only the 128x128 kernels read a [K, N] B operand (column sums: both tile sizes)
  const bool kn = (epi & kEpiBKN) != 0;
  if ((epi & kEpiColSum) && (!(epi & kEpiStoreT) || !g.colsum)) return hipErrorInvalidValue;
  // variants 6 / 7: the register-prefetch 128x128 kernel (2 / 4 K-tiles in VGPRs) for NT products
  // with forward-type epilogues and K a multiple of 2 / 4 K-tiles; any other product asked for it
  // (a DGT_GEMM_VARIANT A/B run reaches the dgrads too) keeps the shape rule
  const bool fwd_type = (epi & ~(kEpiBias | kEpiRelu | kEpiStoreT | kEpiOutF32)) == 0;
  const int rp_depth = (variant == 7 && fwd_type) ? 4 : 2;
  if (variant >= 6 && ((epi & kEpiAdam) || (g.K / GBK) % rp_depth)) variant = 0;
  const bool rp = variant >= 6;
  // (the 256x256 kernel's DMAs carry a 32-bit per-lane byte offset of up to 255 rows: row strides
  // past 4M elements take the 128x128 kernels)
  const bool fits256 = g.M % 256 == 0 && g.N % 256 == 0 && g.K % 128 == 0 && g.lda <= (1 << 22) && g.ldb <= (1 << 22);
  // the big tile needs most of the 256 CUs busy: below ~200 tiles the 128 kernel (4x the blocks)
  // wins
  bool big = fits256 && !kn && (g.M / 256) * (g.N / 256) >= 200;
  if (variant == 1 || variant >= 3) big = false;
  if (variant == 2) {
    if (!fits256 || kn) return hipErrorInvalidValue;
    big = true;
  }
  const int grid = big ? (g.M / 256) * (g.N / 256) : (g.M / GBM) * (g.N / GBN);
  // a grid that fits the chip at one block per CU gains nothing from 2 blocks / CU: spend the LDS on
  // a deep (4-stage) pipeline and 8 waves instead (measured: 8 waves beat 4 on one-wave grids)
  const bool eight = !big && (variant >= 3 || (variant == 0 && grid <= 256));
  // the shape rule's 128x128 choice is the front-loaded-reads form (variant 3): bit-identical to 4,
  // faster hot and cold and inside the MLP step (profiles/r3_gemm_m1024.jsonl)
  // the [K, N] dgrad takes the software-pipelined reads (variant 5: in the MLP step 46.1 vs 48.0 us,
  // hot 41.2 vs 47.1); the NT forward keeps the front-loaded reads (44.5 vs 43.6 us in the step)
  // (profiles/r3_gemm_sp_ab.txt)
  const bool sp = eight && g.K % 128 == 0 && (variant == 5 || (variant == 0 && (epi & kEpiBKN) != 0));
  const bool fr = eight && !sp && (variant == 0 || variant == 3 || variant == 5);
#define DGT_EPI_CASE_KN(E)                                                                        \
  case E:                                                                                         \
    if (rp) {                                                                                     \
      if (!launch_rp<E>(grid, g, stream, rp_depth)) return hipErrorInvalidValue;                  \
    } else if (sp) hipLaunchKernelGGL((gemm_nt_kernel<E, 5, 8, 3>), dim3(grid), dim3(512), 0, stream, g); \
    else if (fr) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8, 1>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
#define DGT_EPI_CASE(E)                                                                           \
  case E:                                                                                         \
    if (rp) {                                                                                     \
      if (!launch_rp<E>(grid, g, stream, rp_depth)) return hipErrorInvalidValue;                  \
    } else if (big && xp) hipLaunchKernelGGL((gemm_nt_256_kernel<E, true>), dim3(grid), dim3(512), 0, stream, g); \
    else if (big) hipLaunchKernelGGL((gemm_nt_256_kernel<E>), dim3(grid), dim3(512), 0, stream, g); \
    else if (sp) hipLaunchKernelGGL((gemm_nt_kernel<E, 5, 8, 3>), dim3(grid), dim3(512), 0, stream, g); \
    else if (fr) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8, 1>), dim3(grid), dim3(512), 0, stream, g); \
    else if (eight) hipLaunchKernelGGL((gemm_nt_kernel<E, 4, 8>), dim3(grid), dim3(512), 0, stream, g); \
    else hipLaunchKernelGGL((gemm_nt_kernel<E, 2>), dim3(grid), dim3(256), 0, stream, g);         \
    break;
  switch (epi) {
    DGT_EPI_CASE(0)                                                // plain bf16 product (wgrad into bf16 grads)
    DGT_EPI_CASE(kEpiAccumulate)                                   // wgrad, bf16 gradient accumulation
    DGT_EPI_CASE(kEpiBias | kEpiRelu | kEpiStoreT)                 // hidden-layer forward
    DGT_EPI_CASE(kEpiBias | kEpiRelu)                              // forward, no transposed copy
    DGT_EPI_CASE(kEpiBias | kEpiStoreT)                            // linear forward (no ReLU)
    DGT_EPI_CASE(kEpiBias)
    DGT_EPI_CASE(kEpiMask | kEpiStoreT)                            // dgrad through ReLU
    DGT_EPI_CASE(kEpiMask | kEpiStoreT | kEpiColSum)               // + bias-gradient partials (W^T given)
    DGT_EPI_CASE(kEpiStoreT)                                       // product + C^T (a transposed [K, N] dgrad)
    DGT_EPI_CASE(kEpiOutF32)                                       // wgrad into fp32 grads
    DGT_EPI_CASE(kEpiOutF32 | kEpiAccumulate)                      // wgrad, gradient accumulation
    DGT_EPI_CASE(kEpiOutF32 | kEpiBias)                            // generic fp32 out
    DGT_EPI_CASE(kEpiAdam)                                         // wgrad consumed by Adam in place
    DGT_EPI_CASE_KN(kEpiMask | kEpiStoreT | kEpiBKN)               // dgrad straight from W[out, in]
    DGT_EPI_CASE_KN(kEpiMask | kEpiStoreT | kEpiBKN | kEpiColSum)  // + the bias-gradient partials
    DGT_EPI_CASE_KN(kEpiBKN)                                       // plain A . B (input gradient)
    DGT_EPI_CASE_KN(kEpiStoreT | kEpiBKN)                          // dgrad, no ReLU below
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
// out[r] (+)= sum_c in[r][c] for a bf16 [rows, cols] matrix: one wave per row, 16-B loads; out is
// fp32 or (the bf16 engine's bias gradients) bf16, an accumulation summed in fp32, rounded once.
template <typename OT>
__global__ __launch_bounds__(256) void rowsum_bf16_kernel(const u16* __restrict__ in, OT* __restrict__ out,
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
  if (l == 0) {
    if constexpr (sizeof(OT) == 4) {
      out[row] = accumulate ? out[row] + s : s;
    } else {
      u16* o = reinterpret_cast<u16*>(out);
      o[row] = f2bf(accumulate ? bf2f(o[row]) + s : s);
    }
  }
}

hipError_t rowsum_bf16(const void* in, void* out, int out_bf16, int rows, int cols, int accumulate,
                       hipStream_t stream) {
  if (cols % 8) return hipErrorInvalidValue;
  if (out_bf16)
    hipLaunchKernelGGL(rowsum_bf16_kernel<u16>, dim3((rows + 3) / 4), dim3(256), 0, stream,
                       static_cast<const u16*>(in), static_cast<u16*>(out), rows, cols, accumulate);
  else
    hipLaunchKernelGGL(rowsum_bf16_kernel<float>, dim3((rows + 3) / 4), dim3(256), 0, stream,
                       static_cast<const u16*>(in), static_cast<float*>(out), rows, cols, accumulate);
  return hipGetLastError();
}

// ------------------------------------------------------------------ BCE head
// z[b] = a[b,:] . w + b0; loss += mean BCE; dz = (sigmoid(z) - y) / B;
// g[b,:] = dz[b] * w * 1[a[b,:] > 0] (bf16, and g^T); dw = sum_b dz[b] a[b,:]; db = sum_b dz[b].
// Kernel 1: one row per wave (every 16-byte load of the row in flight together) computes
// z, dz and the row's loss term into a scratch vector.  No atomics: 1024 float / double atomics
// on ONE address serialised at the L2 and made this kernel 19 us.
// Kernel 2: one wave per 64 x 64 tile, 16-byte rows of a in, 16-byte rows of g and g^T out, the
// tile's dw partial stored to the workspace; tile (0, 0) also reduces dz -> db and the row losses
// -> loss_acc in a fixed order (one atomic, one address, one launch: deterministic).
// Kernel 3 (partials_reduce): dw = the tiles' partials summed in row-tile order.
__global__ __launch_bounds__(256) void head_fwd_kernel(const u16* __restrict__ a, const float* __restrict__ w,
                                                       const float* __restrict__ b0, const float* __restrict__ y,
                                                       int B, int D, float* __restrict__ dz,
                                                       float* __restrict__ lrow, float* __restrict__ dw) {
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
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
                                                      float* __restrict__ dw_part, float* __restrict__ db,
                                                      double* __restrict__ loss_acc, float* __restrict__ bias_part) {
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
  float gsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums of g (bias_part)
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
      gsum[e] += bf2f(gb[k][e]);
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
  // dw partial of the tile: sum the 8 row-blocks (lanes cg, cg + 8, ..., cg + 56) and store it at
  // dw_part[row tile][column]; partials_reduce sums the tiles in order (no atomics: reproducible)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float x = part[e];
    x += __shfl_xor(x, 8);
    x += __shfl_xor(x, 16);
    x += __shfl_xor(x, 32);
    part[e] = x;
  }
  if (rb == 0) {
    float4* o = reinterpret_cast<float4*>(dw_part + (long long)blockIdx.y * D + c);
    o[0] = make_float4(part[0], part[1], part[2], part[3]);
    o[1] = make_float4(part[4], part[5], part[6], part[7]);
  }
  if (bias_part) {  // the same fixed tree over the tile's 8 row blocks, for the column sums of g
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = gsum[e];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 16);
      x += __shfl_xor(x, 32);
      gsum[e] = x;
    }
    if (rb == 0) {
      float4* o = reinterpret_cast<float4*>(bias_part + (long long)blockIdx.y * D + c);
      o[0] = make_float4(gsum[0], gsum[1], gsum[2], gsum[3]);
      o[1] = make_float4(gsum[4], gsum[5], gsum[6], gsum[7]);
    }
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && wv == 0) {  // db and the step's loss, in a fixed order
    // 8 rows per lane in flight per batch, added in row order (the same sums as a plain loop, which
    // the compiler issued as one dependent load round trip per 64 rows: ~16 serial trips at B = 1024,
    // the longest path of this kernel)
    float sd = 0.f, sl = 0.f;
    for (int i0 = l; i0 < B; i0 += 64 * 8) {
      float vd[8], vl[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u;
        vd[u] = i < B ? dz[i] : 0.f;
        vl[u] = i < B ? lrow[i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sd += vd[u];
        sl += vl[u];
      }
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
  float* dwp = h.dw_part ? h.dw_part : h.scratch + h.B;
  hipLaunchKernelGGL(head_bwd_kernel, dim3(h.D / (64 * wpb), h.B / 64), dim3(64 * wpb), 0, stream,
                     static_cast<const u16*>(h.a),
                     h.w, h.dz, h.scratch, h.B, h.D, static_cast<u16*>(h.g), static_cast<u16*>(h.gT),
                     dwp, h.db, h.loss_acc, h.bias_part);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (h.dw_part) return hipSuccess;  // the caller reduces the partials (partials_reduce_multi)
  return partials_reduce(h.scratch + h.B, h.dw, 0, h.B / 64, h.D, 0, stream);
}

}  // namespace dgt
