// Operand-streaming microbenchmark for the M = 1024 MLP GEMM (1024 x 4096 x 4096 bf16, 128 x 128
// tiles, 256 blocks of 512 threads = one block per CU): the GEMM's exact global -> LDS traffic
// (block (tm, tn) reads A rows [128 tm, +128) and B rows [128 tn, +128) over K, 64 columns per K-tile
// = 32 KiB) with NO MFMA, to measure how fast one CU can fetch its 2 MiB of operands:
//   mode 0: LDS-DMA (global_load_lds_dwordx4), S K-tiles in flight (S-stage LDS ring)
//   mode 1: global_load_dwordx4 into VGPRs, D K-tiles of loads in flight, ds_write_b128 into a
//           2-stage LDS ring (the in-flight bytes live in registers, not LDS)
// One barrier per K-tile in both, and one ds_read_b128 per thread per tile folded into a checksum
// so nothing is dead.  Prints us per launch and GB/s per CU.  Reads only; writes one word per block.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/diag/panel_stream.hip -o build/bin/panel_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

typedef unsigned short u16;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int M = 1024, N = 4096, K = 4096, BM = 128, BK = 64, TILE = BM * BK;  // elements per operand tile

__device__ __forceinline__ void tile_of(int bid, int nbm, int nbn, int& tm, int& tn) {
  const int nwg = nbm * nbn, xcd = bid % 8, q = nwg / 8, r = nwg % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  const int group = wgid / (8 * nbn), first = group * 8, gsize = min(nbm - first, 8);
  tm = first + (wgid % (8 * nbn)) % gsize;
  tn = (wgid % (8 * nbn)) / gsize;
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N_ & 15) | ((N_ >> 4) << 14) | (7 << 4) | (15 << 8));
}

// mode 0: each thread's 2 pieces per operand tile (512 threads x 16 B = 8 KiB per instruction set;
// 16 KiB per operand tile = 2 pieces per thread), S stages.
template <int S>
__global__ __launch_bounds__(512, 1) void stream_dma(const u16* __restrict__ A, const u16* __restrict__ B,
                                                     unsigned* out) {
  __shared__ __attribute__((aligned(16))) u16 lds[S][2 * TILE];
  const int t = threadIdx.x;
  int tm, tn;
  tile_of(blockIdx.x, M / BM, N / BM, tm, tn);
  // piece i of a tile: row = (t >> 3) + 64 i, chunk = t & 7 (16 B = 8 bf16)
  const u16* pa[2];
  const u16* pb[2];
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 64 * i, c = t & 7;
    pa[i] = A + (long long)(tm * BM + row) * K + c * 8;
    pb[i] = B + (long long)(tn * BM + row) * K + c * 8;
  }
  const int w = t >> 6;
  auto issue = [&](int kt, int st) {
    for (int i = 0; i < 2; ++i) {
      // the wave's 64 lanes write 1 KiB contiguous: LDS offset of the wave's piece
      u16* la = &lds[st][0] + (i * 64 + w * 8) * BK;
      u16* lb = &lds[st][TILE] + (i * 64 + w * 8) * BK;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pa[i] + kt * BK), reinterpret_cast<int*>(la), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pb[i] + kt * BK), reinterpret_cast<int*>(lb), 16, 0, 0);
    }
  };
  const int nk = K / BK;
  for (int s = 0; s < S - 1; ++s) issue(s, s);
  unsigned acc = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    // tile kt landed: everything but the newest S-1 tiles (4 DMAs each)
    if (kt + S - 1 < nk) {
      if constexpr (S == 2) wait_vm<4>();
      else if constexpr (S == 3) wait_vm<8>();
      else if constexpr (S == 4) wait_vm<12>();
      else wait_vm<16>();
    } else {
      wait_vm<0>();
    }
    __syncthreads();
    const u32x4 v = *reinterpret_cast<const u32x4*>(&lds[kt % S][(t * 8) % (2 * TILE)]);
    acc ^= v.x ^ v.w;
    __syncthreads();  // WAR: stage kt % S is refilled S-1 tiles later
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// mode 1: per thread 4 x 16 B per K-tile (2 of A, 2 of B) held in VGPRs, D tiles in flight
template <int D>
__global__ __launch_bounds__(512, 1) void stream_reg(const u16* __restrict__ A, const u16* __restrict__ B,
                                                     unsigned* out) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2 * TILE];
  const int t = threadIdx.x;
  int tm, tn;
  tile_of(blockIdx.x, M / BM, N / BM, tm, tn);
  const u16* pa[2];
  const u16* pb[2];
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 64 * i, c = t & 7;
    pa[i] = A + (long long)(tm * BM + row) * K + c * 8;
    pb[i] = B + (long long)(tn * BM + row) * K + c * 8;
  }
  u32x4 reg[D][4];
  auto load = [&](int kt, u32x4 (&r)[4]) {
    for (int i = 0; i < 2; ++i) {
      r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pa[i] + kt * BK));
      r[2 + i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pb[i] + kt * BK));
    }
  };
  const int nk = K / BK;
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, reg[d]);
  unsigned acc = 0;
  for (int kt0 = 0; kt0 < nk; kt0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int kt = kt0 + d;
      u16* st = lds[kt & 1];
      for (int i = 0; i < 2; ++i) {
        *reinterpret_cast<u32x4*>(st + (t + 512 * i) * 8) = reg[d][i];
        *reinterpret_cast<u32x4*>(st + TILE + (t + 512 * i) * 8) = reg[d][2 + i];
      }
      if (kt + D < nk) load(kt + D, reg[d]);
      __syncthreads();
      const u32x4 v = *reinterpret_cast<const u32x4*>(st + (t * 8) % (2 * TILE));
      acc ^= v.x ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <typename Kern>
static float time_it(Kern k, const u16* A, const u16* B, unsigned* out, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, A, B, out);
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, A, B, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  u16 *A, *B;
  unsigned* out;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&out, 256 * 4));
  std::vector<u16> h((size_t)N * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (u16)(0x3c00 + (i * 2654435761u >> 20) % 512);
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  const double per_cu = 2.0 * BM * K * 2;  // bytes per block (one block per CU)
  struct R { const char* name; float us; };
  std::vector<R> rs = {
      {"dma S=2", time_it(stream_dma<2>, A, B, out, 50)}, {"dma S=3", time_it(stream_dma<3>, A, B, out, 50)},
      {"dma S=4", time_it(stream_dma<4>, A, B, out, 50)}, {"dma S=5", time_it(stream_dma<5>, A, B, out, 50)},
      {"reg D=1", time_it(stream_reg<1>, A, B, out, 50)}, {"reg D=2", time_it(stream_reg<2>, A, B, out, 50)},
      {"reg D=4", time_it(stream_reg<4>, A, B, out, 50)}};
  CK(hipDeviceSynchronize());
  for (const R& r : rs)
    std::printf("{\"mode\": \"%s\", \"us\": %.2f, \"GBps_per_CU\": %.1f, \"TBps_chip\": %.2f}\n", r.name, r.us,
                per_cu / r.us / 1e3, per_cu * 256 / r.us / 1e6);
  return 0;
}
