// Operand-streaming probe for the M = 1024 bf16 MLP products (1024 x 4096 x 4096): the exact
// global -> LDS operand traffic of several block tilings, with NO MFMA, to measure what a bigger
// tile + split-K buys before writing the GEMM.  Every variant launches 256 blocks of 512 threads
// (one per CU); block b streams its tile's A rows [TM] and B rows [TN] over its K range (K / SPLIT)
// through an S-stage LDS-DMA ring, one barrier per 64-deep K-tile.
//   XS = 1: the K split runs across XCDs (blocks of one tile sit on XCDs x, x+1, ...: each XCD's L2
//           then holds a K-slice of a wider output region, fewer unique bytes per XCD);
//   XS = 0: all K slices of a tile sit on one XCD.
// The 128 x 128 / SPLIT 1 row is today's kernel's traffic (profiles/r4_panel_stream.jsonl).
// Optional fix-up traffic (FX = 1): after its loop, every block but slice 0 writes its fp32 TM x TN
// partial, slice 0 reads them back (no ordering: traffic only, not a correct reduction).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/tile_stream.hip -o build/bin/tile_stream
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
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int M = 1024, N = 4096, K = 4096, BK = 64;

template <int C>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((C & 15) | ((C >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int TM, int TN, int SPLIT, int XS, int S, int FX>
__global__ __launch_bounds__(512, 1) void stream(const u16* __restrict__ A, const u16* __restrict__ B,
                                                 float* __restrict__ ws, unsigned* out) {
  constexpr int NBM = M / TM, NT = NBM * (N / TN);
  static_assert(NT * SPLIT == 256, "one block per CU");
  constexpr int PA = TM / 64, PB = TN / 64;  // 16-B pieces per thread per K-tile
  constexpr int PER = PA + PB;
  __shared__ __attribute__((aligned(16))) u16 lds[S][(TM + TN) * BK];
  const int t = threadIdx.x, w = t >> 6, bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  int s, tile;
  if constexpr (XS) {
    s = xcd % SPLIT;
    tile = (xcd / SPLIT) * 32 + loc;
  } else {
    s = loc % SPLIT;
    tile = xcd * (NT / 8) + loc / SPLIT;
  }
  const int tm = tile % NBM, tn = tile / NBM;
  const int kbase = s * (K / SPLIT), nk = K / SPLIT / BK;
  const u16* pa[PA];
  const u16* pb[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) pa[i] = A + (long long)(tm * TM + (t >> 3) + 64 * i) * K + kbase + (t & 7) * 8;
#pragma unroll
  for (int i = 0; i < PB; ++i) pb[i] = B + (long long)(tn * TN + (t >> 3) + 64 * i) * K + kbase + (t & 7) * 8;
  auto issue = [&](int kt, int st) {
#pragma unroll
    for (int i = 0; i < PA; ++i)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pa[i] + kt * BK),
                                       reinterpret_cast<int*>(&lds[st][(i * 64 + w * 8) * BK]), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < PB; ++i)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(pb[i] + kt * BK),
                                       reinterpret_cast<int*>(&lds[st][(TM + i * 64 + w * 8) * BK]), 16, 0, 0);
  };
  for (int p = 0; p < S - 1; ++p) issue(p, p);
  unsigned acc = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + S - 1 < nk) {
      issue(kt + S - 1, (kt + S - 1) % S);
      wait_vm<(S - 1) * PER>();
    } else {
      wait_vm<0>();
    }
    __syncthreads();
    const u32x4 v = *reinterpret_cast<const u32x4*>(&lds[kt % S][(t * 8) % ((TM + TN) * BK)]);
    acc ^= v.x ^ v.w;
    __syncthreads();
  }
  if constexpr (FX) {
    // TM x TN fp32 partial per block: 512 threads x (TM * TN / 2048) f32x4, lane-linear
    constexpr int V = TM * TN / 4 / 512;
    f32x4* base = reinterpret_cast<f32x4*>(ws) + (long long)tile * SPLIT * TM * TN / 4;
    if (s != 0) {
      f32x4* p = base + (long long)s * TM * TN / 4;
#pragma unroll 4
      for (int i = 0; i < V; ++i) p[i * 512 + t] = f32x4{(float)acc, 1.f, 2.f, 3.f};
    } else {
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
      for (int q = 1; q < SPLIT; ++q) {
        const f32x4* p = base + (long long)q * TM * TN / 4;
#pragma unroll 4
        for (int i = 0; i < V; ++i) sum += p[i * 512 + t];
      }
      acc ^= __float_as_uint(sum.x + sum.y + sum.z + sum.w);
    }
  }
  if (acc == 0x12345678u) out[bid] = acc;
}

template <typename Kern>
static float time_it(Kern k, const u16* A, const u16* B, float* ws, unsigned* out, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, A, B, ws, out);
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, A, B, ws, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  u16 *A, *B;
  float* ws;
  unsigned* out;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&ws, (size_t)M * N * 4 * 4));
  CK(hipMalloc(&out, 256 * 4));
  std::vector<u16> h((size_t)N * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (u16)(0x3c00 + (i * 2654435761u >> 20) % 512);
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  struct R {
    const char* name;
    double mib_per_cu;
    float us;
  };
  const double MiB = 1 << 20;
  auto per_cu = [&](int tm, int tn, int split) { return (double)(tm + tn) * (K / split) * 2 / MiB; };
  std::vector<R> rs;
  for (int rep = 0; rep < 2; ++rep) {
    rs.push_back({"128x128 split1 S4", per_cu(128, 128, 1), time_it(stream<128, 128, 1, 0, 4, 0>, A, B, ws, out, 50)});
    rs.push_back({"128x128 split1 S3", per_cu(128, 128, 1), time_it(stream<128, 128, 1, 0, 3, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x128 split2 XS0 S3", per_cu(256, 128, 2), time_it(stream<256, 128, 2, 0, 3, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x128 split2 XS1 S3", per_cu(256, 128, 2), time_it(stream<256, 128, 2, 1, 3, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x128 split2 XS1 S2", per_cu(256, 128, 2), time_it(stream<256, 128, 2, 1, 2, 0>, A, B, ws, out, 50)});
    rs.push_back({"128x256 split2 XS1 S3", per_cu(128, 256, 2), time_it(stream<128, 256, 2, 1, 3, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x256 split4 XS0 S2", per_cu(256, 256, 4), time_it(stream<256, 256, 4, 0, 2, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x256 split4 XS1 S2", per_cu(256, 256, 4), time_it(stream<256, 256, 4, 1, 2, 0>, A, B, ws, out, 50)});
    rs.push_back({"256x128 split2 XS1 S3 +fixup", per_cu(256, 128, 2), time_it(stream<256, 128, 2, 1, 3, 1>, A, B, ws, out, 50)});
    rs.push_back({"256x256 split4 XS1 S2 +fixup", per_cu(256, 256, 4), time_it(stream<256, 256, 4, 1, 2, 1>, A, B, ws, out, 50)});
  }
  CK(hipDeviceSynchronize());
  for (const R& r : rs)
    std::printf("{\"mode\": \"%s\", \"MiB_per_CU\": %.2f, \"us\": %.2f, \"GBps_per_CU\": %.1f, \"TBps_chip\": %.2f}\n",
                r.name, r.mib_per_cu, r.us, r.mib_per_cu * MiB / r.us / 1e3, r.mib_per_cu * MiB * 256 / r.us / 1e6);
  return 0;
}
