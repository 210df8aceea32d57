// Diagnostic harness (not part of the extension): the MLP's M = 1024 forward product
// C[1024, 4096] = A[1024, 4096] . B[4096, 4096]^T (bf16, plain bf16 store) on a 128 x 128 tile with
// hipBLASLt's macro-tile shape -- 4 waves of 64 x 64, BK = 128 per barrier, two 64 KiB LDS stages --
// staged with LDS-DMA like the shipped kernels, against the shipped 8-wave BK = 64 kernel (variant 4).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc csrc/diag/gemm_bk128.hip -o build/bin/gemm_bk128
//   ./gemm_bk128 [hot|cold]
#include "../gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

namespace dgt {
namespace bk128 {
constexpr int BM = 128, BN = 128, BK = 128;
// one 128 x 128 bf16 operand tile = 32 KiB: 256-byte rows of 16 chunks, chunk XOR-swizzled by
// row & 15 so a 16-lane group reading one chunk index of 16 consecutive rows hits 16 bank groups
template <int NW>
DGT_DEVICE void stage(const u16* __restrict__ src, int ld, int row0, int k0, u16* lds, int w, int l) {
  constexpr int PW = 32 / NW;             // 32 wave-instructions of 1 KiB (4 rows) per tile
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int rblk = (w * PW + i) * 4;    // first of the 4 rows
    const int row = rblk + (l >> 4);
    const int p = l & 15;                 // physical chunk this lane lands in
    const int c = p ^ (row & 15);         // logical chunk fetched
    const u16* g = src + (long long)(row0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const int*>(g), reinterpret_cast<int*>(lds + rblk * BK), 16, 0,
                                     0);
  }
}
DGT_DEVICE bf16x8 frag(const u16* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row * BK + ((chunk ^ (row & 15)) * 8));
}
}  // namespace bk128

template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void gemm_bk128_kernel(GemmArgs g) {
  using namespace bk128;
  constexpr int WN = NW == 8 ? 32 : 64, WCOLS = BN / WN, NJ = WN / 16;
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][BM * BK];  // 128 KiB
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int tm, tn;
  tile_of_block(blockIdx.x, g.M / BM, g.N / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN, wr = w / WCOLS, wc = w % WCOLS;
  const u16* A = static_cast<const u16*>(g.A);
  const u16* B = static_cast<const u16*>(g.B);
  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = g.K / BK;
  stage<NW>(A, g.lda, m0, 0, lds[0][0], w, l);
  stage<NW>(B, g.ldb, n0, 0, lds[0][1], w, l);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    wait_vmcnt<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // stage cur landed for every wave; stage cur^1 free
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) {
      stage<NW>(A, g.lda, m0, (kt + 1) * BK, lds[cur ^ 1][0], w, l);
      stage<NW>(B, g.ldb, n0, (kt + 1) * BK, lds[cur ^ 1][1], w, l);
    }
    const u16* As = lds[cur][0];
    const u16* Bs = lds[cur][1];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (l >> 4);
      bf16x8 af[4], bf[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(As, wr * 64 + i * 16 + (l & 15), chunk);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = frag(Bs, wc * WN + j * 16 + (l & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  u16* C = static_cast<u16*>(g.C);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(long long)(m0 + wr * 64 + i * 16 + 4 * (l >> 4) + r) * g.ldc + n0 + wc * WN + j * 16 + (l & 15)] =
            f2bf(acc[i][j][r] * g.alpha);
}
}  // namespace dgt

int main(int argc, char** argv) {
  const int M = 1024, N = 4096, K = 4096;
  const bool cold = argc > 1 && argv[1][0] == 'c';
  const int NB = cold ? 10 : 1;
  std::vector<unsigned short> h((size_t)N * K);
  for (size_t i = 0; i < h.size(); ++i) {
    unsigned x = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    const float f = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  void *A, *C1, *C2;
  std::vector<void*> Bs(NB);
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&C1, (size_t)M * N * 2));
  CK(hipMalloc(&C2, (size_t)M * N * 2));
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  for (int b = 0; b < NB; ++b) {
    CK(hipMalloc(&Bs[b], (size_t)N * K * 2));
    CK(hipMemcpy(Bs[b], h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  }
  dgt::GemmArgs g{};
  g.A = A; g.B = Bs[0]; g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = K; g.ldc = N; g.alpha = 1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (M / 128) * (N / 128);
  const char* names[3] = {"shipped v4 (8 waves, BK 64)", "bk128 4 waves 64x64", "bk128 8 waves 64x32"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int arm = 0; arm < 3; ++arm) {
      g.C = arm ? C2 : C1;
      auto launch = [&]() {
        if (arm == 0) CK(dgt::gemm_nt(g, 0, 0, 4));
        else if (arm == 1) hipLaunchKernelGGL(dgt::gemm_bk128_kernel<4>, dim3(grid), dim3(256), 0, 0, g);
        else hipLaunchKernelGGL(dgt::gemm_bk128_kernel<8>, dim3(grid), dim3(512), 0, 0, g);
      };
      for (int w = 0; w < 3; ++w) launch();
      CK(hipDeviceSynchronize());
      const int iters = 40;
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) {
        g.B = Bs[i % NB];
        launch();
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      g.B = Bs[0];
      printf("%-28s %s  %.1f us  %.0f TF\n", names[arm],
             cold ? "cold" : "hot ", ms * 1e3 / iters, 2.0 * M * N * K / (ms * 1e-3 / iters) / 1e12);
    }
  }
  // same bits? (both accumulate K in 32-chunks in order)
  std::vector<unsigned short> c1((size_t)M * N), c2((size_t)M * N);
  CK(hipMemcpy(c1.data(), C1, c1.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c2.data(), C2, c2.size() * 2, hipMemcpyDeviceToHost));
  size_t diff = 0;
  for (size_t i = 0; i < c1.size(); ++i) diff += c1[i] != c2[i];
  printf("outputs differing: %zu of %zu\n", diff, c1.size());
  return 0;
}
