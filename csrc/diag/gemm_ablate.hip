// Diagnostic harness (not part of the extension): times the 128x128 4-stage 8-wave GEMM on the
// MLP's M = 1024 shapes with parts of its main loop removed, to see what bounds it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc [-DDGT_GEMM_ABLATE=1|2] csrc/diag/gemm_ablate.hip -o build/bin/gemm_ablate_N
//   DGT_GEMM_ABLATE unset: the shipped loop; 1: no staging inside the loop (operands of the first
//   S-1 tiles reused); 2: LDS fragment reads without MFMAs.
//   ./gemm_ablate_N [variant] [hot|cold]: cold cycles B through 10 copies (> the Infinity Cache).
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

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 4;
  const int M = 1024, N = 4096, K = 4096;
  std::vector<unsigned short> h((size_t)N * K);
  // uniform [-1, 1) operands (bf16 bit patterns from a hash): trivial or one-signed data lets the
  // chip hold a higher clock and ranks variants wrongly (MI355X_MICROARCH.md, DVFS give-back)
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
  // "cold": B cycles through NB copies (10 x 32 MB > the 256 MB Infinity Cache), as the MLP's
  // weights arrive from HBM after the optimizer step; "hot": one B, L2/MALL-resident
  const bool cold = argc > 2 && argv[2][0] == 'c';
  const int NB = cold ? 10 : 1;
  void *A, *C;
  std::vector<void*> Bs(NB);
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  for (int b = 0; b < NB; ++b) {
    CK(hipMalloc(&Bs[b], (size_t)N * K * 2));
    CK(hipMemcpy(Bs[b], h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  }
  void* B = Bs[0];
  dgt::GemmArgs g{};
  g.A = A; g.B = B; g.C = C; g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = K; g.ldc = N; g.alpha = 1.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
#ifdef DGT_GEMM_ABLATE
  const int ab = DGT_GEMM_ABLATE;
#else
  const int ab = 0;
#endif
  // epi 0: B is [N, K] (forward form); kEpiBKN: B is [K, N] (dgrad straight from W)
  for (int epi : {0, (int)dgt::kEpiBKN}) {
    for (int w = 0; w < 5; ++w) CK(dgt::gemm_nt(g, epi, 0, variant));
    CK(hipDeviceSynchronize());
    const int iters = 50;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) {
      g.B = Bs[i % NB];
      CK(dgt::gemm_nt(g, epi, 0, variant));
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned short> c((size_t)M * N);
    CK(hipMemcpy(c.data(), C, c.size() * 2, hipMemcpyDeviceToHost));
    unsigned long long sum = 0;
    for (size_t i = 0; i < c.size(); ++i) sum = sum * 1000003ull + c[i];
    printf("variant=%d ablate=%d B=%s  %.1f us/gemm (%s)  %.0f TF  C hash %016llx\n", variant, ab,
           epi ? "[K,N]" : "[N,K]", ms * 1e3 / iters, cold ? "cold B" : "hot", 2.0 * M * N * K / (ms * 1e-3 / iters) / 1e12,
           sum);
  }
  return 0;
}
