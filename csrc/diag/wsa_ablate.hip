// Diagnostic harness (not part of the extension): the MLP's wgrad + Adam layer (M = N = 4096,
// K = 1024, kEpiAdam) on variants 0 / 4 / 6, and variant 6 with one wave group idled:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc [-DDGT_WSA_ABLATE=1|2] csrc/diag/wsa_ablate.hip -o build/bin/wsa_ablate_N
//   DGT_WSA_ABLATE unset: shipped; 1: Adam waves idle (only the barriers); 2: MFMA waves idle.
#include "../gemm.hip"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

int main() {
  const int M = 4096, N = 4096, K = 1024;
  std::vector<unsigned short> h((size_t)M * K);
  for (size_t i = 0; i < h.size(); ++i) {
    unsigned x = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    const float f = ((float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f) * 0.05f;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  void *A, *B, *lp;
  float *p, *m, *v;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&lp, (size_t)M * N * 2));
  CK(hipMalloc(&p, (size_t)M * N * 4));
  CK(hipMalloc(&m, (size_t)M * N * 4));
  CK(hipMalloc(&v, (size_t)M * N * 4));
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  CK(hipMemset(p, 0, (size_t)M * N * 4));
  CK(hipMemset(m, 0, (size_t)M * N * 4));
  CK(hipMemset(v, 0, (size_t)M * N * 4));
  dgt::GemmArgs g{};
  g.A = A; g.B = B; g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = K; g.ldc = N; g.alpha = 1.f;
  g.adam.master = p; g.adam.m = m; g.adam.v = v; g.adam.lp = lp;
  g.adam.hp = dgt::AdamHyper{1e-4f, 0.999f, 0.1f, 0.001f, 1e-8f, 0.f, 1.f, 0};
  g.adam.step_size_neg = -1e-3f;
  g.adam.bc2_sqrt = 0.05f;
#ifdef DGT_WSA_ABLATE
  const int ab = DGT_WSA_ABLATE;
#else
  const int ab = 0;
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    for (int variant : {0, 4, 6}) {
      if (ab && variant != 6) continue;
      for (int w = 0; w < 3; ++w) CK(dgt::gemm_nt(g, dgt::kEpiAdam, 0, variant));
      CK(hipDeviceSynchronize());
      const int iters = 20;
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) CK(dgt::gemm_nt(g, dgt::kEpiAdam, 0, variant));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("variant=%d ablate=%d  %.1f us per wgrad+Adam layer\n", variant, ab, ms * 1e3 / iters);
    }
  }
  return 0;
}
