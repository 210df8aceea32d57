// Diagnostic harness (not part of the extension): where does one fused training step spend its
// cycles?  Builds the training kernel with per-section s_memtime stamps and reports cycles/step per
// section for waves 0 and 1.  Read the SHARES, not the total: stamps serialize the schedule.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -Icsrc csrc/diag/tiny_stamps.hip \
//         -o build/bin/tiny_stamps
#define DGT_TINY_STAMPS 1
#include "../tiny_mlp.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const int F = 20, H = 64, N = 2000, B = 4;
  const int steps = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937 rng(42);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> X(N * F), Y(N);
  for (auto& v : X) v = nd(rng);
  for (int i = 0; i < N; ++i) {
    float s = 0;
    for (int k = 0; k < F / 2; ++k) s += X[i * F + k];
    Y[i] = s > 0 ? 1.f : 0.f;
  }
  std::vector<int> plan(steps * B), counts(steps, B);
  for (auto& v : plan) v = (int)(rng() % N);
  const int PP = dgt::tiny_mlp_padded_numel(F, H);
  std::vector<float> params(PP, 0.f);
  for (int i = 0; i < H * F + 2 * H + 1; ++i) params[i] = 0.1f * nd(rng);

  float *dX, *dY, *dP, *dM, *dV;
  int *dPlan, *dCounts, *dStatus;
  double* dLoss;
  unsigned long long* dStamps;
  CK(hipMalloc(&dX, X.size() * 4));
  CK(hipMalloc(&dY, Y.size() * 4));
  CK(hipMalloc(&dP, PP * 4));
  CK(hipMalloc(&dM, PP * 4));
  CK(hipMalloc(&dV, PP * 4));
  CK(hipMalloc(&dPlan, plan.size() * 4));
  CK(hipMalloc(&dCounts, counts.size() * 4));
  CK(hipMalloc(&dStatus, 4));
  CK(hipMalloc(&dLoss, 8));
  CK(hipMalloc(&dStamps, 16 * 8));
  CK(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dY, Y.data(), Y.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dP, params.data(), PP * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dM, 0, PP * 4));
  CK(hipMemset(dV, 0, PP * 4));
  CK(hipMemcpy(dPlan, plan.data(), plan.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dCounts, counts.data(), counts.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dLoss, 0, 8));
  CK(hipMemset(dStamps, 0, 16 * 8));

  dgt::TinyTrainArgs a = {};
  a.X = dX; a.Y = dY; a.plan = dPlan; a.counts = dCounts; a.n_steps = steps; a.bmax = B;
  a.params = dP; a.exp_avg = dM; a.exp_avg_sq = dV;
  a.hp = {1e-3f, 0.999f, (float)(1.0 - 0.9), (float)(1.0 - 0.999), 1e-8f, 0.f, 1.f, 0};
  a.lr = 1e-3; a.beta1 = 0.9; a.beta2 = 0.999; a.adam_step0 = 0;
  a.loss_acc = dLoss; a.status = dStatus;
  a.ex.rank = 0; a.ex.world_size = 1;
  a.stamps = dStamps;
  float* dBc;
  CK(hipMalloc(&dBc, (size_t)(steps + 1) * 2 * sizeof(float)));  // +1: read-ahead of the kernel
  a.bc = dBc;
  CK(dgt::tiny_mlp_train(F, H, a, 0));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(dStamps, 0, 16 * 8));
  CK(hipEventRecord(e0, 0));
  CK(dgt::tiny_mlp_train(F, H, a, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long st[16];
  CK(hipMemcpy(st, dStamps, sizeof(st), hipMemcpyDeviceToHost));
  const char* names[5] = {"prefetch+fwd GEMM+partial z", "barrier wait", "loss+bwd+wgrad MFMA",
                          "stage next batch+grad regs", "Adam (packed fp32)"};
  printf("stamped build: %.3f us/step (%d steps), launch event-to-event %.2f us\n", ms * 1e3 / steps, steps,
         ms * 1e3);
  printf("phases of wave 0 (s_memrealtime, 10 ns ticks): operands landed %.2f us, prologue barrier %.2f us, "
         "loop %.2f us, epilogue + store completion %.2f us\n",
         st[5] * 0.01, st[6] * 0.01, st[7] * 0.01, st[13] * 0.01);
  for (int w = 0; w < 2; ++w) {
    unsigned long long tot = 0;
    for (int i = 0; i < 5; ++i) tot += st[w * 8 + i];
    printf("wave %d: total %.0f cyc/step\n", w, (double)tot / steps);
    for (int i = 0; i < 5; ++i)
      printf("  %-30s %8.0f cyc/step  %5.1f%%\n", names[i], (double)st[w * 8 + i] / steps,
             100.0 * st[w * 8 + i] / (double)tot);
  }
  return 0;
}
