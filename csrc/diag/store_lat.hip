// Store-path microbenchmark for the fused kernel's LL exchange: how long W waves of one workgroup
// take to issue K 16-byte-per-lane stores (1 KiB per wave instruction, the mailbox layout) and to
// drain them (s_waitcnt vmcnt(0)), per memory kind: hipMalloc (coarse-grained), uncached
// (hipDeviceMallocUncached, the mailbox default) and fine-grained.  Prints ns per wave-instruction.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/diag/store_lat.hip -o build/bin/store_lat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// out[wave*2+0] = issue ticks, out[wave*2+1] = issue + drain ticks (s_memrealtime, 100 MHz)
__global__ void store_kernel(unsigned* buf, int k, unsigned tag, unsigned long long* out) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned* base = buf + (size_t)w * k * 256 + l * 4;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < k; ++i) {
    u32x4 v = {(unsigned)i, tag, (unsigned)l, tag};
    *reinterpret_cast<u32x4*>(base + (size_t)i * 256) = v;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (l == 0) {
    out[w * 2] = t1 - t0;
    out[w * 2 + 1] = t2 - t0;
  }
}

int main() {
  const int kMaxK = 64, kMaxW = 8;
  const size_t bytes = (size_t)kMaxW * kMaxK * 1024;
  struct Kind {
    const char* name;
    unsigned flags;
    bool plain;
  } kinds[] = {{"hipMalloc", 0, true},
               {"uncached", hipDeviceMallocUncached, false},
               {"finegrained", hipDeviceMallocFinegrained, false}};
  unsigned long long* out;
  CK(hipMalloc(&out, kMaxW * 2 * sizeof(unsigned long long)));
  for (const Kind& kd : kinds) {
    unsigned* buf = nullptr;
    if (kd.plain) CK(hipMalloc(&buf, bytes));
    else CK(hipExtMallocWithFlags((void**)&buf, bytes, kd.flags));
    CK(hipMemset(buf, 0, bytes));
    for (int waves : {1, 4}) {
      for (int k : {4, 12, 28, 56}) {
        std::vector<double> issue, total;
        for (int rep = 0; rep < 50; ++rep) {
          hipLaunchKernelGGL(store_kernel, dim3(1), dim3(64 * waves), 0, 0, buf, k, (unsigned)rep + 1, out);
          CK(hipDeviceSynchronize());
          unsigned long long h[kMaxW * 2];
          CK(hipMemcpy(h, out, waves * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
          if (rep < 5) continue;
          unsigned long long mi = 0, mt = 0;
          for (int w = 0; w < waves; ++w) {
            mi = std::max(mi, h[w * 2]);
            mt = std::max(mt, h[w * 2 + 1]);
          }
          issue.push_back(mi * 10.0);
          total.push_back(mt * 10.0);
        }
        std::sort(issue.begin(), issue.end());
        std::sort(total.begin(), total.end());
        const double mi = issue[issue.size() / 2], mt = total[total.size() / 2];
        std::printf("%-12s waves=%d k=%2d  issue %7.0f ns  issue+drain %7.0f ns  = %6.1f ns per wave-instruction\n",
                    kd.name, waves, k, mi, mt, mt / k);
      }
    }
    CK(hipFree(buf));
  }
  CK(hipFree(out));
  return 0;
}
