// Cross-GPU one-shot all-reduce over xGMI for latency-bound (small) buckets.
//
// Why: the reference's only per-step collective is a 5.6 KB gradient all-reduce.
// A ring all-reduce (RCCL) crosses 2(n-1) = 14 hops at n = 8; on MI355X every GPU has a direct
// xGMI link to each of its 7 peers, so a push-based one-shot exchange costs ONE link latency:
// every rank streams its buffer into each peer's mailbox as low-latency (LL) lines (payload and
// sequence tag in every 8-byte pair, dgt_common.h), then polls its own mailbox until every peer's
// lines carry this call's tag and sums the contributions locally in rank order (bit-identical
// results on every rank).  No fences, no flags, no inter-block synchronisation: every block owns
// a disjoint range of the buffer, so the grid can be as wide as the payload.
//
// Mailbox slot layout (words): float4 i -> LL lines 2*(i/64) and 2*(i/64)+1, lane i%64 -> every
// wave-instruction writes or reads 1 KiB contiguous.
// Reference: the gradient all-reduce of model_engine.backward, train.py:113.
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

constexpr int kMaxBlocks = 256;

DGT_DEVICE long long os_word(long long i) { return (2 * (i >> 6)) * 256 + (i & 63) * 4; }

__global__ __launch_bounds__(256) void oneshot_allreduce_kernel(const float* __restrict__ in,
                                                                float* __restrict__ out, long long n,
                                                                float scale, Exchange ex, int* status,
                                                                int reps) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long first = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  bool late = false;
  // reps > 1 runs back-to-back all-reduces of the same input (latency measurement without launch
  // gaps).  Safe without grid synchronisation: every rank gives thread t the same elements, and a
  // sender reaches rep r+2 (same parity slot) only after reading the peer's rep r+1, which the
  // peer pushes only after it has read rep r.
  for (int r = 0; r < reps && !late; ++r) {
    const long long seq = ex.seq_base + r;
    const int parity = (int)(seq & 1);
    const unsigned tag = (unsigned)(seq + 1);
    const long long mine = ll_slot(ex, parity, ex.rank);

    for (long long i = first; i < n4; i += stride) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(in + 4 * i);
      const long long o = mine + os_word(i);
      for (int p = 0; p < ex.world_size; ++p) {
        if (p == ex.rank) continue;
        ll_put(ex.data[p] + o, v[0], v[1], tag);
        ll_put(ex.data[p] + o + 256, v[2], v[3], tag);
      }
    }

    const unsigned long long t0 = realtime();
    for (long long i = first; i < n4; i += stride) {
      const long long o = os_word(i);
      unsigned long long v[kMaxRanks][4];
      bool ready;
      do {  // re-read every peer's lines per retry: one round trip per poll
        ready = true;
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p) {
          if (p < ex.world_size && p != ex.rank) {
            const unsigned* src = ex.data[ex.rank] + ll_slot(ex, parity, p) + o;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[p][k] = ll_get(src + (k >> 1) * 256 + (k & 1) * 2);
          }
        }
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p) {
          if (p < ex.world_size && p != ex.rank) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ready = ready && ll_ok(v[p][k], tag);
          }
        }
        if (!ready && (long long)(realtime() - t0) > ex.timeout_ticks) late = true;
      } while (!ready && !late);
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p) {
        if (p >= ex.world_size) continue;
        if (p == ex.rank) sum += *reinterpret_cast<const f32x4*>(in + 4 * i);
        else sum += f32x4{ll_val(v[p][0]), ll_val(v[p][1]), ll_val(v[p][2]), ll_val(v[p][3])};
      }
      *reinterpret_cast<f32x4*>(out + 4 * i) = sum * scale;
    }
  }
  if (late) atomicExch(status, (int)kTimeout);
}

hipError_t oneshot_allreduce(const float* in, float* out, long long n, float scale, const Exchange& ex,
                             int* status, hipStream_t stream, int reps) {
  if (reps < 1 || n % 4 != 0 || n > ex.stride || (ex.stride & 255) || ex.world_size < 1 || ex.world_size > kMaxRanks)
    return hipErrorInvalidValue;
  const long long n4 = n / 4;
  long long blocks = (n4 + 255) / 256;  // one float4 per thread up to 256 blocks (1 MiB)
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3((int)blocks), dim3(256), 0, stream, in, out, n, scale, ex,
                     status, reps);
  return hipGetLastError();
}

// ---- bf16 -> fp32 widening of a gradient bucket onto its fp32 wire buffer (bucket_launcher.cpp):
// 8 elements (16 B in, 32 B out) per lane per iteration, grid-stride; a scalar tail / unaligned path.
__global__ __launch_bounds__(256) void widen_bf16_kernel(const unsigned short* __restrict__ src,
                                                          float* __restrict__ dst, long long n, int vec) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  long long done = 0;
  if (vec) {
    const long long n8 = n >> 3;
    const uint4* s8 = reinterpret_cast<const uint4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (long long k = i; k < n8; k += stride) {
      const uint4 v = s8[k];
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[2 * j] = __uint_as_float(w[j] << 16);
        o[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      }
      d4[2 * k] = make_float4(o[0], o[1], o[2], o[3]);
      d4[2 * k + 1] = make_float4(o[4], o[5], o[6], o[7]);
    }
    done = n8 << 3;
  }
  for (long long k = done + i; k < n; k += stride) dst[k] = __uint_as_float((unsigned)src[k] << 16);
}

hipError_t widen_bf16_f32(const void* src, float* dst, long long n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 31) == 0;
  const long long work = vec ? (n >> 3) : n;
  long long blocks = (work + 255) / 256;
  if (blocks > 4096) blocks = 4096;  // grid-stride beyond 16 blocks per CU
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(widen_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     static_cast<const unsigned short*>(src), dst, n, vec);
  return hipGetLastError();
}

}  // namespace dgt
