// Shared device helpers for the MI355X (gfx950 / CDNA4) kernels of distributed_gpu_test_amd.
// Wave64 everywhere: every cross-lane helper assumes 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DGT_HOST_DEVICE __host__ __device__ __forceinline__
#define DGT_DEVICE __device__ __forceinline__

namespace dgt {

constexpr int kWave = 64;
constexpr int kMaxRanks = 8;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- status words written by kernels (read by the host after a sync)
enum Status : int {
  kOk = 0,
  kTimeout = 1,       // a cross-GPU spin exceeded its bound
  kBadShape = 2,      // launch arguments disagree with what the kernel was built for
};

// Scalars are rounded to fp32 on the host from double, the way torch passes python floats to
// its foreach kernels (1 - beta1 is computed in double, THEN rounded).
struct AdamHyper {
  float lr;
  float beta2;
  float one_minus_beta1;
  float one_minus_beta2;
  float eps;
  float weight_decay;
  float decay;  // 1 - lr * weight_decay (AdamW)
  int adamw;    // 1: decoupled weight decay (AdamW); 0: L2 added to the gradient (torch.optim.Adam)
};

// Cross-GPU exchange arguments for the IPC one-shot gradient exchange.  Every rank owns one
// "mailbox" allocation (uncached device memory, IPC-exported); peers write into it over xGMI.
//   data : LL lines [2 parity][kMaxRanks src][stride / 2]     (stride = payload floats per slot)
// A low-latency (LL) line is 16 bytes = two {payload float, tag} pairs; the tag is the exchange's
// sequence number + 1.  Each aligned 8-byte pair is written and read with ONE 64-bit atomic access,
// so a reader that sees both tags of a line has both payloads: no release fence, no separate flag,
// no acquire fence, and the reader's polls return the data itself (one xGMI latency per exchange).
// Tags increase monotonically per channel, so mailboxes are zeroed once, at creation.
struct Exchange {
  int rank;
  int world_size;
  int stride;                       // payload floats per (parity, src) slot; the slot is 2*stride words
  long long seq_base;               // sequence number of the first exchange of this launch (0-based)
  long long timeout_ticks;          // bound on every spin, in s_memrealtime ticks (100 MHz)
  unsigned* data[kMaxRanks];        // each rank's mailbox (index rank = local)
  long long corrupt_step;           // fault injection: at this 1-based optimizer step the fused kernel
                                    // corrupts one payload it sends to rank + 1 (-1 = never)
  int zero1;                        // fused kernel: ZeRO-1 exchange (gradients reduce-scattered to lane
                                    // owners, owners update, parameters all-gathered) instead of the
                                    // one-shot all-to-all of gradients
  int line;                         // fused kernel line format: 3 = LL3 (16-byte lines), 2 = LL2 (8-byte pairs)
  unsigned* xsum;                   // ZeRO-1 transfer checksums (null = off): per thread t, [2t] ^= every
                                    // parameter word its lane sent (owner) or received (all-gather) and
                                    // [2t + 1] ^= every gradient word it sent (non-owner) or received
                                    // from peers (owner), over the launch.  A transfer fault ZeRO-1 would
                                    // heal at the next all-gather still shows up as a mismatch between
                                    // ranks (runtime/tiny_trainer.py: verify_replicas).
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// word offset of (parity, src)'s slot in a mailbox
DGT_DEVICE long long ll_slot(const Exchange& ex, int parity, int src) {
  return (long long)(parity * kMaxRanks + src) * ex.stride * 2;
}

// one {payload, tag} pair as ONE relaxed system-scope 64-bit store (global_store_dwordx2 sc0 sc1: the
// mailbox is uncached memory, so it goes straight to the peer's HBM).  A naturally aligned 64-bit
// atomic access is single-copy atomic, so the pair can never be seen half-written.
DGT_DEVICE void ll_put_pair(unsigned* dst, float a, unsigned tag) {
  const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)tag << 32);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// push one LL line (two payload floats) into a peer's mailbox: two 64-bit atomic pair stores
DGT_DEVICE void ll_put(unsigned* dst, float a, float b, unsigned tag) {
  ll_put_pair(dst, a, tag);
  ll_put_pair(dst + 2, b, tag);
}

// one {payload, tag} pair from the local mailbox: a relaxed system-scope 64-bit load (sc0 sc1,
// never served from a stale cache line; many can be in flight, unlike volatile accesses)
DGT_DEVICE unsigned long long ll_get(const unsigned* src) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(src), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
DGT_DEVICE bool ll_ok(unsigned long long pair, unsigned tag) { return (unsigned)(pair >> 32) == tag; }
// LL3 line: three payload floats and the tag in ONE 16-byte store / load (global_store_dwordx4 /
// global_load_dwordx4).  Correctness needs an aligned 16-byte access to be single-copy atomic end
// to end over xGMI (one request to one 64-byte line on both ends, as RCCL's LL128 assumes for whole
// 128-byte lines).  No document available to this build guarantees that width: the guaranteed
// width is the 64-bit atomic that the LL2 format (ll_put_pair / ll_get) is built on.  So LL3 is
// used only after an in-kernel stress test of >= 1000 exchanges with payloads that expose any torn
// line (tiny_xch_stress, runtime/tiny_trainer.py) passed on this node; otherwise the trainer falls
// back to LL2, and a replica divergence at run time re-runs the epoch on RCCL.  The poll loop must
// re-issue the load every round (ll_fence_compiler() at the top of the loop).
DGT_DEVICE void ll3_put(unsigned* dst, float a, float b, float c, unsigned tag) {
  u32x4 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), tag};
  *reinterpret_cast<u32x4*>(dst) = v;
}
DGT_DEVICE u32x4 ll3_get(const unsigned* src) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
}

// Line formats of the fused kernel's exchange, as one interface: LN payload floats per 16-byte line.
//   LL3: {p0, p1, p2, tag}, one 16-byte store / load;  LL2: {p0, tag, p1, tag}, two 64-bit atomics each way.
template <int LN>
struct LLine;

template <>
struct LLine<3> {
  DGT_DEVICE static void put(unsigned* dst, float a, float b, float c, unsigned tag) { ll3_put(dst, a, b, c, tag); }
  DGT_DEVICE static u32x4 get(const unsigned* src) { return ll3_get(src); }
  DGT_DEVICE static bool ok(const u32x4& v, unsigned tag) { return v[3] == tag; }
  DGT_DEVICE static unsigned word(const u32x4& v, int i) { return v[i]; }
};

template <>
struct LLine<2> {
  DGT_DEVICE static void put(unsigned* dst, float a, float b, float, unsigned tag) { ll_put(dst, a, b, tag); }
  DGT_DEVICE static u32x4 get(const unsigned* src) {
    const unsigned long long lo = ll_get(src), hi = ll_get(src + 2);
    return u32x4{(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
  }
  DGT_DEVICE static bool ok(const u32x4& v, unsigned tag) { return v[1] == tag && v[3] == tag; }
  DGT_DEVICE static unsigned word(const u32x4& v, int i) { return v[2 * i]; }
};
DGT_DEVICE void ll_fence_compiler() { asm volatile("" ::: "memory"); }
DGT_DEVICE float ll_val(unsigned long long pair) { return __uint_as_float((unsigned)pair); }

// Full-row DPP permutations (quad_perm, row mirrors, row_newbcast) have a source lane for every
// lane, so bound_ctrl = true: no "old" value has to be materialised and an add can fold the move.
template <int CTRL>
DGT_DEVICE float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Sum over the 16 lanes of a DPP row (lanes sharing lane>>4), result in every lane of the row.
// DPP quad permutes + row (half-)mirrors: 4 v_add_f32_dpp, no LDS traffic (ds_bpermute costs an
// LDS round trip per step).  Every lane ends with the bitwise-same value.
DGT_DEVICE float wave_sum16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// Sum over each quad (lanes 4q..4q+3): enough for a row reduction when only lanes 0..3 of each DPP
// row can be non-zero (micro-batch <= 4); the result is in every lane of the quad.
DGT_DEVICE float quad_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  return v;
}

// Sum over the 4 rows of the wave (lane, lane^16, lane^32, lane^48) with the gfx950
// v_permlane16_swap / v_permlane32_swap half-exchanges.
DGT_DEVICE float wave_sum_groups(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

DGT_DEVICE float wave_sum(float v) {
  return wave_sum_groups(wave_sum16(v));
}

DGT_DEVICE unsigned long long realtime() { return __builtin_amdgcn_s_memrealtime(); }

// Wave-uniform read of memory that no kernel writes during the launch, through the constant
// address space: the compiler emits a scalar s_load (lgkmcnt) instead of a vector load, so
// waiting for it does not also wait for every older vector load (vmcnt retires in order).
template <typename T>
DGT_DEVICE T load_uniform(const T* p) {
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// torch.lerp for weight < 0.5 (what Adam's exp_avg.lerp_(grad, 1 - beta1) evaluates)
DGT_DEVICE float lerp_torch(float self, float end, float w) {
  return (fabsf(w) < 0.5f) ? fmaf(w, end - self, self) : end - (end - self) * (1.0f - w);
}

// One Adam/AdamW update of a single element, in the op order of torch's foreach Adam
// (torch/optim/adam.py _multi_tensor_adam: lerp_, mul_, addcmul_, sqrt, div_, add_, addcdiv_).
DGT_DEVICE float adam_update(float p, float g, float& m, float& v, const AdamHyper& h,
                             float step_size_neg, float bc2_sqrt) {
  if (h.weight_decay != 0.f) {
    if (h.adamw) p = p * h.decay;
    else g = fmaf(h.weight_decay, p, g);
  }
  m = lerp_torch(m, g, h.one_minus_beta1);
  v = v * h.beta2;
  v = v + h.one_minus_beta2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + h.eps;
  return p + step_size_neg * (m / denom);
}

// Latency-optimised variant for the persistent tiny-model kernel: hardware v_sqrt_f32 / v_rcp_f32
// (<= 1 ulp) instead of the IEEE division sequences, and the 1/sqrt(1 - beta2^t) factor as a
// multiply.  Differs from adam_update by a few ulp per step; exact-formula Adam stays in adam_flat.
DGT_DEVICE float adam_update_fast(float p, float g, float& m, float& v, const AdamHyper& h,
                                  float step_size_neg, float inv_bc2_sqrt) {
  if (h.weight_decay != 0.f) {
    if (h.adamw) p = p * h.decay;
    else g = fmaf(h.weight_decay, p, g);
  }
  m = fmaf(h.one_minus_beta1, g - m, m);  // torch.lerp, weight < 0.5 branch (host checks beta1 > 0.5)
  v = v * h.beta2;
  v = v + h.one_minus_beta2 * g * g;
  const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2_sqrt, h.eps);
  return fmaf(step_size_neg, m * __builtin_amdgcn_rcpf(denom), p);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// adam_update_fast on two elements: the non-transcendental math runs as packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth per instruction, same IEEE result
// per element as the scalar form); sqrt and rcp stay per element.
// WD = false: compiled without the weight-decay branches (the caller checked weight_decay == 0).
template <bool WD = true>
DGT_DEVICE f32x2 adam_update_fast2(f32x2 p, f32x2 g, f32x2& m, f32x2& v, const AdamHyper& h, float step_size_neg,
                                   float inv_bc2_sqrt) {
  if (WD && h.weight_decay != 0.f) {
    if (h.adamw) p = p * h.decay;
    else g = __builtin_elementwise_fma(f32x2(h.weight_decay), p, g);
  }
  m = __builtin_elementwise_fma(f32x2(h.one_minus_beta1), g - m, m);
  v = v * h.beta2;
  v = __builtin_elementwise_fma(f32x2(h.one_minus_beta2) * g, g, v);
  f32x2 r;
  r.x = __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(v.x), inv_bc2_sqrt, h.eps));
  r.y = __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(v.y), inv_bc2_sqrt, h.eps));
  return __builtin_elementwise_fma(f32x2(step_size_neg), m * r, p);
}

}  // namespace dgt
