// Fused training kernels for the reference model (SimpleNet: Linear(F,H) -> ReLU -> Linear(H,1),
// BCE-with-logits, Adam; reference train.py:26-36, 96, 107-115).
//
// Design (MI355X-first, not a translation of the reference's ~30 ATen/cuBLAS launches per step):
//   * ONE workgroup of H/16 waves trains the model; a launch runs many optimizer steps.
//   * Each wave OWNS 16 hidden units end to end: its rows of W1, its slice of b1 and W2, their
//     gradients and Adam moments — all in VGPRs for the whole launch.  The only cross-wave
//     dependency of a step is the sum of the per-wave partial logits, so a step has ONE workgroup
//     barrier (the partial-logit buffer is double-buffered by step parity).  The shared scalar b2
//     is updated redundantly (bit-identically) by every wave.
//   * Both GEMM-shaped products run on the matrix cores with exact-fp32 MFMA
//     (v_mfma_f32_16x16x4_f32).  The weight gradient is computed transposed,
//     dW1^T[k][j] = sum_b x[b][k] dh[b][j], with the MFMA's A rows permuted so that lane
//     (l&15, l>>4) receives dW1[j = l&15][k] for k = 16ct + (l>>4) + 4r ("slot" 4ct + r).  The
//     forward H^T = W1 . X^T walks its K dimension in exactly that slot order, so the lane that
//     receives a weight's gradient is the lane that owns the weight, updates it with Adam and
//     feeds it to the next forward MFMA — no LDS round trip for parameters or gradients.  The
//     stride-4 slot order packs the padding of the last K tile (K = F + 1 is rarely a multiple of
//     16) into whole slots that are skipped: F = 20 runs 6 of 8 slots (6 forward MFMAs, 8 Adam
//     updates per lane).  LDS only stages the two transposed operands of the weight gradient.
//   * b1 is folded into the GEMMs as an augmented weight column: x carries a constant 1 at feature
//     index F, so the forward MFMA adds the bias and the weight-gradient MFMA produces db1 in the
//     same registers as dW1.  W2 is owned by 4 lanes per DPP row and broadcast with row_newbcast.
//   * Row reductions use DPP (v_add_f32_dpp) and the gfx950 v_permlane{16,32}_swap exchanges,
//     never ds_bpermute.
//   * Minibatch rows are gathered from the device-resident dataset by sampler index; the next
//     step's rows are prefetched into registers while the current step computes (no per-step H2D,
//     no host sync: SURVEY K1/K2/K24).
//   * World size > 1: each wave pushes its gradient slice into every peer's IPC mailbox over
//     xGMI as LL lines (payload + sequence tag per 8 bytes, dgt_common.h), polls its own mailbox
//     until every peer's tags match and sums the contributions in rank order, so every rank
//     applies bit-identical updates.  This replaces DeepSpeed's flatten -> NCCL all_reduce ->
//     scale -> unflatten.
//   * Adam's bias corrections of every step of the launch are formed by the kernel itself, in its
//     prologue (one step per thread, in double with torch's formula, beta^t advanced by one
//     multiply per T steps), into a caller-owned workspace that the loop then reads one step ahead
//     through the scalar cache: no double math and no extra basic block in the loop (an LDS ring
//     refilled inside the loop measured 0.80-0.86 us/step against 0.75, profiles/r2_tiny_bias_ab.txt).
// Reference: train.py:26-36 (model), 96 (loss), 98-117 (loop), 113 (all-reduce), 114 (Adam step).
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

// Diagnostic build only (-DDGT_TINY_STAMPS): per-section s_memtime cycle sums of wave 0 / wave 1
// written to TinyTrainArgs::stamps.  The shipped kernel executes no stamp.
#ifdef DGT_TINY_STAMPS
#define DGT_STAMP(i)                                                                    \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long t_;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if ((i) > 0) st_acc[(i)-1] += t_ - st_last;                                         \
    st_last = t_;                                                                       \
  } while (0)
#else
#define DGT_STAMP(i) do {} while (0)
#endif

template <int F, int H>
struct TinyCfg {
  static constexpr int NW = H / 16;              // waves; wave w owns hidden units [16w, 16w+16)
  static constexpr int T = 64 * NW;              // threads
  static constexpr int NKT = (F + 1 + 15) / 16;  // 16-wide tiles of the augmented features [x, 1]
  static constexpr int NS = 4 * NKT;             // W1 slots per lane: (ct, r) -> k = 16ct + (l>>4) + 4r
  static constexpr int REM = F + 1 - 16 * (NKT - 1);      // live k in the last tile (1..16)
  static constexpr int NSL = 4 * (NKT - 1) + (REM + 3) / 4;  // slots holding any live k
  static constexpr int NSP = NSL + (NSL & 1);    // rounded up to packed-fp32 pairs (extra slot stays 0)
  // Exchange payload per lane.  DENSE: the last W1 slot is live only in lane row lq == 0 (REM % 4
  // == 1, e.g. F = 20), so its 48 dead lanes carry the W2 gradients (12 in place, 4 moved from
  // lanes 0-3 to 20-23) and b2 (lane 24): NSL floats per lane.  Otherwise the W1 slots, W2 and b2
  // padded to float4s.  ZeRO-1 (NPAYZ) always uses the plain layout: a lane's payload then holds
  // only the parameters whose Adam state lives in that lane (plus the replicated b2), so the rank
  // that owns the lane can update them.  A line carries LN = 3 (LL3) or 2 (LL2) payload floats.
  static constexpr bool DENSE = (REM & 3) == 1 && NSL >= 2;
  static constexpr int NPAY = DENSE ? NSL : NSL + 2;
  static constexpr int NPAYZ = NSL + 2;
  static constexpr int NLMAX = (NPAYZ + 1) / 2;  // the most lines per lane and peer (ZeRO-1, LL2)
  static constexpr int XCH = NW * NLMAX * 128;   // mailbox slot = 2*XCH words = NW*NLMAX lines of 1 KiB
  static constexpr int SX = NKT * 16 + 1;        // LDS row stride of the staged batch (+1: conflict-free)
  static constexpr int BM = 16;                  // max micro-batch (MFMA N of the forward)
  static constexpr int P = H * F + 2 * H + 1;    // global flat parameter count
  static constexpr int PP = (P + 3) / 4 * 4;
  static constexpr int G_B1 = H * F, G_W2 = H * F + H, G_B2 = H * F + 2 * H;
  static_assert(H % 16 == 0 && H >= 16 && H <= 256, "hidden must be a multiple of 16 in [16, 256]");
  static_assert((NW & (NW - 1)) == 0, "the loss ring rotates over a power-of-two number of waves");
  static_assert(F % 4 == 0 && F >= 4 && F <= 64, "n_features must be a multiple of 4 in [4, 64]");

  // feature index of W1 slot i (= 4ct + r) in lane-row lq
  static DGT_HOST_DEVICE int slot_k(int i, int lq) { return 16 * (i >> 2) + lq + 4 * (i & 3); }
  // global index of W1 slot i of lane (lr, lq) in wave w: W1 column k < F, b1 at k == F, else -1
  static DGT_HOST_DEVICE int slot_index(int w, int lr, int lq, int i) {
    const int k = slot_k(i, lq);
    if (k < F) return (16 * w + lr) * F + k;
    if (k == F) return G_B1 + 16 * w + lr;
    return -1;
  }
  // global index of the W2 element owned by lane (lr < 4, lq) of wave w; -1 if none
  static DGT_HOST_DEVICE int bw_index(int w, int lr, int lq) {
    return lr < 4 ? G_W2 + 16 * w + 4 * lq + lr : -1;
  }
};

template <int F, int H>
struct __attribute__((aligned(16))) WaveSmem {
  using C = TinyCfg<F, H>;
  float X[C::BM * C::SX];    // this step's minibatch, row-major (A operand of the weight gradient)
  float DH[C::BM * 17];      // dL/d(pre-activation) [batch][hidden] (B operand of the weight gradient)
};

template <int F, int H>
struct __attribute__((aligned(16))) TinySmem {
  using C = TinyCfg<F, H>;
  WaveSmem<F, H> w[C::NW];
  double loss[C::NW];        // per-wave deferred-loss totals, summed in wave order at the end
  float Z[2][C::NW * 16];    // per-wave partial logits, double-buffered by step parity
  int err;
};

// Register-resident per-lane training state of one wave.
template <int F, int H>
struct LaneState {
  using C = TinyCfg<F, H>;
  float w1[C::NSP], m1[C::NSP], v1[C::NSP];  // [W1 | b1][16w + (l&15)][slot_k(i, l>>4)]
  // {W2 element (lanes 0-3 of each DPP row), b2 (replicated in every lane)}: value, exp_avg,
  // exp_avg_sq as 2-vectors, the form the packed Adam update works on.  (Six scalar fields read
  // pairwise made the compiler combine overlapping vector loads of the struct, which kept it in
  // memory -- promoted to LDS -- and put an LDS round trip into every step.)
  f32x2 p2, m2, v2;
};

template <int F, int H>
DGT_DEVICE void load_state(LaneState<F, H>& st, const float* __restrict__ p, const float* __restrict__ m,
                           const float* __restrict__ v, int w, int lr, int lq) {
  using C = TinyCfg<F, H>;
#pragma unroll
  for (int i = 0; i < C::NSP; ++i) {
    const int gi = i < C::NSL ? C::slot_index(w, lr, lq, i) : -1;
    const bool ok = gi >= 0;
    st.w1[i] = ok ? p[gi] : 0.f;
    st.m1[i] = (ok && m) ? m[gi] : 0.f;
    st.v1[i] = (ok && v) ? v[gi] : 0.f;
  }
  const int bi = C::bw_index(w, lr, lq);
  st.p2 = f32x2{bi >= 0 ? p[bi] : 0.f, p[C::G_B2]};
  st.m2 = f32x2{(bi >= 0 && m) ? m[bi] : 0.f, m ? m[C::G_B2] : 0.f};
  st.v2 = f32x2{(bi >= 0 && v) ? v[bi] : 0.f, v ? v[C::G_B2] : 0.f};
}

// Minibatch values for the lane's row b = l&15: x[b][slot_k(i, l>>4)] and y[b].  A padding row
// (id < 0) loads row 0 instead of zeros: its dz is masked to 0 (valid = b < Bt), so its dh and
// its weight-gradient terms are exact zeros for any finite x, and its loss term is weighted 0 —
// no per-value selects in the step.
// Slot k's are stride-4 (k = 16ct + lq + 4r): scalar loads, issued a step ahead of their use.
template <int F, int H>
DGT_DEVICE void load_rows(const float* __restrict__ X, const float* __restrict__ Y, int id, int lq,
                          float (&x)[TinyCfg<F, H>::NSP], float& y) {
  using C = TinyCfg<F, H>;
  const float* row = X + (long long)(id >= 0 ? id : 0) * F;
#pragma unroll
  for (int i = 0; i < C::NSP; ++i) {
    const int k = C::slot_k(i, lq);
    float v = 0.f;
    if (i < C::NSL) {
      if (16 * (i >> 2) + 15 < F) v = row[k];  // full tile: every k is a feature
      else v = k < F ? row[k] : (k == F ? 1.f : 0.f);
    }
    x[i] = v;
  }
  y = Y[id >= 0 ? id : 0];
}

// Forward (MFMA) + bias + ReLU; publishes the wave's partial logits; stages x for the wgrad.
// H^T = W1 . X^T with K visited in slot order: A[i = l&15][kk = l>>4] = W1[j = l&15][slot_k],
// B[kk = l>>4][col = l&15] = x[b = l&15][slot_k]; D: col = batch row b = l&15,
// row = hidden 4*(l>>4) + r.
template <int F, int H>
DGT_DEVICE void wave_forward(const LaneState<F, H>& st, WaveSmem<F, H>& ws, float* Zbuf, int w, int lr, int lq,
                             const float (&x)[TinyCfg<F, H>::NSP], float (&h)[4], float (&w2v)[4]) {
  using C = TinyCfg<F, H>;
  // three independent accumulation chains: a dependent 16x16x4 f32 MFMA waits ~40 cycles for its
  // predecessor, so NSL = 6 slots run as 3 chains of 2 instead of 2 chains of 3
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < C::NSL; i += 3) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(st.w1[i], x[i], acc0, 0, 0, 0);
    if (i + 1 < C::NSL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(st.w1[i + 1], x[i + 1], acc1, 0, 0, 0);
    if (i + 2 < C::NSL) acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(st.w1[i + 2], x[i + 2], acc2, 0, 0, 0);
  }
  const f32x4 acc = (acc0 + acc1) + acc2;
  // stage this step's rows for the weight-gradient MFMA (row-major, conflict-free stride)
#pragma unroll
  for (int i = 0; i < C::NSL; ++i) ws.X[lr * C::SX + C::slot_k(i, lq)] = x[i];
  w2v[0] = dpp_mov<0x150>(st.p2.x);  // row_newbcast: W2[4lq + r] from lane r of the DPP row
  w2v[1] = dpp_mov<0x151>(st.p2.x);
  w2v[2] = dpp_mov<0x152>(st.p2.x);
  w2v[3] = dpp_mov<0x153>(st.p2.x);
  float pz = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    h[r] = fmaxf(acc[r], 0.f);  // bias already added by the augmented column
    pz = fmaf(h[r], w2v[r], pz);
  }
  pz = wave_sum_groups(pz);  // over the wave's 16 hidden units, for row b = l&15
  if (lq == 0) Zbuf[w * 16 + lr] = pz;
}

struct StepGrads {
  float bw, b2, loss, z;  // z: the lane's logit (row l&15), for the deferred loss
};

// BCE-with-logits of one row, torch's form (1-y)*z - log_sigmoid(z); 1 + e^-|z| is in [1, 2], so
// the raw v_log_f32 (log2) needs no denormal range fix-up.
DGT_DEVICE float bce_term(float z, float y) {
  const float e = __expf(-fabsf(z));
  const float l1pe = __builtin_amdgcn_logf(1.f + e) * 0.6931471805599453f;
  return (1.f - y) * z - (fminf(z, 0.f) - l1pe);
}

// After the barrier: logits, BCE, backward.  W1 gradients land in gw1 (slot layout).
// SMALLB: micro-batch <= 4 (the reference's 4 per rank): only lanes 0..3 of a DPP row carry
// batch rows, so row reductions are quad reductions and the weight gradient is one MFMA per tile.
template <int F, int H, bool WANT_LOSS, bool SMALLB>
DGT_DEVICE StepGrads wave_backward(const LaneState<F, H>& st, WaveSmem<F, H>& ws, const float* Zbuf, int lr,
                                   int lq, const float (&h)[4], const float (&w2v)[4], float y, int Bt,
                                   float invB, float (&gw1)[TinyCfg<F, H>::NSP]) {
  using C = TinyCfg<F, H>;
  float s = 0.f;
#pragma unroll
  for (int ww = 0; ww < C::NW; ++ww) s += Zbuf[ww * 16 + lr];
  const float z = s + st.p2.y;
  const bool valid = lr < Bt;
  // BCE-with-logits (torch: (1-y)*z - log_sigmoid(z)); d/dz = sigmoid(z) - y, times 1/B (mean)
  const float e = __expf(-fabsf(z));
  const float rinv = __builtin_amdgcn_rcpf(1.f + e);
  const float sig = (z >= 0.f) ? rinv : e * rinv;
  const float dz = valid ? (sig - y) * invB : 0.f;
  StepGrads out;
  out.loss = 0.f;
  out.z = z;
  if (WANT_LOSS) {
    const float term = valid ? bce_term(z, y) : 0.f;
    out.loss = (SMALLB ? quad_sum(term) : wave_sum16(term)) * invB;
  }
  float dw2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ws.DH[lr * 17 + 4 * lq + r] = (h[r] > 0.f) ? dz * w2v[r] : 0.f;
    dw2[r] = SMALLB ? quad_sum(dz * h[r]) : wave_sum16(dz * h[r]);  // over the batch rows: W2[4lq + r]
  }
  // b2 is replicated in every lane: a quad sum is broadcast from lane 0 of each row
  out.b2 = SMALLB ? dpp_mov<0x150>(quad_sum(dz)) : wave_sum16(dz);
  // the lane's own W2 element (lanes 0-3 of each row); db1 comes out of the wgrad MFMA
  float gbw = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) gbw = (lr == r) ? dw2[r] : gbw;
  out.bw = gbw;
  __builtin_amdgcn_wave_barrier();
  // weight gradient on MFMA, transposed: dW1^T[k][j] = sum_b x[b][k] dh[b][j]
  // A[i (l&15)][kk = b (l>>4)] = x[b][16ct + (i>>2) + 4(i&3)], B[kk = b][col = j (l&15)] = dh[b][j];
  // D row i = 4lq + r lands in lane (lr, lq): dW1[j = lr][k = 16ct + lq + 4r] = W1 slot 4ct + r.
  const int nks = SMALLB ? 1 : (Bt + 3) >> 2;
  const int arow = (lr >> 2) + 4 * (lr & 3);
#pragma unroll
  for (int ct = 0; ct < C::NKT; ++ct) {
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < (SMALLB ? 1 : C::BM / 4); ++ks) {
      if (SMALLB || ks < nks) {  // wave-uniform
        const int b = 4 * ks + lq;
        g = __builtin_amdgcn_mfma_f32_16x16x4f32(ws.X[b * C::SX + 16 * ct + arow], ws.DH[b * 17 + lr], g, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * ct + r < C::NSP) gw1[4 * ct + r] = (4 * ct + r < C::NSL) ? g[r] : 0.f;
  }
  __builtin_amdgcn_wave_barrier();
  return out;
}

// sum over the wave of the ring's (row, step) terms, each weighted 1/B of its step (0 = empty)
DGT_DEVICE float deferred_loss(float zs, float ys, float ibs) {
  return wave_sum(ibs != 0.f ? bce_term(zs, ys) * ibs : 0.f);
}

DGT_DEVICE int plan_at(const int* plan, int n_steps, int bmax, int step, int row) {
  return (step < n_steps && row < bmax) ? plan[(long long)step * bmax + row] : -1;
}

// Adam bias corrections of one optimizer step from beta1^t and beta2^t, in double as torch's
// non-capturable foreach Adam forms them on the host (adam.py: step_size = lr / (1 - beta1 ** step),
// bias_correction2_sqrt = sqrt(1 - beta2 ** step)), rounded to fp32 once.
DGT_DEVICE float2 adam_bias_pair(double b1p, double b2p, double lr) {
  return float2{(float)(-(lr / (1.0 - b1p))), (float)(1.0 / sqrt(1.0 - b2p))};
}

// beta^n by binary exponentiation (<= 2 log2(n) double roundings: ~1e-14 relative at n = 1e6, far
// below the fp32 rounding of the result; far less code and register pressure than ocml's pow).
DGT_DEVICE double ipow(double b, long long n) {
  double r = 1.0;
  while (n > 0) {
    if (n & 1) r *= b;
    b *= b;
    n >>= 1;
  }
  return r;
}

// Prologue: bc[2s], bc[2s+1] = bias corrections of launch step s (optimizer step step0 + s + 1) for
// every s < n_steps; thread t fills s = t, t + T, ... carrying beta^(step) in double.  The stores are
// drained before the prologue barrier, so the loop's scalar loads (K$ misses: the scalar cache
// holds none of these lines yet in this dispatch) read them from L2.
template <int T>
DGT_DEVICE void fill_bias_table(const TinyTrainArgs& a, int t) {
  if (t >= a.n_steps) return;
  double b1p = ipow(a.beta1, a.adam_step0 + t + 1), b2p = ipow(a.beta2, a.adam_step0 + t + 1);
  const double b1T = ipow(a.beta1, T), b2T = ipow(a.beta2, T);
  for (int s = t; s < a.n_steps; s += T) {
    const float2 bc = adam_bias_pair(b1p, b2p, a.lr);
    a.bc[2 * s] = bc.x;
    a.bc[2 * s + 1] = bc.y;
    b1p *= b1T;
    b2p *= b2T;
  }
}

// ------------------------------------------------------------------ gradient exchange (NP > 1)
// Lines of one lane's payload for one peer: line j of wave w, lane l sits at word
// (w * NL + j) * 256 + 4 l of the (parity, sender) slot, so every store or poll instruction of a
// wave moves 1 KiB contiguous.
template <int NPAY, int LN>
struct LinesOf {
  static constexpr int NL = (NPAY + LN - 1) / LN;
};

// Poll the given peers' lines of this lane in the local mailbox until all carry `tag` (or the
// timeout passes: late).  Every retry re-reads the peers still pending: one local round trip per
// poll, not one per line or per peer.  (Spinning on one line per peer first and reading the rest
// after measured slower: the extra round trip costs more than the smaller polls save,
// profiles/r2_xch_exchange_ab.txt.)  `pend` is a wave-uniform mask of the peers to wait for.
template <int NPAY, int NP, int LN>
DGT_DEVICE void poll_peers(const Exchange& ex, int parity, long long wofs, unsigned tag, unsigned pend,
                           u32x4 (&v)[NP][LinesOf<NPAY, LN>::NL], unsigned long long t0, bool& late) {
  constexpr int NL = LinesOf<NPAY, LN>::NL;
  do {
    ll_fence_compiler();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if ((pend >> p) & 1u) {
        const unsigned* src = ex.data[ex.rank] + ll_slot(ex, parity, p) + wofs;
#pragma unroll
        for (int j = 0; j < NL; ++j) v[p][j] = LLine<LN>::get(src + j * 256);
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if ((pend >> p) & 1u) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < NL; ++j) ok = ok && LLine<LN>::ok(v[p][j], tag);
        if (__all(ok)) pend &= ~(1u << p);
      }
    }
    if (pend && (long long)(realtime() - t0) > ex.timeout_ticks) late = true;
  } while (pend && !late);
}

template <int NPAY, int LN>
DGT_DEVICE float line_payload(const u32x4 (&v)[LinesOf<NPAY, LN>::NL], int k) {
  return __uint_as_float(LLine<LN>::word(v[k / LN], k % LN));
}

// every peer's payload of this lane, summed with the lane's own in rank order (the same order, so
// the same bits, on every rank)
template <int NPAY, int NP, int LN>
DGT_DEVICE void poll_sum_peers(const Exchange& ex, int parity, long long wofs, unsigned tag,
                               const float (&pay)[NPAY], float (&sum)[NPAY], unsigned long long t0, bool& late,
                               unsigned& rx) {
  u32x4 v[NP][LinesOf<NPAY, LN>::NL];
  unsigned pend = 0;
#pragma unroll
  for (int p = 0; p < NP; ++p)
    if (p < ex.world_size && p != ex.rank) pend |= 1u << p;
  poll_peers<NPAY, NP, LN>(ex, parity, wofs, tag, pend, v, t0, late);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (p >= ex.world_size) continue;
#pragma unroll
    for (int k = 0; k < NPAY; ++k) {
      const float r = line_payload<NPAY, LN>(v[p], k);
      if (p != ex.rank) rx ^= __float_as_uint(r);  // (ZeRO-1 checksum; dead code in the one-shot kernel)
      sum[k] += p == ex.rank ? pay[k] : r;
    }
  }
}

template <int NPAY>
DGT_DEVICE unsigned xor_words(const float (&pay)[NPAY]) {
  unsigned x = 0;
#pragma unroll
  for (int k = 0; k < NPAY; ++k) x ^= __float_as_uint(pay[k]);
  return x;
}

// push this lane's payload into one peer's mailbox as LN-payload lines (c0 replaces pay[0]: fault
// injection)
template <int NPAY, int LN>
DGT_DEVICE void push_payload(unsigned* dst, const float (&pay)[NPAY], float c0, unsigned tag) {
#pragma unroll
  for (int j = 0; j < LinesOf<NPAY, LN>::NL; ++j) {
    const int k = LN * j;
    LLine<LN>::put(dst + j * 256, j == 0 ? c0 : pay[k], k + 1 < NPAY ? pay[k + 1] : 0.f,
                   k + 2 < NPAY ? pay[k + 2] : 0.f, tag);
  }
}

// x * y rounded on its own: never contracted into a following add (an FMA there would round
// differently depending on how the compiler inlined the caller -- the one-shot and ZeRO-1 kernels
// must scale the summed gradients to the same bits)
DGT_DEVICE float mul_rounded(float x, float y) {
#pragma clang fp contract(off)
  return x * y;
}

// ZeRO-1 payload (plain layout, either direction): the lane's W1 slots, its W2 element and b2
template <int F, int H>
DGT_DEVICE void pack_plain(const float (&w1)[TinyCfg<F, H>::NSP], float bw, float b2,
                           float (&pay)[TinyCfg<F, H>::NPAYZ]) {
  using C = TinyCfg<F, H>;
#pragma unroll
  for (int i = 0; i < C::NSL; ++i) pay[i] = w1[i];
  pay[C::NSL] = bw;
  pay[C::NSL + 1] = b2;
}
template <int F, int H>
DGT_DEVICE void unpack_plain(const float (&pay)[TinyCfg<F, H>::NPAYZ], float scale,
                             float (&w1)[TinyCfg<F, H>::NSP], float& bw, float& b2) {
  using C = TinyCfg<F, H>;
#pragma unroll
  for (int i = 0; i < C::NSP; ++i) w1[i] = i < C::NSL ? mul_rounded(pay[i], scale) : 0.f;
  bw = mul_rounded(pay[C::NSL], scale);
  b2 = mul_rounded(pay[C::NSL + 1], scale);
}

// gradients of one lane -> exchange payload (see TinyCfg::DENSE for the dense layout)
template <int F, int H>
DGT_DEVICE void pack_payload(const float (&gw1)[TinyCfg<F, H>::NSP], float gbw, float gb2, int l,
                             float (&pay)[TinyCfg<F, H>::NPAY]) {
  using C = TinyCfg<F, H>;
  const int lr = l & 15, lq = l >> 4;
  if constexpr (C::DENSE) {
    const float moved = __shfl(gbw, (l + 44) & 63);  // lanes 20-23 take the W2 gradients of lanes 0-3
#pragma unroll
    for (int i = 0; i < C::NSL - 1; ++i) pay[i] = gw1[i];
    pay[C::NSL - 1] = lq == 0 ? gw1[C::NSL - 1]
                    : lr < 4  ? gbw
                    : (lq == 1 && lr < 8) ? moved
                    : l == 24 ? gb2
                              : 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < C::NPAY; ++i) pay[i] = i < C::NSL ? gw1[i] : (i == C::NSL ? gbw : (i == C::NSL + 1 ? gb2 : 0.f));
  }
}

// summed payload -> mean gradients of the lane (sum first, then the 1/world scale, as before the
// dense layout: the same bits)
template <int F, int H>
DGT_DEVICE void unpack_payload(const float (&sum)[TinyCfg<F, H>::NPAY], float inv_ws, int l,
                               float (&gw1)[TinyCfg<F, H>::NSP], float& gbw, float& gb2) {
  using C = TinyCfg<F, H>;
  const int lr = l & 15, lq = l >> 4;
  if constexpr (C::DENSE) {
    const float last = sum[C::NSL - 1];
    const float back = __shfl(last, (l + 20) & 63);  // lanes 0-3 take their W2 sums back from 20-23
#pragma unroll
    for (int i = 0; i < C::NSL - 1; ++i) gw1[i] = mul_rounded(sum[i], inv_ws);
    gw1[C::NSL - 1] = lq == 0 ? mul_rounded(last, inv_ws) : 0.f;
    gbw = lr < 4 ? mul_rounded(lq == 0 ? back : last, inv_ws) : 0.f;
    gb2 = mul_rounded(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(last), 24)), inv_ws);
  } else {
#pragma unroll
    for (int i = 0; i < C::NPAY; ++i) {
      const float v = mul_rounded(sum[i], inv_ws);
      if (i < C::NSL) gw1[i] = v;
      else if (i == C::NSL) gbw = v;
      else if (i == C::NSL + 1) gb2 = v;
    }
  }
}

// ------------------------------------------------------------------ persistent training kernel
// NP > 1: the exchange is compiled in (for up to NP ranks).  The single-rank kernel has no exchange
// branch, so backward and Adam form one basic block the scheduler can interleave.
// WD: weight decay != 0 (Adam's L2 term / AdamW's decay compiled in; the reference's Adam has none,
// and the per-pair uniform branches cost ~12 scalar branches per step).
// One Adam step of the lane's register-resident parameters: two per packed-fp32 update (W2 and b2
// form the last pair).
#ifdef DGT_TINY_SCALAR_ADAM
// A/B: the same update per element with single fp32 ops (the same operations in the same order,
// so the same bits as the packed form)
template <bool WD>
DGT_DEVICE float adam_update_fast1(float p, float g, float& m, float& v, const AdamHyper& h, float step_size_neg,
                                   float inv_bc2_sqrt) {
  if (WD && h.weight_decay != 0.f) {
    if (h.adamw) p = p * h.decay;
    else g = fmaf(h.weight_decay, p, g);
  }
  m = fmaf(h.one_minus_beta1, g - m, m);
  v = v * h.beta2;
  v = fmaf(h.one_minus_beta2 * g, g, v);
  const float r = __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2_sqrt, h.eps));
  return fmaf(step_size_neg, m * r, p);
}
#endif

template <int F, int H, bool WD>
DGT_DEVICE void adam_lane(LaneState<F, H>& st, const float (&gw1)[TinyCfg<F, H>::NSP], float gbw, float gb2,
                          const AdamHyper& hp, float step_size_neg, float inv_bc2_sqrt) {
  using C = TinyCfg<F, H>;
#ifdef DGT_TINY_SCALAR_ADAM
#pragma unroll
  for (int i = 0; i < C::NSP; ++i)
    st.w1[i] = adam_update_fast1<WD>(st.w1[i], gw1[i], st.m1[i], st.v1[i], hp, step_size_neg, inv_bc2_sqrt);
  float m2x = st.m2.x, v2x = st.v2.x, m2y = st.m2.y, v2y = st.v2.y;
  const float px = adam_update_fast1<WD>(st.p2.x, gbw, m2x, v2x, hp, step_size_neg, inv_bc2_sqrt);
  const float py = adam_update_fast1<WD>(st.p2.y, gb2, m2y, v2y, hp, step_size_neg, inv_bc2_sqrt);
  st.p2 = f32x2{px, py};
  st.m2 = f32x2{m2x, m2y};
  st.v2 = f32x2{v2x, v2y};
  return;
#endif
#pragma unroll
  for (int i = 0; i < C::NSP; i += 2) {
    f32x2 m = {st.m1[i], st.m1[i + 1]}, v = {st.v1[i], st.v1[i + 1]};
    const f32x2 pn = adam_update_fast2<WD>(f32x2{st.w1[i], st.w1[i + 1]}, f32x2{gw1[i], gw1[i + 1]}, m, v, hp,
                                           step_size_neg, inv_bc2_sqrt);
    st.w1[i] = pn.x;
    st.w1[i + 1] = pn.y;
    st.m1[i] = m.x;
    st.m1[i + 1] = m.y;
    st.v1[i] = v.x;
    st.v1[i + 1] = v.y;
  }
  f32x2 m = st.m2, v = st.v2;
  st.p2 = adam_update_fast2<WD>(st.p2, f32x2{gbw, gb2}, m, v, hp, step_size_neg, inv_bc2_sqrt);
  st.m2 = m;
  st.v2 = v;
}

template <int F, int H, bool SMALLB, int NP, bool WD, int LN, bool Z>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_mlp_train_kernel(TinyTrainArgs a) {
  using C = TinyCfg<F, H>;
  // NP: ranks the exchange is compiled for (1 = none; else the world size rounded up to 2, 4 or 8):
  // the poll registers scale with it, so 2- and 4-rank jobs do not carry the 8-rank register set.
  // LN: exchange line format (3 = LL3, 2 = LL2; dgt_common.h).  Z: ZeRO-1 exchange (gradients
  // reduce-scattered to lane owners, the owner's Adam, parameters all-gathered) instead of the
  // one-shot all-to-all of gradients.
  constexpr bool XCH = NP > 1;
  static_assert(!Z || XCH, "the ZeRO-1 exchange needs ranks to exchange with");
  __shared__ TinySmem<F, H> sm;
  const int t = threadIdx.x, l = t & 63, lr = l & 15, lq = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: scalar branches on w
  const Exchange& ex = a.ex;
  WaveSmem<F, H>& ws = sm.w[w];
#ifdef DGT_TINY_STAMPS
  const unsigned long long rt_entry = realtime();
#endif

  if (a.bmax > (SMALLB ? 4 : C::BM) || a.bmax < 1 || (ex.world_size > 1) != XCH || ex.world_size > NP ||
      (ex.world_size > 1 && (ex.stride < C::XCH || (ex.stride & 3) || ex.line != LN)) || (ex.zero1 != 0) != Z) {
    if (t == 0) *a.status = kBadShape;
    return;
  }

  // ---- prologue: state -> registers, LDS zeroed, batch 0 loaded, indices of steps 1 and 2 in flight
  LaneState<F, H> st;
  load_state<F, H>(st, a.params, a.exp_avg, a.exp_avg_sq, w, lr, lq);
  for (int i = l; i < C::BM * C::SX; i += 64) ws.X[i] = 0.f;
  for (int i = l; i < C::BM * 17; i += 64) ws.DH[i] = 0.f;
  if (t == 0) sm.err = 0;
  float x[C::NSP], y, xn[C::NSP], yn;
  load_rows<F, H>(a.X, a.Y, plan_at(a.plan, a.n_steps, a.bmax, 0, lr), lq, x, y);
  int idx_next = plan_at(a.plan, a.n_steps, a.bmax, 1, lr);
  int idx_next2 = plan_at(a.plan, a.n_steps, a.bmax, 2, lr);
  fill_bias_table<C::T>(a, t);
  __builtin_amdgcn_s_waitcnt(0);  // the table's stores have reached L2 before any wave reads it
#ifdef DGT_TINY_STAMPS
  const unsigned long long rt_loaded = realtime();
#endif
  __syncthreads();
#ifdef DGT_TINY_STAMPS
  const unsigned long long rt_loop = realtime();
#endif

  double loss_total = 0.0;
  unsigned xs_ag = 0, xs_rs = 0;  // ZeRO-1 transfer checksums (Exchange::xsum)
  float zs = 0.f, ys = 0.f, ibs = 0.f;  // deferred-loss ring (wave 0)
  const float inv_ws = 1.0f / (float)ex.world_size;
  // Adam bias corrections of the current step, loaded a step ahead: the scalar load of step s+1's
  // pair is in flight during step s (a K$ miss every 8th step otherwise stalled the Adam section)
  float bc_ss = load_uniform(a.bc), bc_ib = load_uniform(a.bc + 1);
#ifdef DGT_TINY_STAMPS
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_last = 0;
#endif
  for (int s = 0; s < a.n_steps; ++s) {
    DGT_STAMP(0);
    const int Bt = load_uniform(a.counts + s);
    const float invB = __builtin_amdgcn_rcpf((float)Bt);
    const float bc_ss_next = load_uniform(a.bc + 2 * s + 2), bc_ib_next = load_uniform(a.bc + 2 * s + 3);
    // prefetch step s+1 rows into registers; consumed by the next step's forward
    load_rows<F, H>(a.X, a.Y, idx_next, lq, xn, yn);
    // sampler index of step s+3, issued now so the end-of-step rotation never waits on it
    const int idx_next3 = plan_at(a.plan, a.n_steps, a.bmax, s + 3, lr);

    float h[4], w2v[4];
    float* Zb = sm.Z[s & 1];
    wave_forward<F, H>(st, ws, Zb, w, lr, lq, x, h, w2v);
    DGT_STAMP(1);
    __syncthreads();  // the step's only workgroup barrier: all partial logits published
    DGT_STAMP(2);
    float gw1[C::NSP];
    const StepGrads sg = wave_backward<F, H, false, SMALLB>(st, ws, Zb, lr, lq, h, w2v, y, Bt, invB, gw1);
    // only the exchange can fail, so the single-rank loop reads no flag; with the exchange the flag
    // is read AFTER the backward (which changes no state), so its LDS round trip overlaps the
    // backward's instead of sitting between the barrier and the partial-logit reads
    if constexpr (XCH) {
      if (sm.err) break;
    }
    float gbw = sg.bw, gb2 = sg.b2;
    // Deferred loss (reporting only, off the per-step critical path): steps 4j..4j+3 belong to
    // wave j % NW, whose lane row lq keeps step s's logits when s % 4 == lq; at the block's last
    // step one wave-wide reduction folds the 4 steps in.  Rotating the owner spreads the work
    // evenly, so no wave is the last to reach the barrier every step.  (Logging the logits to
    // memory for a follow-up kernel measured slower: the store joins the in-order vmcnt queue the
    // row prefetch waits on.)
    if (w == ((s >> 2) & (C::NW - 1))) {
      if (lq == (s & 3)) {
        zs = sg.z;
        ys = y;
        ibs = lr < Bt ? invB : 0.f;
      }
      if ((s & 3) == 3) {
        loss_total += (double)deferred_loss(zs, ys, ibs);
        ibs = 0.f;
      }
    }
    DGT_STAMP(3);

    // Adam bias corrections of this step from the table (wave-uniform, prefetched)
    const float step_size_neg = bc_ss, inv_bc2_sqrt = bc_ib;
    bc_ss = bc_ss_next;
    bc_ib = bc_ib_next;
    if constexpr (XCH) {
      // ---- LL exchange of this wave's gradients over xGMI.
      // Every rank maps lanes to parameters identically, so the mailbox is lane-linear: lane l of
      // wave w packs its payload into NL lines at [w][line][l]; every store instruction writes
      // 1 KiB contiguous into a peer, every poll reads the local mailbox.  The wave's
      // memory-instruction throughput on uncached memory (~11 ns per 1 KiB instruction and CU,
      // csrc/diag/store_lat.hip), not the round trip, bounds the exchange at 4-8 ranks: hence the
      // dense one-shot payload (2 LL3 lines per peer for F = 20).
      const long long seq = ex.seq_base + s;
      const int parity = (int)(seq & 1);
      const unsigned tag = (unsigned)(seq + 1);
      constexpr int NPX = Z ? C::NPAYZ : C::NPAY;
      constexpr int NL = LinesOf<NPX, LN>::NL;
      const long long wofs = (long long)w * NL * 256 + l * 4;
      const long long mine = ll_slot(ex, parity, ex.rank) + wofs;
      float pay[NPX], sum[NPX];
#pragma unroll
      for (int k = 0; k < NPX; ++k) sum[k] = 0.f;
      const unsigned long long t0 = realtime();
      bool late = false;
      static_assert(NP <= kMaxRanks, "at most kMaxRanks ranks per exchange");
      // fault injection (--fail-at R:S:corrupt): one payload to rank + 1 is off by 1.0 at step S, so
      // the replicas diverge and the per-epoch replica check must catch it (scalar test otherwise)
      const int victim = (ex.corrupt_step == a.adam_step0 + s + 1 && w == 0) ? (ex.rank + 1) % ex.world_size : -1;
      if constexpr (!Z) {
        // ---- one-shot: push to every peer, poll every peer, sum in rank order, everybody updates
        pack_payload<F, H>(gw1, gbw, gb2, l, pay);
        for (int p = 0; p < ex.world_size; ++p) {
          if (p == ex.rank) continue;
          push_payload<NPX, LN>(ex.data[p] + mine, pay, (p == victim && l == 0) ? pay[0] + 1.0f : pay[0], tag);
        }
        // every peer's lines in flight at once: ONE local round trip per poll whatever the world
        // size (polling in batches of 4 peers cost a second round trip per step at 5-8 ranks)
        unsigned rx_unused = 0;
        poll_sum_peers<NPX, NP, LN>(ex, parity, wofs, tag, pay, sum, t0, late, rx_unused);
        if (late) sm.err = 1;
        unpack_payload<F, H>(sum, inv_ws, l, gw1, gbw, gb2);
        adam_lane<F, H, WD>(st, gw1, gbw, gb2, a.hp, step_size_neg, inv_bc2_sqrt);
      } else {
        // ---- ZeRO-1: lane l (its W1 slots, W2 element, Adam moments) is owned by rank l % P.
        // Reduce-scatter: every lane sends its gradient payload to its owner only; the owner sums
        // all ranks in rank order (the same order, so the same bits, as the one-shot), applies Adam
        // to the state only it keeps current, and all-gathers the updated PARAMETERS to every
        // peer.  Both phases land in the receiver's [parity][sender] slot at lane l: reduce-scatter
        // traffic on the lanes the receiver owns, all-gather traffic on the lanes the sender owns,
        // so one mailbox holds both.  Non-owner lanes never touch their moments: each rank's
        // optimizer state is current only for its 1/P of the lanes (its checkpoint shard).
        pack_plain<F, H>(gw1, gbw, gb2, pay);
        const int own = l % ex.world_size;
        if (own != ex.rank) {
          push_payload<NPX, LN>(ex.data[own] + mine, pay, pay[0], tag);
          xs_rs ^= xor_words<NPX>(pay);
        }
        // owner lanes FIRST, in program order: a lane waiting for an all-gather must never run
        // ahead of its own wave's owner lanes, which other ranks wait on
        if (own == ex.rank) {
          poll_sum_peers<NPX, NP, LN>(ex, parity, wofs, tag, pay, sum, t0, late, xs_rs);
          if (!late) {
            unpack_plain<F, H>(sum, inv_ws, gw1, gbw, gb2);
            adam_lane<F, H, WD>(st, gw1, gbw, gb2, a.hp, step_size_neg, inv_bc2_sqrt);
            pack_plain<F, H>(st.w1, st.p2.x, st.p2.y, pay);
            xs_ag ^= xor_words<NPX>(pay);  // what every peer must receive
            for (int p = 0; p < ex.world_size; ++p) {
              if (p == ex.rank) continue;
              push_payload<NPX, LN>(ex.data[p] + mine, pay, (p == victim && l == ex.rank) ? pay[0] + 1.0f : pay[0],
                                    tag);
            }
          }
        }
        if (own != ex.rank) {
          const unsigned* src = ex.data[ex.rank] + ll_slot(ex, parity, own) + wofs;
          u32x4 v[NL];
          bool ready;
          do {
            ll_fence_compiler();
            ready = true;
#pragma unroll
            for (int j = 0; j < NL; ++j) v[j] = LLine<LN>::get(src + j * 256);
#pragma unroll
            for (int j = 0; j < NL; ++j) ready = ready && LLine<LN>::ok(v[j], tag);
            if (!ready && (long long)(realtime() - t0) > ex.timeout_ticks) late = true;
          } while (!ready && !late);
#pragma unroll
          for (int k = 0; k < NPX; ++k) sum[k] = line_payload<NPX, LN>(v, k);
          xs_ag ^= xor_words<NPX>(sum);
          float bw, b2;
          unpack_plain<F, H>(sum, 1.0f, st.w1, bw, b2);
          st.p2 = f32x2{bw, b2};
        }
        if (late) sm.err = 1;
      }
    } else {
      adam_lane<F, H, WD>(st, gw1, gbw, gb2, a.hp, step_size_neg, inv_bc2_sqrt);
    }
    DGT_STAMP(4);
    // rotate the prefetch pipeline
#pragma unroll
    for (int i = 0; i < C::NSP; ++i) x[i] = xn[i];
    y = yn;
    idx_next = idx_next2;
    idx_next2 = idx_next3;
    DGT_STAMP(5);
  }
  if constexpr (Z) {
    if (ex.xsum) {  // one thread per word pair, XOR-accumulated across the epoch's launches
      ex.xsum[2 * t] ^= xs_ag;
      ex.xsum[2 * t + 1] ^= xs_rs;
    }
  }
  loss_total += (double)deferred_loss(zs, ys, ibs);  // the partial last ring (empty rings add 0)
  if (l == 0) sm.loss[w] = loss_total;
#ifdef DGT_TINY_STAMPS
  if (a.stamps && l == 0 && w < 2)
    for (int i = 0; i < 5; ++i) a.stamps[w * 8 + i] = st_acc[i];
  const unsigned long long rt_loop_end = realtime();
#endif

  // ---- epilogue: state back to HBM (b2 belongs to wave 0, lane 0)
#pragma unroll
  for (int i = 0; i < C::NSL; ++i) {
    const int gi = C::slot_index(w, lr, lq, i);
    if (gi >= 0) {
      a.params[gi] = st.w1[i];
      a.exp_avg[gi] = st.m1[i];
      a.exp_avg_sq[gi] = st.v1[i];
    }
  }
  const int bi = C::bw_index(w, lr, lq);
  if (bi >= 0) {
    a.params[bi] = st.p2.x;
    a.exp_avg[bi] = st.m2.x;
    a.exp_avg_sq[bi] = st.v2.x;
  }
  // b2 is replicated in every lane and stored once: under ZeRO-1 a lane's moments are current only
  // on the rank that owns it, so each rank stores b2's state from a lane it owns (lane = rank of
  // wave 0); the next launch loads it into every lane, and the owners carry on from current moments
  if (t == (Z ? ex.rank : 0)) {
    a.params[C::G_B2] = st.p2.y;
    a.exp_avg[C::G_B2] = st.m2.y;
    a.exp_avg_sq[C::G_B2] = st.v2.y;
  }
  __syncthreads();
  if (t == 0) {
    double total = 0.0;
#pragma unroll
    for (int i = 0; i < C::NW; ++i) total += sm.loss[i];
    // no-return atomic add: the epilogue does not wait a load round trip for the old value (one
    // writer per launch, so the sum is the same as a read-modify-write)
    __hip_atomic_fetch_add(a.loss_acc, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *a.status = sm.err ? kTimeout : kOk;
  }
#ifdef DGT_TINY_STAMPS
  // phase split in s_memrealtime ticks (10 ns) of wave 0: [5] entry -> operands landed,
  // [6] -> past the prologue barrier, [7] loop, [13] epilogue incl. its stores' completion
  __builtin_amdgcn_s_waitcnt(0);
  if (a.stamps && t == 0) {
    a.stamps[5] = rt_loaded - rt_entry;
    a.stamps[6] = rt_loop - rt_loaded;
    a.stamps[7] = rt_loop_end - rt_loop;
    a.stamps[13] = realtime() - rt_loop_end;
  }
#endif
}

// One step's gradient only (the RCCL path: grad -> all_reduce -> adam_flat).
template <int F, int H>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_mlp_grad_kernel(TinyGradArgs a) {
  using C = TinyCfg<F, H>;
  __shared__ TinySmem<F, H> sm;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, lr = l & 15, lq = l >> 4;
  WaveSmem<F, H>& ws = sm.w[w];
  LaneState<F, H> st;
  load_state<F, H>(st, a.params, nullptr, nullptr, w, lr, lq);
  for (int i = l; i < C::BM * C::SX; i += 64) ws.X[i] = 0.f;
  for (int i = l; i < C::BM * 17; i += 64) ws.DH[i] = 0.f;
  float x[C::NSP], y;
  const int id = (lr < a.bmax) ? a.plan[(long long)a.step * a.bmax + lr] : -1;
  load_rows<F, H>(a.X, a.Y, id, lq, x, y);
  const int Bt = a.counts[a.step];
  const float invB = __builtin_amdgcn_rcpf((float)Bt);
  float h[4], w2v[4], gw1[C::NSP];
  __builtin_amdgcn_wave_barrier();
  wave_forward<F, H>(st, ws, sm.Z[0], w, lr, lq, x, h, w2v);
  __syncthreads();
  const StepGrads sg = wave_backward<F, H, true, false>(st, ws, sm.Z[0], lr, lq, h, w2v, y, Bt, invB, gw1);
#pragma unroll
  for (int i = 0; i < C::NSL; ++i) {
    const int gi = C::slot_index(w, lr, lq, i);
    if (gi >= 0) a.grad[gi] = gw1[i];
  }
  const int bi = C::bw_index(w, lr, lq);
  if (bi >= 0) a.grad[bi] = sg.bw;
  if (t == 0) {
    a.grad[C::G_B2] = sg.b2;
    *a.loss_acc += (double)sg.loss;
  }
}

// ------------------------------------------------------------------ exchange stress test
// n_steps exchanges through the training kernel's own mailbox layout, line format and push / poll
// code, every lane of every wave to every peer, with payloads that name (sequence, sender, wave,
// lane, slot).  A line observed with the current tag but any word from an earlier exchange -- a
// torn line -- fails the word comparison, as does a lost or misplaced write.  Bad words are counted
// into *errors (one vector atomic per lane at the end); a spin past the timeout sets *status.
// Payload words are normal floats in +-[1, 2) carrying 24 hashed bits.
DGT_DEVICE unsigned stress_word(long long seq, int src, int w, int l, int k) {
  unsigned x = (unsigned)seq * 0x9E3779B1u ^ (unsigned)(seq >> 32) * 0x85EBCA77u;
  x ^= (unsigned)src * 0x27D4EB2Fu + (unsigned)w * 0x165667B1u + (unsigned)l * 0xC2B2AE3Du + (unsigned)k * 0x61C88647u;
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 12;
  return (x & 0x807FFFFFu) | 0x3F800000u;
}

template <int F, int H, int NP, int LN>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_xch_stress_kernel(Exchange ex, int n_steps, int* status,
                                                                            int* errors) {
  using C = TinyCfg<F, H>;
  constexpr int NPX = C::NPAYZ, NL = LinesOf<NPX, LN>::NL;  // the longest payload of the training kernel
  const int t = threadIdx.x, l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  if (ex.world_size < 2 || ex.world_size > NP || ex.stride < C::XCH || (ex.stride & 3) || ex.line != LN) {
    if (t == 0) *status = kBadShape;
    return;
  }
  int bad = 0;
  bool late = false;
  unsigned all = 0;
#pragma unroll
  for (int p = 0; p < NP; ++p)
    if (p < ex.world_size && p != ex.rank) all |= 1u << p;
  for (int s = 0; s < n_steps && !late; ++s) {
    const long long seq = ex.seq_base + s;
    const int parity = (int)(seq & 1);
    const unsigned tag = (unsigned)(seq + 1);
    const long long wofs = (long long)w * NL * 256 + l * 4;
    const long long mine = ll_slot(ex, parity, ex.rank) + wofs;
    float pay[NPX];
#pragma unroll
    for (int k = 0; k < NPX; ++k) pay[k] = __uint_as_float(stress_word(seq, ex.rank, w, l, k));
    for (int p = 0; p < ex.world_size; ++p)
      if (p != ex.rank) push_payload<NPX, LN>(ex.data[p] + mine, pay, pay[0], tag);
    u32x4 v[NP][NL];
    poll_peers<NPX, NP, LN>(ex, parity, wofs, tag, all, v, realtime(), late);
    if (!late) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        if (!((all >> p) & 1u)) continue;
#pragma unroll
        for (int k = 0; k < NPX; ++k) bad += LLine<LN>::word(v[p][k / LN], k % LN) != stress_word(seq, p, w, l, k);
      }
    }
  }
  if (bad) atomicAdd(errors, bad);
  if (late) atomicExch(status, (int)kTimeout);
}

// ------------------------------------------------------------------ dispatch
#define DGT_TINY_SHAPES(X) X(20, 64) X(32, 64) X(20, 128) X(8, 16)

hipError_t tiny_xch_stress(int f, int h, const Exchange& ex, int n_steps, int* status, int* errors,
                           hipStream_t stream) {
  if (n_steps < 1 || ex.world_size < 2 || ex.world_size > kMaxRanks || (ex.line != 2 && ex.line != 3))
    return hipErrorInvalidValue;
#define DGT_XS_NP(F_, H_, NP_)                                                                           \
  do {                                                                                                   \
    if (ex.line == 2)                                                                                    \
      hipLaunchKernelGGL((tiny_xch_stress_kernel<F_, H_, NP_, 2>), dim3(1), blk, 0, stream, ex, n_steps, status, errors); \
    else                                                                                                 \
      hipLaunchKernelGGL((tiny_xch_stress_kernel<F_, H_, NP_, 3>), dim3(1), blk, 0, stream, ex, n_steps, status, errors); \
  } while (0)
#define X_(F_, H_)                                                  \
  if (f == F_ && h == H_) {                                         \
    const dim3 blk(TinyCfg<F_, H_>::T);                             \
    if (ex.world_size <= 2) DGT_XS_NP(F_, H_, 2);                   \
    else if (ex.world_size <= 4) DGT_XS_NP(F_, H_, 4);              \
    else DGT_XS_NP(F_, H_, 8);                                      \
    return hipGetLastError();                                       \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
#undef DGT_XS_NP
  return hipErrorInvalidValue;
}

bool tiny_mlp_supported(int f, int h) {
#define X_(F_, H_) if (f == F_ && h == H_) return true;
  DGT_TINY_SHAPES(X_)
#undef X_
  return false;
}

int tiny_mlp_padded_numel(int f, int h) { return (h * f + 2 * h + 1 + 3) / 4 * 4; }

int tiny_mlp_exchange_floats(int f, int h) {
#define X_(F_, H_) if (f == F_ && h == H_) return TinyCfg<F_, H_>::XCH;
  DGT_TINY_SHAPES(X_)
#undef X_
  return 0;
}

// The kernel instantiation a launch of shape (f, h) with these arguments runs, and its block size;
// nullptr if none (bad shape or line format).  Shared by the per-call launch and the prepared
// launcher (bindings.cpp), which resolves it once.
const void* tiny_mlp_train_symbol(int f, int h, const TinyTrainArgs& a, int* threads) {
  if (!a.bc) return nullptr;
  const bool wd = a.hp.weight_decay != 0.f;
  const bool ll2 = a.ex.line == 2, z = a.ex.zero1 != 0;
  if (a.ex.world_size > 1 && a.ex.line != 2 && a.ex.line != 3) return nullptr;
#define DGT_TINY_LAUNCH_K(F_, H_, SB, NP_, LN_, Z_)                                                   \
  do {                                                                                             \
    if (wd) return reinterpret_cast<const void*>(&tiny_mlp_train_kernel<F_, H_, SB, NP_, true, LN_, Z_>); \
    return reinterpret_cast<const void*>(&tiny_mlp_train_kernel<F_, H_, SB, NP_, false, LN_, Z_>);      \
  } while (0)
// exchange kernels: line format x ZeRO-1, for 2, 4 or 8 compiled ranks
#define DGT_TINY_LAUNCH_NP(F_, H_, SB, NP_)                                                        \
  do {                                                                                             \
    if (ll2 && z) DGT_TINY_LAUNCH_K(F_, H_, SB, NP_, 2, true);                                     \
    else if (ll2) DGT_TINY_LAUNCH_K(F_, H_, SB, NP_, 2, false);                                    \
    else if (z) DGT_TINY_LAUNCH_K(F_, H_, SB, NP_, 3, true);                                       \
    else DGT_TINY_LAUNCH_K(F_, H_, SB, NP_, 3, false);                                             \
  } while (0)
#define DGT_TINY_LAUNCH(F_, H_, SB, XC)                                                            \
  do {                                                                                             \
    if (!(XC)) DGT_TINY_LAUNCH_K(F_, H_, SB, 1, 3, false);                                         \
    else if (a.ex.world_size <= 2) DGT_TINY_LAUNCH_NP(F_, H_, SB, 2);                              \
    else if (a.ex.world_size <= 4) DGT_TINY_LAUNCH_NP(F_, H_, SB, 4);                              \
    else DGT_TINY_LAUNCH_NP(F_, H_, SB, 8);                                                        \
  } while (0)
#define X_(F_, H_)                                                                            \
  if (f == F_ && h == H_) {                                                                   \
    *threads = TinyCfg<F_, H_>::T;                                                            \
    const bool xch = a.ex.world_size > 1;                                                     \
    if (a.bmax <= 4 && !xch) DGT_TINY_LAUNCH(F_, H_, true, false);                            \
    else if (a.bmax <= 4) DGT_TINY_LAUNCH(F_, H_, true, true);                                \
    else if (!xch) DGT_TINY_LAUNCH(F_, H_, false, false);                                     \
    else DGT_TINY_LAUNCH(F_, H_, false, true);                                                \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
#undef DGT_TINY_LAUNCH
#undef DGT_TINY_LAUNCH_NP
#undef DGT_TINY_LAUNCH_K
  return nullptr;
}

hipError_t tiny_mlp_train(int f, int h, const TinyTrainArgs& a, hipStream_t stream) {
  int threads = 0;
  const void* k = tiny_mlp_train_symbol(f, h, a, &threads);
  if (!k) return hipErrorInvalidValue;
  void* args[] = {const_cast<TinyTrainArgs*>(&a)};
  return hipLaunchKernel(k, dim3(1), dim3(threads), args, 0, stream);
}

hipError_t tiny_mlp_grad(int f, int h, const TinyGradArgs& a, hipStream_t stream) {
#define X_(F_, H_)                                                                           \
  if (f == F_ && h == H_) {                                                                  \
    hipLaunchKernelGGL((tiny_mlp_grad_kernel<F_, H_>), dim3(1), dim3(TinyCfg<F_, H_>::T), 0, \
                       stream, a);                                                           \
    return hipGetLastError();                                                                \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
  return hipErrorInvalidValue;
}

}  // namespace dgt
