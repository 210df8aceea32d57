// Fused training kernels for the reference model (SimpleNet: Linear(F,H) -> ReLU -> Linear(H,1),
// BCE-with-logits, Adam; reference train.py:26-36, 96, 107-115).
//
// Design (MI355X-first, not a translation of the reference's ~30 ATen/cuBLAS launches per step):
//   * ONE workgroup of 4*H threads (H/16 waves) owns the whole model.  Parameters and gradients
//     live in LDS for the entire launch; Adam moments live in registers (each thread owns fixed
//     float4 chunks of the flat parameter vector).  A launch runs many optimizer steps.
//   * Both GEMM-shaped products run on the matrix cores with exact-fp32 MFMA
//     (v_mfma_f32_16x16x4_f32): the forward x.W1^T (M = batch, N = hidden, K = features) and the
//     weight gradient dh^T.x (M = hidden, N = features, K = batch).  Each wave owns one 16-wide
//     hidden tile, so the hidden tile is the MFMA N (fwd) / M (wgrad) dimension.  Operands are
//     staged through LDS with padded strides (no 16-way bank conflicts on the strided reads).
//   * The minibatch rows are gathered from the device-resident dataset by sampler index, with
//     the next step's rows prefetched into registers while the current step computes
//     (no per-step H2D copy, no host sync: SURVEY K1/K2/K24).
//   * World size > 1: after the local gradient is complete, the workgroup pushes it into every
//     peer's IPC mailbox over xGMI, raises a per-peer sequence flag (system-scope release), waits
//     for its own flags, and sums the world_size contributions in rank order, so every rank
//     applies bit-identical updates.  This replaces DeepSpeed's flatten -> NCCL all_reduce ->
//     scale -> unflatten with one latency-bound exchange inside the kernel.
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

template <int F, int H>
struct TinyCfg {
  static constexpr int NW = H / 16;              // waves; wave w owns hidden units [16w, 16w+16)
  static constexpr int T = 64 * NW;              // threads
  static constexpr int FP = (F + 3) / 4 * 4;     // K of the forward GEMM, padded for 16x16x4
  static constexpr int NKT = (F + 15) / 16;      // 16-wide feature tiles of the weight gradient
  static constexpr int SX = NKT * 16 + 1;        // LDS row stride of the batch (padded: no 16-way conflict)
  static constexpr int SD = H + 1;               // LDS row stride of dh
  static constexpr int BM = 16;                  // max micro-batch (MFMA M of the forward)
  static constexpr int P = H * F + 2 * H + 1;
  static constexpr int PP = (P + 3) / 4 * 4;
  static constexpr int NCH = PP / 4;             // float4 chunks
  static constexpr int CPT = (NCH + T - 1) / T;  // chunks per thread
  static constexpr int XE = BM * F;
  static constexpr int XPT = (XE + T - 1) / T;   // batch elements loaded per thread per step
  static constexpr int OFF_B1 = H * F, OFF_W2 = H * F + H, OFF_B2 = H * F + 2 * H;
  static_assert(H % 16 == 0 && H >= 16 && H <= 256, "hidden must be a multiple of 16 in [16, 256]");
  static_assert(F >= 1 && F <= 64, "n_features must be in [1, 64]");
};

template <int F, int H>
struct __attribute__((aligned(16))) TinySmem {
  using C = TinyCfg<F, H>;
  float P[C::PP];          // parameters
  float G[C::PP];          // gradient of the current step
  float X[C::BM * C::SX];  // current minibatch, rows >= batch and cols >= F are zero
  float Y[C::BM];
  float Z[C::NW * 16];     // per-wave partial logits
  float DH[C::BM * C::SD]; // dL/d(pre-activation)
  int idx[C::BM];          // sample indices of the NEXT step (prefetch pipeline)
  int err;
};

// Forward + BCE + backward of one step; the gradient lands in sm.G.  Returns the step's mean loss
// (identical in every lane).  Contains two workgroup barriers; the caller provides the others.
template <int F, int H>
DGT_DEVICE float tiny_fwd_bwd(TinySmem<F, H>& sm, int Bt) {
  using C = TinyCfg<F, H>;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, lr = l & 15, lq = l >> 4;
  const int j0 = 16 * w, j = j0 + lr;

  // ---- forward GEMM on MFMA: D[b][j] = sum_k x[b][k] * W1[j][k]
  // 16x16x4 f32 operand maps: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15];
  // D: col = l&15 (hidden j), row = 4*(l>>4) + r (batch b).
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < C::FP / 4; ++ks) {
    const int k = 4 * ks + lq;
    const float a = sm.X[lr * C::SX + k];
    const float b = (F % 4 == 0 || k < F) ? sm.P[j * F + k] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const float b1 = sm.P[C::OFF_B1 + j];
  const float w2 = sm.P[C::OFF_W2 + j];
  float h[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    h[r] = fmaxf(acc[r] + b1, 0.f);
    const float pz = wave_sum16(h[r] * w2);  // partial logit over this wave's 16 hidden units
    if (lr == 0) sm.Z[w * 16 + 4 * lq + r] = pz;
  }
  __syncthreads();

  // ---- logits, BCE-with-logits (torch: (1-y)*z - log_sigmoid(z)), dL/dz = (sigmoid(z)-y)/B
  const float b2 = sm.P[C::OFF_B2];
  const float invB = 1.0f / (float)Bt;
  float dz[4];
  float lsum = 0.f, db2 = 0.f, dw2 = 0.f, db1 = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = 4 * lq + r;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < C::NW; ++ww) s += sm.Z[ww * 16 + b];
    const float z = s + b2;
    const float y = sm.Y[b];
    const bool valid = b < Bt;
    const float e = __expf(-fabsf(z));
    const float log_sig = fminf(z, 0.f) - log1pf(e);
    const float sig = (z >= 0.f) ? 1.f / (1.f + e) : e / (1.f + e);
    dz[r] = valid ? (sig - y) * invB : 0.f;
    lsum += valid ? (1.f - y) * z - log_sig : 0.f;
    // backward through Linear(H,1) and ReLU
    dw2 = fmaf(dz[r], h[r], dw2);
    const float dh = (h[r] > 0.f) ? dz[r] * w2 : 0.f;
    sm.DH[b * C::SD + j] = dh;
    db1 += dh;
    db2 += dz[r];
  }
  dw2 = wave_sum_groups(dw2);
  db1 = wave_sum_groups(db1);
  db2 = wave_sum_groups(db2);
  lsum = wave_sum_groups(lsum);
  if (lq == 0) {
    sm.G[C::OFF_W2 + j] = dw2;
    sm.G[C::OFF_B1 + j] = db1;
  }
  if (t == 0) sm.G[C::OFF_B2] = db2;
  __syncthreads();

  // ---- weight gradient on MFMA: dW1[j][k] = sum_b dh[b][j] * x[b][k]
  // A[i = hidden (l&15)][kk = batch (l>>4)], B[kk = batch][col = feature (l&15)];
  // D: col = feature 16*ct + (l&15), row = hidden j0 + 4*(l>>4) + r.
  const int nks = (Bt + 3) >> 2;
#pragma unroll
  for (int ct = 0; ct < C::NKT; ++ct) {
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C::BM / 4; ++ks) {
      if (ks < nks) {  // wave-uniform
        const int b = 4 * ks + lq;
        const float a = sm.DH[b * C::SD + j0 + lr];
        const float xb = sm.X[b * C::SX + 16 * ct + lr];
        g = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xb, g, 0, 0, 0);
      }
    }
    const int k = 16 * ct + lr;
    if (k < F) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sm.G[(j0 + 4 * lq + r) * F + k] = g[r];
    }
  }
  return lsum / (float)Bt;
}

// Gather the x / y values this thread stages for one step (rows from sm.idx).
template <int F, int H>
DGT_DEVICE void gather_rows(const TinySmem<F, H>& sm, const float* __restrict__ X, const float* __restrict__ Y,
                            float (&xv)[TinyCfg<F, H>::XPT], float& yv) {
  using C = TinyCfg<F, H>;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < C::XPT; ++q) {
    const int e = t + q * C::T;
    float v = 0.f;
    if (e < C::XE) {
      const int id = sm.idx[e / F];
      if (id >= 0) v = X[(long long)id * F + (e % F)];
    }
    xv[q] = v;
  }
  yv = 0.f;
  if (t < C::BM) {
    const int id = sm.idx[t];
    if (id >= 0) yv = Y[id];
  }
}

template <int F, int H>
DGT_DEVICE void stage_rows(TinySmem<F, H>& sm, const float (&xv)[TinyCfg<F, H>::XPT], float yv) {
  using C = TinyCfg<F, H>;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < C::XPT; ++q) {
    const int e = t + q * C::T;
    if (e < C::XE) sm.X[(e / F) * C::SX + (e % F)] = xv[q];
  }
  if (t < C::BM) sm.Y[t] = yv;
}

DGT_DEVICE int plan_at(const int* plan, int n_steps, int bmax, int step, int row) {
  return (step < n_steps && row < bmax) ? plan[(long long)step * bmax + row] : -1;
}

template <int F, int H>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_mlp_train_kernel(TinyTrainArgs a) {
  using C = TinyCfg<F, H>;
  __shared__ TinySmem<F, H> sm;
  const int t = threadIdx.x;
  const Exchange& ex = a.ex;

  if (a.bmax > C::BM || a.bmax < 1 || ex.world_size < 1 || ex.world_size > kMaxRanks ||
      (ex.world_size > 1 && ex.stride < C::PP)) {
    if (t == 0) *a.status = kBadShape;
    return;
  }

  // ---- prologue: parameters -> LDS, moments -> registers, batch 0 staged, batch 1 in flight
  for (int i = t; i < C::PP; i += C::T) {
    sm.P[i] = (i < C::P) ? a.params[i] : 0.f;
    sm.G[i] = 0.f;
  }
  for (int i = t; i < C::BM * C::SX; i += C::T) sm.X[i] = 0.f;
  if (t == 0) sm.err = 0;
  f32x4 m[C::CPT], v[C::CPT];
#pragma unroll
  for (int c = 0; c < C::CPT; ++c) {
    const int ch = t + c * C::T;
    if (ch < C::NCH) {
      m[c] = *reinterpret_cast<const f32x4*>(a.exp_avg + 4 * ch);
      v[c] = *reinterpret_cast<const f32x4*>(a.exp_avg_sq + 4 * ch);
    } else {
      m[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      v[c] = m[c];
    }
  }
  if (t < C::BM) sm.idx[t] = plan_at(a.plan, a.n_steps, a.bmax, 0, t);
  __syncthreads();
  float xv[C::XPT], yv;
  gather_rows<F, H>(sm, a.X, a.Y, xv, yv);
  __syncthreads();  // every thread has read sm.idx (step 0)
  stage_rows<F, H>(sm, xv, yv);
  if (t < C::BM) sm.idx[t] = plan_at(a.plan, a.n_steps, a.bmax, 1, t);
  int idx_reg = (t < C::BM) ? plan_at(a.plan, a.n_steps, a.bmax, 2, t) : -1;
  __syncthreads();

  double b1p = pow(a.beta1, (double)a.adam_step0);
  double b2p = pow(a.beta2, (double)a.adam_step0);
  double loss_total = 0.0;
  const float inv_ws = 1.0f / (float)ex.world_size;
  int s = 0;
  for (; s < a.n_steps; ++s) {
    const int Bt = a.counts[s];
    // prefetch step s+1 rows (indices already in sm.idx); consumed after this step's last barrier
    if (s + 1 < a.n_steps) gather_rows<F, H>(sm, a.X, a.Y, xv, yv);

    const float step_loss = tiny_fwd_bwd<F, H>(sm, Bt);
    __syncthreads();  // gradient complete in sm.G; nobody reads sm.X / sm.idx / sm.P any more

    if (s + 1 < a.n_steps) stage_rows<F, H>(sm, xv, yv);
    if (t < C::BM) {
      sm.idx[t] = idx_reg;
      idx_reg = plan_at(a.plan, a.n_steps, a.bmax, s + 3, t);
    }

    f32x4 g[C::CPT];
#pragma unroll
    for (int c = 0; c < C::CPT; ++c) {
      const int ch = t + c * C::T;
      g[c] = (ch < C::NCH) ? *reinterpret_cast<const f32x4*>(&sm.G[4 * ch]) : f32x4{0.f, 0.f, 0.f, 0.f};
    }

    if (ex.world_size > 1) {
      // ---- one-shot exchange over xGMI: push to every peer, flag, wait, sum in rank order
      const long long seq = ex.seq_base + s;
      const int parity = (int)(seq & 1);
      const unsigned val = (unsigned)(seq + 1);
#pragma unroll
      for (int c = 0; c < C::CPT; ++c) {
        const int ch = t + c * C::T;
        if (ch < C::NCH) {
          for (int p = 0; p < ex.world_size; ++p) {
            if (p == ex.rank) continue;
            float* dst = ex.data[p] + (long long)(parity * kMaxRanks + ex.rank) * ex.stride + 4 * ch;
            *reinterpret_cast<f32x4*>(dst) = g[c];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t < ex.world_size && t != ex.rank) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store_release_system(ex.flags[t] + parity * kMaxRanks + ex.rank, val);
        if (!spin_geq(ex.flags[ex.rank] + parity * kMaxRanks + t, val, ex.timeout_ticks)) sm.err = 1;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (sm.err) break;
#pragma unroll
      for (int c = 0; c < C::CPT; ++c) {
        const int ch = t + c * C::T;
        if (ch < C::NCH) {
          f32x4 sum = {0.f, 0.f, 0.f, 0.f};
          for (int p = 0; p < ex.world_size; ++p) {
            f32x4 gp;
            if (p == ex.rank) {
              gp = g[c];
            } else {
              const float* src = ex.data[ex.rank] + (long long)(parity * kMaxRanks + p) * ex.stride + 4 * ch;
              gp = *reinterpret_cast<const f32x4*>(src);
            }
            sum += gp;
          }
          g[c] = sum * inv_ws;
        }
      }
    }

    // ---- Adam (torch foreach op order); bias correction formed in double like torch does on host
    b1p *= a.beta1;
    b2p *= a.beta2;
    const float step_size_neg = (float)(-(a.lr / (1.0 - b1p)));
    const float bc2_sqrt = (float)sqrt(1.0 - b2p);
#pragma unroll
    for (int c = 0; c < C::CPT; ++c) {
      const int ch = t + c * C::T;
      if (ch < C::NCH) {
        f32x4 p4 = *reinterpret_cast<const f32x4*>(&sm.P[4 * ch]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float mm = m[c][e], vv = v[c][e];
          p4[e] = adam_update(p4[e], g[c][e], mm, vv, a.hp, step_size_neg, bc2_sqrt);
          m[c][e] = mm;
          v[c][e] = vv;
        }
        *reinterpret_cast<f32x4*>(&sm.P[4 * ch]) = p4;
      }
    }
    loss_total += (double)step_loss;
    __syncthreads();
  }

  // ---- epilogue: state back to HBM
  for (int i = t; i < C::P; i += C::T) a.params[i] = sm.P[i];
#pragma unroll
  for (int c = 0; c < C::CPT; ++c) {
    const int ch = t + c * C::T;
    if (ch < C::NCH) {
      *reinterpret_cast<f32x4*>(a.exp_avg + 4 * ch) = m[c];
      *reinterpret_cast<f32x4*>(a.exp_avg_sq + 4 * ch) = v[c];
    }
  }
  if (t == 0) {
    *a.loss_acc += loss_total;
    *a.status = sm.err ? kTimeout : kOk;
  }
}

// One step's gradient only (the RCCL path: grad -> all_reduce -> adam_flat).
template <int F, int H>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_mlp_grad_kernel(TinyGradArgs a) {
  using C = TinyCfg<F, H>;
  __shared__ TinySmem<F, H> sm;
  const int t = threadIdx.x;
  for (int i = t; i < C::PP; i += C::T) {
    sm.P[i] = (i < C::P) ? a.params[i] : 0.f;
    sm.G[i] = 0.f;
  }
  for (int i = t; i < C::BM * C::SX; i += C::T) sm.X[i] = 0.f;
  if (t < C::BM) sm.idx[t] = (t < a.bmax) ? a.plan[(long long)a.step * a.bmax + t] : -1;
  __syncthreads();
  float xv[C::XPT], yv;
  gather_rows<F, H>(sm, a.X, a.Y, xv, yv);
  stage_rows<F, H>(sm, xv, yv);
  __syncthreads();
  const float loss = tiny_fwd_bwd<F, H>(sm, a.counts[a.step]);
  __syncthreads();
  for (int i = t; i < C::PP; i += C::T) a.grad[i] = sm.G[i];
  if (t == 0) *a.loss_acc += (double)loss;
}

// ------------------------------------------------------------------ dispatch
#define DGT_TINY_SHAPES(X) X(20, 64) X(32, 64) X(20, 128) X(8, 16)

bool tiny_mlp_supported(int f, int h) {
#define X_(F_, H_) if (f == F_ && h == H_) return true;
  DGT_TINY_SHAPES(X_)
#undef X_
  return false;
}

int tiny_mlp_padded_numel(int f, int h) { return (h * f + 2 * h + 1 + 3) / 4 * 4; }

hipError_t tiny_mlp_train(int f, int h, const TinyTrainArgs& a, hipStream_t stream) {
#define X_(F_, H_)                                                                        \
  if (f == F_ && h == H_) {                                                               \
    hipLaunchKernelGGL((tiny_mlp_train_kernel<F_, H_>), dim3(1), dim3(TinyCfg<F_, H_>::T), 0, \
                       stream, a);                                                        \
    return hipGetLastError();                                                             \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
  return hipErrorInvalidValue;
}

hipError_t tiny_mlp_grad(int f, int h, const TinyGradArgs& a, hipStream_t stream) {
#define X_(F_, H_)                                                                        \
  if (f == F_ && h == H_) {                                                               \
    hipLaunchKernelGGL((tiny_mlp_grad_kernel<F_, H_>), dim3(1), dim3(TinyCfg<F_, H_>::T), 0, \
                       stream, a);                                                        \
    return hipGetLastError();                                                             \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
  return hipErrorInvalidValue;
}

}  // namespace dgt
