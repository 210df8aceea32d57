// Fused training kernels for the reference model (SimpleNet: Linear(F,H) -> ReLU -> Linear(H,1),
// BCE-with-logits, Adam; reference train.py:26-36, 96, 107-115).
//
// Design (MI355X-first, not a translation of the reference's ~30 ATen/cuBLAS launches per step):
//   * ONE workgroup of H/16 waves trains the model; a launch runs many optimizer steps.
//   * Each wave OWNS 16 hidden units end to end: its rows of W1, its slice of b1 and W2, their
//     gradients, their Adam moments (registers) and a private copy of the minibatch.  The only
//     cross-wave dependency of a step is the sum of the per-wave partial logits, so a step has
//     ONE workgroup barrier (the partial-logit buffer is double-buffered by step parity).
//     The shared scalar b2 is updated redundantly (bit-identically) by every wave.
//   * Both GEMM-shaped products run on the matrix cores with exact-fp32 MFMA
//     (v_mfma_f32_16x16x4_f32): the forward x.W1^T (M = batch, N = the wave's 16 hidden units,
//     K = features) and the weight gradient dh^T.x (M = hidden, N = features, K = batch).
//     Operands are staged through LDS with padded strides.
//   * Row reductions use DPP (v_add_f32_dpp) and the gfx950 v_permlane{16,32}_swap exchanges,
//     never ds_bpermute.
//   * Minibatch rows are gathered from the device-resident dataset by sampler index; the next
//     step's rows are prefetched into registers while the current step computes (no per-step H2D,
//     no host sync: SURVEY K1/K2/K24).
//   * World size > 1: each wave pushes its gradient slice into every peer's IPC mailbox over
//     xGMI, raises a per-(wave, rank) sequence flag (system-scope release), waits for its own flags
//     and sums the contributions in rank order, so every rank applies bit-identical updates.  This
//     replaces DeepSpeed's flatten -> NCCL all_reduce -> scale -> unflatten.
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

template <int F, int H>
struct TinyCfg {
  static constexpr int NW = H / 16;              // waves; wave w owns hidden units [16w, 16w+16)
  static constexpr int T = 64 * NW;              // threads
  static constexpr int FP = (F + 3) / 4 * 4;     // K of the forward GEMM, padded for 16x16x4
  static constexpr int NKT = (F + 15) / 16;      // 16-wide feature tiles of the weight gradient
  static constexpr int SX = NKT * 16 + 1;        // LDS row stride of the batch (+1: no 16-way conflict)
  static constexpr int BM = 16;                  // max micro-batch (MFMA M of the forward)
  static constexpr int P = H * F + 2 * H + 1;    // global flat parameter count
  static constexpr int PP = (P + 3) / 4 * 4;
  // a wave's local parameter vector: [W1 rows 16 x F][b1 16][W2 16][b2]
  static constexpr int L_B1 = 16 * F, L_W2 = 16 * F + 16, L_B2 = 16 * F + 32;
  static constexpr int WP = 16 * F + 33;
  static constexpr int NPL = (WP + 63) / 64;     // owned elements per lane
  static constexpr int WPP = NPL * 64;
  static constexpr int XE = BM * F;
  static constexpr int XPL = (XE + 63) / 64;     // batch elements each lane stages
  static constexpr int G_B1 = H * F, G_W2 = H * F + H, G_B2 = H * F + 2 * H;
  static_assert(H % 16 == 0 && H >= 16 && H <= 256, "hidden must be a multiple of 16 in [16, 256]");
  static_assert(F >= 1 && F <= 64, "n_features must be in [1, 64]");

  // local element e of wave w -> index in the global flat vector
  static DGT_HOST_DEVICE int global_index(int w, int e) {
    if (e < L_B1) return 16 * w * F + e;
    if (e < L_W2) return G_B1 + 16 * w + (e - L_B1);
    if (e < L_B2) return G_W2 + 16 * w + (e - L_W2);
    return G_B2;
  }
};

template <int F, int H>
struct __attribute__((aligned(16))) WaveSmem {
  using C = TinyCfg<F, H>;
  float P[C::WPP];           // this wave's parameters
  float G[C::WPP];           // their gradient for the current step
  float X[C::BM * C::SX];    // private copy of the minibatch (rows >= batch, cols >= F are zero)
  float DH[C::BM * 17];      // dL/d(pre-activation) of this wave's 16 hidden units
  float Y[C::BM];
  int idx[C::BM];            // sample indices of the NEXT step (prefetch pipeline)
};

template <int F, int H>
struct __attribute__((aligned(16))) TinySmem {
  using C = TinyCfg<F, H>;
  WaveSmem<F, H> w[C::NW];
  float Z[2][C::NW * 16];    // per-wave partial logits, double-buffered by step parity
  int err;
};

// ------------------------------------------------------------------ per-wave step pieces

// Forward GEMM on MFMA + bias + ReLU; publishes this wave's partial logits into Zbuf.
template <int F, int H>
DGT_DEVICE void wave_forward(WaveSmem<F, H>& ws, float* Zbuf, int w, int l, float (&h)[4]) {
  using C = TinyCfg<F, H>;
  const int lr = l & 15, lq = l >> 4;
  // 16x16x4 f32 operand maps: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15];
  // D: col = l&15 (hidden unit), row = 4*(l>>4) + r (batch row).
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < C::FP / 4; ++ks) {
    const int k = 4 * ks + lq;
    const float a = ws.X[lr * C::SX + k];
    const float b = (F % 4 == 0 || k < F) ? ws.P[lr * F + k] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const float b1 = ws.P[C::L_B1 + lr];
  const float w2 = ws.P[C::L_W2 + lr];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    h[r] = fmaxf(acc[r] + b1, 0.f);
    const float pz = wave_sum16(h[r] * w2);
    if (lr == 0) Zbuf[w * 16 + 4 * lq + r] = pz;
  }
}

// After the barrier: logits, loss, backward into ws.G.  Returns the step's mean loss (every lane).
template <int F, int H, bool WANT_LOSS>
DGT_DEVICE float wave_backward(WaveSmem<F, H>& ws, const float* Zbuf, int l, const float (&h)[4], int Bt,
                               float invB) {
  using C = TinyCfg<F, H>;
  const int lr = l & 15, lq = l >> 4;
  const float b2 = ws.P[C::L_B2];
  const float w2 = ws.P[C::L_W2 + lr];
  float lsum = 0.f, dw2 = 0.f, db1 = 0.f, db2 = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = 4 * lq + r;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < C::NW; ++ww) s += Zbuf[ww * 16 + b];
    const float z = s + b2;
    const float y = ws.Y[b];
    const bool valid = b < Bt;
    // BCE-with-logits (torch: (1-y)*z - log_sigmoid(z)); d/dz = sigmoid(z) - y, times 1/B (mean)
    const float e = __expf(-fabsf(z));
    const float rinv = __builtin_amdgcn_rcpf(1.f + e);
    const float sig = (z >= 0.f) ? rinv : e * rinv;
    const float dz = valid ? (sig - y) * invB : 0.f;
    if (WANT_LOSS) lsum += valid ? (1.f - y) * z - (fminf(z, 0.f) - __logf(1.f + e)) : 0.f;
    dw2 = fmaf(dz, h[r], dw2);
    const float dh = (h[r] > 0.f) ? dz * w2 : 0.f;
    ws.DH[b * 17 + lr] = dh;
    db1 += dh;
    db2 += dz;
  }
  dw2 = wave_sum_groups(dw2);
  db1 = wave_sum_groups(db1);
  db2 = wave_sum_groups(db2);
  if (lq == 0) {
    ws.G[C::L_W2 + lr] = dw2;
    ws.G[C::L_B1 + lr] = db1;
  }
  if (l == 0) ws.G[C::L_B2] = db2;
  __builtin_amdgcn_wave_barrier();

  // weight gradient on MFMA: dW1[jj][k] = sum_b dh[b][jj] * x[b][k]
  // A[i = hidden (l&15)][kk = batch (l>>4)], B[kk = batch][col = feature (l&15)];
  // D: col = feature 16*ct + (l&15), row = hidden 4*(l>>4) + r.
  const int nks = (Bt + 3) >> 2;
#pragma unroll
  for (int ct = 0; ct < C::NKT; ++ct) {
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C::BM / 4; ++ks) {
      if (ks < nks) {  // wave-uniform
        const int b = 4 * ks + lq;
        g = __builtin_amdgcn_mfma_f32_16x16x4f32(ws.DH[b * 17 + lr], ws.X[b * C::SX + 16 * ct + lr], g, 0, 0, 0);
      }
    }
    const int k = 16 * ct + lr;
    if (k < F) {
#pragma unroll
      for (int r = 0; r < 4; ++r) ws.G[(4 * lq + r) * F + k] = g[r];
    }
  }
  __builtin_amdgcn_wave_barrier();
  return WANT_LOSS ? wave_sum_groups(lsum) * invB : 0.f;
}

// Gather the x / y values this lane stages for one step (rows from ws.idx).
template <int F, int H>
DGT_DEVICE void gather_rows(const WaveSmem<F, H>& ws, const float* __restrict__ X, const float* __restrict__ Y,
                            int l, float (&xv)[TinyCfg<F, H>::XPL], float& yv) {
  using C = TinyCfg<F, H>;
#pragma unroll
  for (int q = 0; q < C::XPL; ++q) {
    const int e = l + 64 * q;
    float v = 0.f;
    if (e < C::XE) {
      const int id = ws.idx[e / F];
      if (id >= 0) v = X[(long long)id * F + (e % F)];
    }
    xv[q] = v;
  }
  yv = 0.f;
  if (l < C::BM) {
    const int id = ws.idx[l];
    if (id >= 0) yv = Y[id];
  }
}

template <int F, int H>
DGT_DEVICE void stage_rows(WaveSmem<F, H>& ws, int l, const float (&xv)[TinyCfg<F, H>::XPL], float yv) {
  using C = TinyCfg<F, H>;
#pragma unroll
  for (int q = 0; q < C::XPL; ++q) {
    const int e = l + 64 * q;
    if (e < C::XE) ws.X[(e / F) * C::SX + (e % F)] = xv[q];
  }
  if (l < C::BM) ws.Y[l] = yv;
}

DGT_DEVICE int plan_at(const int* plan, int n_steps, int bmax, int step, int row) {
  return (step < n_steps && row < bmax) ? plan[(long long)step * bmax + row] : -1;
}

template <int F, int H>
DGT_DEVICE void wave_init(WaveSmem<F, H>& ws, const float* __restrict__ params, int w, int l) {
  using C = TinyCfg<F, H>;
  for (int e = l; e < C::WPP; e += 64) {
    ws.P[e] = (e < C::WP) ? params[C::global_index(w, e)] : 0.f;
    ws.G[e] = 0.f;
  }
  for (int i = l; i < C::BM * C::SX; i += 64) ws.X[i] = 0.f;
  for (int i = l; i < C::BM * 17; i += 64) ws.DH[i] = 0.f;
}

// ------------------------------------------------------------------ persistent training kernel
template <int F, int H>
__global__ __launch_bounds__((TinyCfg<F, H>::T)) void tiny_mlp_train_kernel(TinyTrainArgs a) {
  using C = TinyCfg<F, H>;
  __shared__ TinySmem<F, H> sm;
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const Exchange& ex = a.ex;
  WaveSmem<F, H>& ws = sm.w[w];

  if (a.bmax > C::BM || a.bmax < 1 || ex.world_size < 1 || ex.world_size > kMaxRanks ||
      (ex.world_size > 1 && ex.stride < C::PP)) {
    if (t == 0) *a.status = kBadShape;
    return;
  }

  // ---- prologue: parameters -> LDS, moments -> registers, batch 0 staged, batch 1 indices ready
  wave_init<F, H>(ws, a.params, w, l);
  if (t == 0) sm.err = 0;
  float m[C::NPL], v[C::NPL];
#pragma unroll
  for (int i = 0; i < C::NPL; ++i) {
    const int e = l + 64 * i;
    m[i] = v[i] = 0.f;
    if (e < C::WP) {
      const int gi = C::global_index(w, e);
      m[i] = a.exp_avg[gi];
      v[i] = a.exp_avg_sq[gi];
    }
  }
  if (l < C::BM) ws.idx[l] = plan_at(a.plan, a.n_steps, a.bmax, 0, l);
  __builtin_amdgcn_wave_barrier();
  float xv[C::XPL], yv;
  gather_rows<F, H>(ws, a.X, a.Y, l, xv, yv);
  __builtin_amdgcn_wave_barrier();
  stage_rows<F, H>(ws, l, xv, yv);
  if (l < C::BM) ws.idx[l] = plan_at(a.plan, a.n_steps, a.bmax, 1, l);
  int idx_reg = (l < C::BM) ? plan_at(a.plan, a.n_steps, a.bmax, 2, l) : -1;
  __syncthreads();

  double b1p = pow(a.beta1, (double)a.adam_step0);
  double b2p = pow(a.beta2, (double)a.adam_step0);
  double loss_total = 0.0;
  const float inv_ws = 1.0f / (float)ex.world_size;
  for (int s = 0; s < a.n_steps; ++s) {
    const int Bt = a.counts[s];
    const float invB = 1.0f / (float)Bt;
    // prefetch step s+1 rows (indices already in ws.idx); consumed after this step's wgrad
    if (s + 1 < a.n_steps) gather_rows<F, H>(ws, a.X, a.Y, l, xv, yv);

    float h[4];
    float* Zb = sm.Z[s & 1];
    wave_forward<F, H>(ws, Zb, w, l, h);
    __syncthreads();  // the step's only workgroup barrier: all partial logits published
    if (sm.err) break;
    const float step_loss = (w == 0) ? wave_backward<F, H, true>(ws, Zb, l, h, Bt, invB)
                                     : wave_backward<F, H, false>(ws, Zb, l, h, Bt, invB);

    // this wave is done reading its batch copy: stage the next one
    if (s + 1 < a.n_steps) stage_rows<F, H>(ws, l, xv, yv);
    if (l < C::BM) {
      ws.idx[l] = idx_reg;
      idx_reg = plan_at(a.plan, a.n_steps, a.bmax, s + 3, l);
    }

    float g[C::NPL];
#pragma unroll
    for (int i = 0; i < C::NPL; ++i) g[i] = ws.G[l + 64 * i];

    if (ex.world_size > 1) {
      // ---- one-shot exchange of this wave's slice over xGMI: push, flag, wait, sum in rank order
      const long long seq = ex.seq_base + s;
      const int parity = (int)(seq & 1);
      const unsigned val = (unsigned)(seq + 1);
#pragma unroll
      for (int i = 0; i < C::NPL; ++i) {
        const int e = l + 64 * i;
        if (e < C::WP) {
          const long long gi = C::global_index(w, e);
          for (int p = 0; p < ex.world_size; ++p) {
            if (p == ex.rank) continue;
            ex.data[p][(long long)(parity * kMaxRanks + ex.rank) * ex.stride + gi] = g[i];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (l < ex.world_size && l != ex.rank) {
        const int fo = (w * 2 + parity) * kMaxRanks;
        store_release_system(ex.flags[l] + fo + ex.rank, val);
        if (!spin_geq(ex.flags[ex.rank] + fo + l, val, ex.timeout_ticks)) sm.err = 1;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < C::NPL; ++i) {
        const int e = l + 64 * i;
        if (e < C::WP) {
          const long long gi = C::global_index(w, e);
          float sum = 0.f;
          for (int p = 0; p < ex.world_size; ++p)
            sum += (p == ex.rank) ? g[i] : ex.data[ex.rank][(long long)(parity * kMaxRanks + p) * ex.stride + gi];
          g[i] = sum * inv_ws;
        }
      }
    }

    // ---- Adam (torch foreach op order); bias correction formed in double like torch does on host
    b1p *= a.beta1;
    b2p *= a.beta2;
    const float step_size_neg = (float)(-(a.lr / (1.0 - b1p)));
    const float bc2_sqrt = (float)sqrt(1.0 - b2p);
#pragma unroll
    for (int i = 0; i < C::NPL; ++i) {
      const int e = l + 64 * i;
      if (e < C::WP) ws.P[e] = adam_update(ws.P[e], g[i], m[i], v[i], a.hp, step_size_neg, bc2_sqrt);
    }
    __builtin_amdgcn_wave_barrier();
    loss_total += (double)step_loss;
  }

  // ---- epilogue: state back to HBM (b2 belongs to wave 0)
#pragma unroll
  for (int i = 0; i < C::NPL; ++i) {
    const int e = l + 64 * i;
    if (e < C::WP && (e != C::L_B2 || w == 0)) {
      const int gi = C::global_index(w, e);
      a.params[gi] = ws.P[e];
      a.exp_avg[gi] = m[i];
      a.exp_avg_sq[gi] = v[i];
    }
  }
  __syncthreads();
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
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  WaveSmem<F, H>& ws = sm.w[w];
  wave_init<F, H>(ws, a.params, w, l);
  if (l < C::BM) ws.idx[l] = (l < a.bmax) ? a.plan[(long long)a.step * a.bmax + l] : -1;
  __builtin_amdgcn_wave_barrier();
  float xv[C::XPL], yv;
  gather_rows<F, H>(ws, a.X, a.Y, l, xv, yv);
  stage_rows<F, H>(ws, l, xv, yv);
  __builtin_amdgcn_wave_barrier();
  const int Bt = a.counts[a.step];
  const float invB = 1.0f / (float)Bt;
  float h[4];
  wave_forward<F, H>(ws, sm.Z[0], w, l, h);
  __syncthreads();
  const float loss = wave_backward<F, H, true>(ws, sm.Z[0], l, h, Bt, invB);
  for (int e = l; e < C::WP; e += 64) {
    if (e != C::L_B2 || w == 0) a.grad[C::global_index(w, e)] = ws.G[e];
  }
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
#define X_(F_, H_)                                                                            \
  if (f == F_ && h == H_) {                                                                   \
    hipLaunchKernelGGL((tiny_mlp_train_kernel<F_, H_>), dim3(1), dim3(TinyCfg<F_, H_>::T), 0, \
                       stream, a);                                                            \
    return hipGetLastError();                                                                 \
  }
  DGT_TINY_SHAPES(X_)
#undef X_
  return hipErrorInvalidValue;
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
