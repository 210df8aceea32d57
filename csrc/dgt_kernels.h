// Host-side launch API of the HIP kernels (no torch headers: the .hip translation units compile fast
// and the torch binding layer in bindings.cpp only sees these declarations).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dgt_common.h"

namespace dgt {

// ---------------------------------------------------------------- tiny MLP (reference model)
// Which (n_features, hidden) pairs have a compiled fused kernel.
bool tiny_mlp_supported(int n_features, int hidden);
int tiny_mlp_padded_numel(int n_features, int hidden);  // flat length incl. float4 padding
int tiny_mlp_exchange_floats(int n_features, int hidden);  // IPC mailbox floats per (parity, rank)

struct TinyTrainArgs {
  const float* X;        // [n_samples, F]
  const float* Y;        // [n_samples]
  const int* plan;       // [n_steps, bmax] sample indices, -1 = padding
  const int* counts;     // [n_steps] valid rows per step
  int n_steps;
  int bmax;              // <= 16
  float* params;         // [padded numel] flat: W1[H,F], b1[H], W2[H], b2
  float* exp_avg;        // [padded numel]
  float* exp_avg_sq;     // [padded numel]
  AdamHyper hp;
  double lr;             // python-double lr (bias-corrected step size is formed in double)
  double beta1, beta2;
  long long adam_step0;  // optimizer steps already taken before this launch
  float* bc;             // [n_steps + 1][2] workspace: the kernel fills it with its steps' bias corrections
  double* loss_acc;      // += sum over steps of the step's mean loss
  int* status;           // Status
  Exchange ex;           // world_size 1 -> no exchange
  unsigned long long* stamps;  // diagnostic builds only (-DDGT_TINY_STAMPS); nullptr otherwise
};

hipError_t tiny_mlp_train(int n_features, int hidden, const TinyTrainArgs& a, hipStream_t stream);
// the instantiation tiny_mlp_train would launch for these arguments (nullptr: none) and its block size
const void* tiny_mlp_train_symbol(int n_features, int hidden, const TinyTrainArgs& a, int* threads);

// n_steps exchanges of the fused kernel's mailbox layout and line format (ex.line) with payloads that
// expose any torn or lost line: bad words are added to *errors, a timeout sets *status.
hipError_t tiny_xch_stress(int n_features, int hidden, const Exchange& ex, int n_steps, int* status, int* errors,
                           hipStream_t stream);

struct TinyGradArgs {
  const float* X;
  const float* Y;
  const int* plan;       // [n_steps, bmax]
  const int* counts;     // [n_steps]
  int step;              // which row of the plan
  int bmax;
  const float* params;   // flat (padded)
  float* grad;           // flat (padded), overwritten
  double* loss_acc;      // += this step's mean loss
};

hipError_t tiny_mlp_grad(int n_features, int hidden, const TinyGradArgs& a, hipStream_t stream);

// ---------------------------------------------------------------- flat fused Adam
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

struct AdamFlatArgs {
  float* master;         // fp32 master params [n]
  void* param_lp;        // optional low-precision copy (nullptr = none)
  int lp_dtype;          // DType of param_lp
  const void* grad;      // [n]
  int grad_dtype;        // DType
  float* exp_avg;
  float* exp_avg_sq;
  long long n;           // multiple of 4
  AdamHyper hp;
  float step_size_neg;   // -lr / (1 - beta1^t)
  float bc2_sqrt;        // sqrt(1 - beta2^t)
  float grad_scale;      // multiplies the gradient (1/world_size, 1/loss_scale ...)
  const float* grad_scale_dev;  // optional extra device-side multiplier (clip coefficient)
  // optional device-resident step counter (graph replay): when set, the kernel forms the bias
  // corrections from *step_dev (the 1-based step of THIS update) instead of the host scalars
  long long* step_dev;
  // with step_dev: advance the counter in this launch -- this update is step *step_dev + 1, and the
  // last block to finish stores it back (a zeroed ticket it counts on and resets): a graph-replayed
  // step needs no separate increment node
  unsigned* step_ticket;
  double lr_d, beta1_d, beta2_d;
};

// *counter += 1 on the stream (advances the device-side Adam step inside a captured graph)
hipError_t step_increment(long long* counter, hipStream_t stream);

hipError_t adam_flat(const AdamFlatArgs& a, hipStream_t stream);

// ---------------------------------------------------------------- fused BCE-with-logits (loss.hip)
// loss[0] = mean BCE-with-logits of z[n] (fp32 or bf16) against y[n]; dz[n] = (sigmoid(z) - y) / n.
// fused small-batch Linear (+ReLU) forward / backward for the engine's kernel injection (fp32)
hipError_t linear_fwd(const float* x, const float* W, const float* b, float* y, int M, int N, int K, bool relu,
                      hipStream_t stream);
hipError_t linear_bwd(const float* dy, const float* x, const float* W, const float* y, float* dx, float* dW,
                      float* db, int M, int N, int K, bool accumulate, hipStream_t stream);
// a two-layer chain Linear(K, H)(+ReLU) -> Linear(H, O)(+ReLU) in ONE workgroup (small batches: M * H
// <= 4096, bitwise the two per-layer launches)
bool linear2_fits(int M, int K, int H, int O);
hipError_t linear2_fwd(const float* x, const float* W1, const float* b1, const float* W2, const float* b2, float* h,
                       float* y, int M, int K, int H, int O, bool relu1, bool relu2, hipStream_t stream);
hipError_t linear2_bwd(const float* dy, const float* x, const float* W1, const float* h, const float* W2,
                       const float* y, float* dx, float* dW1, float* db1, float* dW2, float* db2, int M, int K, int H,
                       int O, bool relu1, bool acc1, bool acc2, hipStream_t stream);
hipError_t bce_logits(const void* z, int z_dtype, const float* y, long long n, float* loss, float* dz, void* dz_lp,
                      double* sum_into, hipStream_t stream);

// ---------------------------------------------------------------- exact-fp32 MFMA GEMM (gemm_f32.hip)
// C[M, N] (+)= epi(sum_k A(m, k) B(n, k)); A layout la: 0 = [M][K] (lda), 1 = [K][M]; B layout
// lb: 0 = [N][K] (ldb), 1 = [K][N].  maskA (same layout / ld as A, optional): A(m, k) counts only
// where maskA > 0 (the ReLU mask of a backward).  Epilogue: + bias[n], ReLU, accumulate into C.
struct GemmF32Args {
  const float* A;
  const float* B;
  const float* maskA;
  const float* bias;
  float* C;
  int M, N, K;
  long long lda, ldb, ldc;
  int relu;
  int accumulate;
  // optional: rowsum[m] (+)= sum_k A'(m, k), A' = A after the mask (the wgrad's bias gradient,
  // sum over the batch of g = dy * 1[y > 0]); (+)= follows `accumulate`
  float* rowsum;
  // optional: the product masked by 1[maskC > 0] ([M, N], row stride N) before it is stored or
  // accumulated -- a dgrad writing the ReLU-masked gradient of the layer below directly
  const float* maskC;
  // optional split-K across workgroups (gemm_f32_split; the 64x64 K-split-4 tile, no rowsum):
  // `split` workgroups per output tile, each over 1/split of K; partial tiles go to sk_slab
  // (tiles * split * 4096 floats) and the last of a tile's workgroups to arrive (counter
  // sk_flags[tile], zero before and after every launch) sums them in slice order, then runs the
  // epilogue.  split <= 1: off.
  float* sk_slab;
  int* sk_flags;
  int split;
};
// wave tile / workgroup shape: 128x64 waves in 2x2 (256x128 tiles), 64x64 waves in 2x2 (128x128),
// 64x64 waves 1x2 with K split 2 (64x128), 64x64 waves with K split 4 (64x64)
enum GemmF32Cfg : int { kF32Wave128 = 0, kF32Wave64 = 1, kF32Wave64Split2 = 2, kF32Wave64Split4 = 3 };
struct GemmF32Plan {
  int cfg = kF32Wave64Split4;
};
// force_cfg >= 0: that configuration (A/B knob); else the largest wave tile that still gives every
// SIMD a wave
GemmF32Plan gemm_f32_plan(int M, int N, int K, int force_cfg = -1);
// workgroups per output tile for the cross-workgroup split-K of a small grid under `plan` (1: none);
// force >= 1 caps it (1 = off), force < 0 = the shape rule
int gemm_f32_split(int M, int N, int K, const GemmF32Plan& plan, int force = -1);
hipError_t gemm_f32(const GemmF32Args& a, int la, int lb, const GemmF32Plan& plan, hipStream_t stream);
// db[n] (+)= sum_m dy[m][n] * (y ? 1[y[m][n] > 0] : 1) over row slices (part: slices * N floats)
int colsum_f32_slices(int M, int N);
hipError_t colsum_f32(const float* dy, const float* y, float* db, float* part, int M, int N, int slices,
                      bool accumulate, hipStream_t stream);

// ---------------------------------------------------------------- IPC one-shot all-reduce
// in[n] (fp32) from every rank -> out[n] = scale * sum over ranks (rank order, identical bits on
// every rank).  Uses the Exchange mailboxes; n <= ex.stride.
hipError_t oneshot_allreduce(const float* in, float* out, long long n, float scale, const Exchange& ex,
                             int* status, hipStream_t stream, int reps = 1);

// ---------------------------------------------------------------- bf16 MFMA GEMM (gemm.hip)
enum GemmEpilogue : int {
  kEpiBias = 1,        // + bias[n] (fp32)
  kEpiRelu = 2,        // max(., 0)
  kEpiMask = 4,        // * 1[mask[m][n] > 0]   (mask: bf16 [M, N], row stride ldmask)
  kEpiStoreT = 8,      // also write C^T (bf16, row stride ldct)
  kEpiOutF32 = 16,     // C is fp32 (else bf16)
  kEpiAccumulate = 32, // C += result (fp32, or bf16 summed in fp32 and rounded once)
  kEpiBKN = 64,        // B is given as [K, N] (N contiguous): C = A . B, read with transposed LDS reads
  kEpiAdam = 128,      // C is a weight GRADIENT consumed in place: Adam updates adam.master / m / v [M, ldc]
                       // and writes the bf16 copy adam.lp; no gradient is stored (single-rank ZeRO-0)
  kEpiColSum = 256,    // with kEpiStoreT, 128x128 kernels: colsum[m0 / 128][n] = sum over the tile's 128
                       // rows of the (bf16-rounded, masked) output: bias-gradient partials, fixed order
};

struct GemmAdam {      // kEpiAdam: fp32 master, moments and the bf16 compute copy of the [M, N] weight
  float* master;
  float* m;
  float* v;
  void* lp;            // bf16
  AdamHyper hp;
  float step_size_neg; // -lr / (1 - beta1^t)
  float bc2_sqrt;      // sqrt(1 - beta2^t)
};

struct GemmArgs {      // C[M,N] = alpha * A[M,K] . B[N,K]^T (+ epilogue); bf16 A/B, fp32 accumulate
                       // (kEpiBKN: B is [K,N] and C = alpha * A . B)
  const void* A;
  const void* B;
  void* C;             // bf16 or fp32 [M, ldc]; may be null when only C^T is wanted
  void* CT;            // bf16 [N, ldct]
  const void* bias;     // fp32, or bf16 when bias_bf16
  int bias_bf16;
  int adam_nt;         // kEpiAdam: nontemporal optimizer-state accesses
  const void* mask;
  int M, N, K;
  int lda, ldb, ldc, ldct, ldmask;
  float alpha;
  GemmAdam adam;       // kEpiAdam only (the gradient is alpha * A . B^T; ldc = row stride of the weight)
  float* colsum;       // kEpiColSum: fp32 [M / 128, N]
  float* sk_slab;      // split-K kernel (variant 9): 4 fp32 128 x 128 partials per tile (per row half:
                       // the publisher's, a finisher's that gave up)
  int* sk_flags;       // split-K kernel: 4 ints per tile (a state word per 128-row half, 2 spare), zero
                       // between launches
  int skn_split;       // 128 x 128 split-K mode (variant 10): blocks per tile
  int sk_xs;           // split-K kernel: bit 0 = a tile's two K halves on neighbouring XCDs (else one XCD);
                       // bits 1-2: timing diagnostics (gemm.hip), wrong results; bit 3: finishers never
                       // wait (the hand-over paths, for tests)
};

hipError_t gemm_nt(const GemmArgs& g, int epilogue, hipStream_t stream, int variant = 0);
// the 128 x 128 split-K mode (variant 10; the shape rule's choice for grids of <= 128 tiles): its
// split for these arguments (0: does not apply); the caller sets skn_split to it and provides
// sk_slab (tiles x split x 128 x 128 fp32) and sk_flags (tiles ints, zero between launches)
int gemm_nt_skn_split(const GemmArgs& g, int epilogue);
int gemm_nt_uses_skn(const GemmArgs& g, int epilogue, int variant);
// the 256 x 256 kernel's split-K 2 mode (variant 11; the shape rule's for 100-128 tiles of 256 x 256):
// 1 if it runs for these arguments (the caller provides sk_slab: tiles x 2 x 256 x 256 fp32, sk_flags:
// tiles ints)
int gemm_nt_uses_spk256(const GemmArgs& g, int epilogue, int variant);
// whether a [K, N]-B product should be run as NT on B^T (a grid larger than the chip; the caller
// transposes B into a [N, K] workspace with transpose_bf16 and calls gemm_nt without kEpiBKN)
bool gemm_nt_kn_transposes(const GemmArgs& g, int epilogue, int variant);
// the split-K kernel's shape rule (256 x 128 tiles, a multiple of 8 of them, K % 128 == 0, staged
// bf16 epilogue); the caller provides sk_slab / sk_flags for (M / 256) * (N / 128) tiles
bool gemm_nt_sk_fits(const GemmArgs& g, int epilogue);
// whether gemm_nt(g, epilogue, ., variant) runs the split-K kernel (needs its workspace)
bool gemm_nt_uses_sk(const GemmArgs& g, int epilogue, int variant);
hipError_t transpose_bf16(const void* in, void* out, int rows, int cols, hipStream_t stream);
// out (fp32, or bf16 when out_bf16) [rows] (+)= row sums of a bf16 [rows, cols] matrix
hipError_t rowsum_bf16(const void* in, void* out, int out_bf16, int rows, int cols, int accumulate,
                       hipStream_t stream);

// ---------------------------------------------------------------- skinny bf16 Linear (head.hip)
// The binary head of an MLP (Linear(K, N), N <= 4) in bf16 for the engine's MFMA chain:
//   forward   z[M, N] = a[M, K] . W[N, K]^T + b           (bf16 in / out, fp32 accumulation)
//   backward  g[M, K] = (dz . W) * 1[a > 0] (mask optional), g^T[K, M] (optional),
//             dW[N, K] (+)= dz^T . a, db[N] (+)= sum_m dz (fp32, or bf16 when dw_bf16: summed in fp32,
//             rounded once; accumulate = 0 stores); part_ws: fp32 [M / 64, N, K] workspace (per-row-tile
//             dW partials, summed in a fixed order: no atomics); bias_part (optional): fp32 [M / 64, K]
//             per-row-tile column sums of g (the layer below's bias-gradient partials); dW == nullptr:
//             part_ws is left to the caller to reduce (db is still formed)
hipError_t skinny_fwd_bf16(const void* a, const void* W, const void* b, void* z, int M, int N, int K,
                           hipStream_t stream);
hipError_t skinny_bwd_bf16(const void* dz, const void* a, const void* W, int mask, void* g, void* gT, void* dW,
                           void* db, int dw_bf16, int accumulate, float* part_ws, int M, int N, int K,
                           hipStream_t stream, float* bias_part = nullptr);

// fp32 skinny Linear (N <= 4) for the engine's fp32 Linear path: z = act(a . W^T + b) (K % 4);
// backward g = dz * 1[y > 0] (y optional), dx = (g . W) * 1[a > 0] (mask; dx optional),
// dW (+)= g^T a via part_ws [M / 64, N, K] + the fixed-order partials_reduce, db (+)= sum g (optional);
// M % 64, K % 32
hipError_t skinny_f32_fwd(const float* a, const float* W, const float* b, float* z, int M, int N, int K, int relu,
                          hipStream_t stream);
hipError_t skinny_f32_bwd(const float* dz, const float* y, const float* a, const float* W, int mask, float* dx,
                          float* dW, float* db, int accumulate, float* part_ws, int M, int N, int K,
                          hipStream_t stream);

// out[i] (+)= sum over t = 0 .. tiles-1 (in this order) of part[t * n + i]: the fixed-order reduction of
// per-tile partials that replaces float atomics (bit-reproducible gradients); out fp32 or bf16
// (out_bf16); n % 4 == 0, aligned
hipError_t partials_reduce(const float* part, void* out, int out_bf16, int tiles, int n, int accumulate,
                           hipStream_t stream);

struct HeadArgs {      // binary head of the synthetic MLP: Linear(D, 1) + BCE-with-logits (mean)
  const void* a;       // bf16 [B, D] last hidden activation
  const float* w;      // fp32 [D]
  const float* b0;     // fp32 [1]
  const float* y;      // fp32 [B]
  int B, D;
  float* dz;           // fp32 [B]
  float* dw;           // fp32 [D]  (overwritten)
  float* db;           // fp32 [1]  (overwritten)
  double* loss_acc;    // += mean loss
  float* scratch;      // fp32 [B + (B / 64) * D] workspace: per-row loss terms, then per-row-tile dw partials
  void* g;             // bf16 [B, D] gradient wrt the last pre-activation
  void* gT;            // bf16 [D, B]
  float* dw_part;      // optional fp32 [B / 64, D]: the dw partials land here and are NOT reduced (the
                       // caller's partials_reduce_multi does it, with other sums, in one launch)
  float* bias_part;    // optional fp32 [B / 64, D]: per-row-tile column sums of g (the gradient of the
                       // last hidden layer's bias, before its reduction)
};

hipError_t mlp_head(const HeadArgs& h, hipStream_t stream);

// Several fixed-order partial reductions in ONE launch: out_s[i] (+)= sum over t (in order) of
// part_s[t][i] (fp32 partials; fp32 or bf16 out), for up to kMaxReduceSegs segments s (n_s % 4 == 0,
// partials 16-byte aligned, outs 16 (fp32) or 8 (bf16) byte aligned).
constexpr int kMaxReduceSegs = 8;
struct ReduceSegs {
  const float* part[kMaxReduceSegs];
  void* out[kMaxReduceSegs];     // fp32, or bf16 (flag 1: the sum in fp32, rounded once)
  int tiles[kMaxReduceSegs];
  int n[kMaxReduceSegs];
  int flags[kMaxReduceSegs];     // 1 = bf16 out, 2 = accumulate into out
  int count;
};
// Optional Adam on the reduced values (a single-rank small region: nothing reduces it across
// ranks): element o = (out_s - grads) + i of master / m / v takes torch's Adam step with gradient
// grad_scale * sum, exactly as adam_flat would over the same region.
struct ReduceAdam {
  int on;
  const float* grads;  // base of the region the outs live in
  float* master;
  float* m;
  float* v;
  AdamHyper hp;
  float step_size_neg, bc2_sqrt, grad_scale;
};
hipError_t partials_reduce_multi(const ReduceSegs& r, const ReduceAdam& adam, hipStream_t stream);

// data.hip: rows idx[0..n_out) of up to kMaxGather row-major tensors (row_words 4-byte words per
// row, n_rows rows each) into contiguous outputs, one launch.
constexpr int kMaxGather = 4;
struct GatherArgs {
  const long long* idx;
  long long n_rows;
  const void* src[kMaxGather];
  void* dst[kMaxGather];
  int row_words[kMaxGather];
  int count;
  int vec_mask;  // bit t: tensor t's rows are 16-byte words at 16-byte-aligned addresses
  int* bad;  // optional: set to 1 when an index is out of range
};
hipError_t gather_rows(const GatherArgs& a, int n_out, hipStream_t stream);

// comm.hip: dst[i] = float(src[i]) for a bf16 src (the gradient bucket's wire cast to fp32), n
// elements, 16-byte vectors where both pointers allow.
hipError_t widen_bf16_f32(const void* src, float* dst, long long n, hipStream_t stream);

}  // namespace dgt
