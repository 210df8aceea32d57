// torch.ops.dgt.* bindings for the MI355X kernels and the IPC runtime.
// Host-only translation unit: validates shapes/devices, picks the current HIP stream, and calls
// the launch functions declared in dgt_kernels.h.  Every op fails loudly on a non-GPU tensor.
// Reference: the ops that replace train.py:85 (Adam), train.py:107/113 (forward/backward), train.py:113 (all-reduce).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/extension.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include "dgt_kernels.h"

namespace {

#define DGT_CHECK_HIP(expr)                                                               \
  do {                                                                                    \
    hipError_t err_ = (expr);                                                             \
    TORCH_CHECK(err_ == hipSuccess, "HIP error ", hipGetErrorString(err_), " in ", #expr); \
  } while (0)

void check_gpu(const at::Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), "dgt: ", name, " must be a GPU (HIP) tensor");
  TORCH_CHECK(t.scalar_type() == dt, "dgt: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "dgt: ", name, " must be contiguous");
}

hipStream_t stream_of(const at::Tensor& t) {
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

dgt::AdamHyper make_hyper(double lr, double beta1, double beta2, double eps, double wd, bool adamw) {
  dgt::AdamHyper h;
  h.lr = (float)lr;
  h.beta2 = (float)beta2;
  h.one_minus_beta1 = (float)(1.0 - beta1);
  h.one_minus_beta2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.weight_decay = (float)wd;
  h.decay = (float)(1.0 - lr * wd);
  h.adamw = adamw ? 1 : 0;
  return h;
}

// zero1 / line: the fused kernel's exchange shape (ZeRO-1 or one-shot) and line format (3 = LL3,
// 2 = LL2), chosen by the trainer (runtime/tiny_trainer.py) and the same on every rank
dgt::Exchange make_exchange(c10::ArrayRef<int64_t> data_ptrs, int64_t rank, int64_t world_size, int64_t stride,
                            int64_t seq_base, int64_t timeout_ticks, int64_t zero1 = 0, int64_t line = 3,
                            int64_t xsum = 0) {
  dgt::Exchange ex;
  std::memset(&ex, 0, sizeof(ex));
  TORCH_CHECK(world_size >= 1 && world_size <= dgt::kMaxRanks, "dgt: world_size must be in [1, 8], got ", world_size);
  TORCH_CHECK(rank >= 0 && rank < world_size, "dgt: bad rank ", rank);
  ex.rank = (int)rank;
  ex.world_size = (int)world_size;
  ex.stride = (int)stride;
  ex.seq_base = seq_base;
  ex.timeout_ticks = timeout_ticks;
  ex.corrupt_step = -1;
  TORCH_CHECK(line == 2 || line == 3, "dgt: exchange line format must be 2 (LL2) or 3 (LL3), got ", line);
  ex.zero1 = zero1 ? 1 : 0;
  ex.line = (int)line;
  TORCH_CHECK(xsum % 4 == 0, "dgt: misaligned ZeRO-1 checksum buffer");
  ex.xsum = reinterpret_cast<unsigned*>(xsum);  // caller-owned int32 [2 * threads] on the device (0 = off)
  if (world_size > 1) {
    TORCH_CHECK((int64_t)data_ptrs.size() == world_size, "dgt: need one mailbox pointer per rank");
    TORCH_CHECK(stride > 0 && stride % 256 == 0, "dgt: mailbox stride must be a positive multiple of 256 floats");
    for (int64_t i = 0; i < world_size; ++i) {
      TORCH_CHECK(data_ptrs[i] != 0, "dgt: null mailbox pointer for rank ", i);
      ex.data[i] = reinterpret_cast<unsigned*>(data_ptrs[i]);
    }
  }
  return ex;
}

int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return dgt::kF32;
    case at::kBFloat16: return dgt::kBF16;
    case at::kHalf: return dgt::kF16;
    default: TORCH_CHECK(false, "dgt: unsupported dtype ", t);
  }
}

// ------------------------------------------------------------------------------ tiny MLP
bool tiny_mlp_supported(int64_t f, int64_t h) { return dgt::tiny_mlp_supported((int)f, (int)h); }
int64_t tiny_mlp_padded_numel(int64_t f, int64_t h) { return dgt::tiny_mlp_padded_numel((int)f, (int)h); }
int64_t tiny_mlp_exchange_floats(int64_t f, int64_t h) { return dgt::tiny_mlp_exchange_floats((int)f, (int)h); }

void tiny_mlp_train(const at::Tensor& X, const at::Tensor& Y, const at::Tensor& plan, const at::Tensor& counts,
                    const at::Tensor& params, const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq,
                    const at::Tensor& loss_acc, const at::Tensor& status, int64_t n_features, int64_t hidden,
                    double lr, double beta1, double beta2, double eps, double weight_decay, bool adamw,
                    int64_t adam_step0, c10::ArrayRef<int64_t> data_ptrs,
                    int64_t rank, int64_t world_size, int64_t stride, int64_t seq_base, int64_t timeout_ticks,
                    int64_t corrupt_step, const std::optional<at::Tensor>& workspace, int64_t zero1,
                    int64_t line, int64_t xsum) {
  TORCH_CHECK(dgt::tiny_mlp_supported((int)n_features, (int)hidden), "dgt: no fused kernel for F=", n_features,
              " H=", hidden);
  TORCH_CHECK(beta1 > 0.5 && beta1 < 1.0 && beta2 > 0.0 && beta2 < 1.0, "dgt: fused kernel needs 0.5 < beta1 < 1");
  check_gpu(X, "X", at::kFloat);
  check_gpu(Y, "Y", at::kFloat);
  check_gpu(plan, "plan", at::kInt);
  check_gpu(counts, "counts", at::kInt);
  check_gpu(params, "params", at::kFloat);
  check_gpu(exp_avg, "exp_avg", at::kFloat);
  check_gpu(exp_avg_sq, "exp_avg_sq", at::kFloat);
  check_gpu(loss_acc, "loss_acc", at::kDouble);
  check_gpu(status, "status", at::kInt);
  const int64_t pp = dgt::tiny_mlp_padded_numel((int)n_features, (int)hidden);
  TORCH_CHECK(params.numel() >= pp && exp_avg.numel() >= pp && exp_avg_sq.numel() >= pp,
              "dgt: flat buffers need ", pp, " elements");
  TORCH_CHECK(X.dim() == 2 && X.size(1) == n_features, "dgt: X must be [N, ", n_features, "]");
  TORCH_CHECK(Y.numel() == X.size(0), "dgt: Y must have one label per row of X");
  TORCH_CHECK(plan.dim() == 2 && plan.size(1) >= 1 && plan.size(1) <= 16, "dgt: plan must be [steps, bmax<=16]");
  TORCH_CHECK(counts.numel() == plan.size(0), "dgt: counts must have one entry per plan row");
  c10::DeviceGuard guard(X.device());
  dgt::TinyTrainArgs a;
  a.X = X.data_ptr<float>();
  a.Y = Y.data_ptr<float>();
  a.plan = plan.data_ptr<int>();
  a.counts = counts.data_ptr<int>();
  a.n_steps = (int)plan.size(0);
  a.bmax = (int)plan.size(1);
  a.params = params.data_ptr<float>();
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
  a.lr = lr;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.adam_step0 = adam_step0;
  // the kernel writes its steps' Adam bias corrections here (+1 row: the loop reads a step ahead);
  // a caller-owned workspace keeps allocation (a hipMalloc on a cache miss) off the launch path
  const int64_t bc_need = (plan.size(0) + 1) * 2;
  at::Tensor bc;
  if (workspace.has_value() && workspace->defined()) {
    check_gpu(*workspace, "workspace", at::kFloat);
    TORCH_CHECK(workspace->numel() >= bc_need, "dgt: tiny_mlp_train workspace needs ", bc_need, " floats");
    bc = *workspace;
  } else {
    bc = at::empty({bc_need}, X.options());
  }
  a.bc = bc.data_ptr<float>();
  a.loss_acc = loss_acc.data_ptr<double>();
  a.status = status.data_ptr<int>();
  a.ex = make_exchange(data_ptrs, rank, world_size, stride, seq_base, timeout_ticks, zero1, line, xsum);
  a.ex.corrupt_step = corrupt_step;
  a.stamps = nullptr;
  if (world_size > 1) {
    const int64_t need = dgt::tiny_mlp_exchange_floats((int)n_features, (int)hidden);
    TORCH_CHECK(stride >= need && stride % 4 == 0, "dgt: mailbox stride ", stride, " < ", need);
  }
  if (a.n_steps == 0) return;
  DGT_CHECK_HIP(dgt::tiny_mlp_train((int)n_features, (int)hidden, a, stream_of(X)));
}

// ------------------------------------------------------------------------------ lean fused launcher
// The per-epoch (and bench) launch of the fused trainer without the dispatcher: everything that is
// fixed for a trainer (tensors, hyper-parameters, mailboxes, stream) is validated and packed ONCE
// into a heap TinyTrainArgs; each launch then passes only the plan, the step count and the
// sequence numbers through a plain C entry point (dgt_tiny_launch, called with ctypes), so the
// host cost of a launch is hipLaunchKernel itself.
struct TinyLauncher {
  dgt::TinyTrainArgs a;
  int f, h, device;
  hipStream_t stream;
};

// dgt_tiny_prepare: one plan's complete argument block and the resolved kernel, so that
// dgt_tiny_launch_prepared passes only the step base and sequence number
struct TinyPrepared {
  dgt::TinyTrainArgs a;
  hipFunction_t fn;
  int threads, device;
  hipStream_t stream;
};

int64_t tiny_launcher_create(const at::Tensor& X, const at::Tensor& Y, const at::Tensor& params,
                             const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq, const at::Tensor& loss_acc,
                             const at::Tensor& status, int64_t n_features, int64_t hidden, double lr, double beta1,
                             double beta2, double eps, double weight_decay, bool adamw,
                             c10::ArrayRef<int64_t> data_ptrs, int64_t rank, int64_t world_size, int64_t stride,
                             int64_t timeout_ticks, int64_t corrupt_step, int64_t zero1, int64_t line,
                             int64_t xsum) {
  TORCH_CHECK(dgt::tiny_mlp_supported((int)n_features, (int)hidden), "dgt: no fused kernel for F=", n_features,
              " H=", hidden);
  TORCH_CHECK(beta1 > 0.5 && beta1 < 1.0 && beta2 > 0.0 && beta2 < 1.0, "dgt: fused kernel needs 0.5 < beta1 < 1");
  check_gpu(X, "X", at::kFloat);
  check_gpu(Y, "Y", at::kFloat);
  check_gpu(params, "params", at::kFloat);
  check_gpu(exp_avg, "exp_avg", at::kFloat);
  check_gpu(exp_avg_sq, "exp_avg_sq", at::kFloat);
  check_gpu(loss_acc, "loss_acc", at::kDouble);
  check_gpu(status, "status", at::kInt);
  const int64_t pp = dgt::tiny_mlp_padded_numel((int)n_features, (int)hidden);
  TORCH_CHECK(params.numel() >= pp && exp_avg.numel() >= pp && exp_avg_sq.numel() >= pp,
              "dgt: flat buffers need ", pp, " elements");
  TORCH_CHECK(X.dim() == 2 && X.size(1) == n_features, "dgt: X must be [N, ", n_features, "]");
  TORCH_CHECK(Y.numel() == X.size(0), "dgt: Y must have one label per row of X");
  if (world_size > 1) {
    const int64_t need = dgt::tiny_mlp_exchange_floats((int)n_features, (int)hidden);
    TORCH_CHECK(stride >= need && stride % 4 == 0, "dgt: mailbox stride ", stride, " < ", need);
  }
  auto* L = new TinyLauncher();
  std::memset(&L->a, 0, sizeof(L->a));
  L->a.X = X.data_ptr<float>();
  L->a.Y = Y.data_ptr<float>();
  L->a.params = params.data_ptr<float>();
  L->a.exp_avg = exp_avg.data_ptr<float>();
  L->a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  L->a.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
  L->a.lr = lr;
  L->a.beta1 = beta1;
  L->a.beta2 = beta2;
  L->a.loss_acc = loss_acc.data_ptr<double>();
  L->a.status = status.data_ptr<int>();
  L->a.ex = make_exchange(data_ptrs, rank, world_size, stride, 0, timeout_ticks, zero1, line, xsum);
  L->a.ex.corrupt_step = corrupt_step;
  L->a.stamps = nullptr;
  L->f = (int)n_features;
  L->h = (int)hidden;
  L->device = (int)X.device().index();
  L->stream = stream_of(X);
  return reinterpret_cast<int64_t>(L);
}

void tiny_launcher_destroy(int64_t handle) { delete reinterpret_cast<TinyLauncher*>(handle); }

// the fused kernel's exchange alone, n_steps times, with torn-line-revealing payloads (tiny_mlp.hip)
void tiny_xch_stress(int64_t n_features, int64_t hidden, c10::ArrayRef<int64_t> data_ptrs, int64_t rank,
                     int64_t world_size, int64_t stride, int64_t seq_base, int64_t timeout_ticks, int64_t line,
                     int64_t n_steps, const at::Tensor& status, const at::Tensor& errors) {
  TORCH_CHECK(dgt::tiny_mlp_supported((int)n_features, (int)hidden), "dgt: no fused kernel for F=", n_features,
              " H=", hidden);
  TORCH_CHECK(world_size >= 2 && n_steps >= 1, "dgt: the exchange stress test needs 2+ ranks and 1+ steps");
  check_gpu(status, "status", at::kInt);
  check_gpu(errors, "errors", at::kInt);
  const int64_t need = dgt::tiny_mlp_exchange_floats((int)n_features, (int)hidden);
  TORCH_CHECK(stride >= need && stride % 4 == 0, "dgt: mailbox stride ", stride, " < ", need);
  c10::DeviceGuard guard(status.device());
  const dgt::Exchange ex = make_exchange(data_ptrs, rank, world_size, stride, seq_base, timeout_ticks, 0, line);
  DGT_CHECK_HIP(dgt::tiny_xch_stress((int)n_features, (int)hidden, ex, (int)n_steps, status.data_ptr<int>(),
                                     errors.data_ptr<int>(), stream_of(status)));
}

}  // namespace

// C entry points (ctypes): the per-launch arguments only.  ``workspace`` holds >= 2 (n_steps + 1)
// floats (the caller sizes it).  Returns a hipError_t (0 = launched).
extern "C" int dgt_tiny_launch(int64_t handle, int64_t plan, int64_t counts, int n_steps, int bmax,
                               long long step0, long long seq_base, int64_t workspace) {
  auto* L = reinterpret_cast<TinyLauncher*>(handle);
  if (!L || !plan || !counts || !workspace || n_steps < 0 || bmax < 1 || bmax > 16) return (int)hipErrorInvalidValue;
  if (n_steps == 0) return 0;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return (int)hipErrorInvalidDevice;
  if (cur != L->device && hipSetDevice(L->device) != hipSuccess) return (int)hipErrorInvalidDevice;
  dgt::TinyTrainArgs a = L->a;
  a.plan = reinterpret_cast<const int*>(plan);
  a.counts = reinterpret_cast<const int*>(counts);
  a.n_steps = n_steps;
  a.bmax = bmax;
  a.adam_step0 = step0;
  a.bc = reinterpret_cast<float*>(workspace);
  a.ex.seq_base = seq_base;
  const hipError_t e = dgt::tiny_mlp_train(L->f, L->h, a, L->stream);
  if (cur != L->device) (void)hipSetDevice(cur);
  return (int)e;
}

// Bind one plan (device pointers, step count, row bound, workspace) and the launcher's stream into a
// TinyPrepared and resolve its kernel once; dgt_tiny_launch_prepared then launches it with the
// kernel-argument block passed as a buffer (no per-argument marshalling, no host-function lookup).
// Returns the handle (0 on failure, *err = the hipError_t); free with dgt_tiny_prepared_free.
extern "C" int64_t dgt_tiny_prepare(int64_t handle, int64_t plan, int64_t counts, int n_steps, int bmax,
                                    int64_t workspace, int* err) {
  auto* L = reinterpret_cast<TinyLauncher*>(handle);
  *err = (int)hipErrorInvalidValue;
  if (!L || !plan || !counts || !workspace || n_steps < 1 || bmax < 1 || bmax > 16) return 0;
  auto* P = new TinyPrepared();
  P->a = L->a;
  P->a.plan = reinterpret_cast<const int*>(plan);
  P->a.counts = reinterpret_cast<const int*>(counts);
  P->a.n_steps = n_steps;
  P->a.bmax = bmax;
  P->a.bc = reinterpret_cast<float*>(workspace);
  P->device = L->device;
  P->stream = L->stream;
  const void* k = dgt::tiny_mlp_train_symbol(L->f, L->h, P->a, &P->threads);
  int cur = -1;
  hipError_t e = k ? hipGetDevice(&cur) : hipErrorInvalidValue;
  if (e == hipSuccess && cur != L->device) e = hipSetDevice(L->device);
  if (e == hipSuccess) e = hipGetFuncBySymbol(&P->fn, k);
  if (cur >= 0 && cur != L->device) (void)hipSetDevice(cur);
  *err = (int)e;
  if (e != hipSuccess) {
    delete P;
    return 0;
  }
  return reinterpret_cast<int64_t>(P);
}

extern "C" int dgt_tiny_launch_prepared(int64_t prepared, long long step0, long long seq_base) {
  auto* P = reinterpret_cast<TinyPrepared*>(prepared);
  if (!P) return (int)hipErrorInvalidValue;
  P->a.adam_step0 = step0;
  P->a.ex.seq_base = seq_base;
  size_t size = sizeof(dgt::TinyTrainArgs);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &P->a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
  return (int)hipModuleLaunchKernel(P->fn, 1, 1, 1, (unsigned)P->threads, 1, 1, 0, P->stream, nullptr, extra);
}

extern "C" void dgt_tiny_prepared_free(int64_t prepared) { delete reinterpret_cast<TinyPrepared*>(prepared); }

// Re-target a launcher at another HIP stream (the caller's current stream changed).
extern "C" void dgt_tiny_launcher_set_stream(int64_t handle, int64_t stream) {
  reinterpret_cast<TinyLauncher*>(handle)->stream = reinterpret_cast<hipStream_t>(stream);
}

namespace {

// ------------------------------------------------------------------------------ fused BCE loss
void linear_fwd(const at::Tensor& x, const at::Tensor& W, const std::optional<at::Tensor>& b, const at::Tensor& y,
                bool relu) {
  check_gpu(x, "x", at::kFloat);
  check_gpu(W, "W", at::kFloat);
  check_gpu(y, "y", at::kFloat);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && W.size(1) == x.size(1) && y.dim() == 2 && y.size(0) == x.size(0) &&
                  y.size(1) == W.size(0),
              "dgt: linear_fwd shapes: x [M, K], W [N, K], y [M, N]");
  const float* bp = nullptr;
  if (b.has_value() && b->defined()) {
    check_gpu(*b, "b", at::kFloat);
    TORCH_CHECK(b->numel() == W.size(0), "dgt: linear_fwd bias must have N elements");
    bp = b->data_ptr<float>();
  }
  if (x.size(0) == 0) return;
  c10::DeviceGuard guard(x.device());
  DGT_CHECK_HIP(dgt::linear_fwd(x.data_ptr<float>(), W.data_ptr<float>(), bp, y.data_ptr<float>(), (int)x.size(0),
                                (int)W.size(0), (int)W.size(1), relu, stream_of(x)));
}

// the two-layer chain in one launch (linear.hip linear2_*): x [M, K], W1 [H, K], W2 [O, H]
float* opt_f32(const std::optional<at::Tensor>& t, const char* name, int64_t numel) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_gpu(*t, name, at::kFloat);
  TORCH_CHECK(t->numel() == numel, "dgt: linear2 ", name, " has ", t->numel(), " elements, expected ", numel);
  return t->data_ptr<float>();
}

bool linear2_fits(int64_t M, int64_t K, int64_t H, int64_t O) {
  return M < (1 << 30) && K < (1 << 30) && H < (1 << 30) && O < (1 << 30) &&
         dgt::linear2_fits((int)M, (int)K, (int)H, (int)O);
}

void linear2_fwd(const at::Tensor& x, const at::Tensor& W1, const std::optional<at::Tensor>& b1, const at::Tensor& W2,
                 const std::optional<at::Tensor>& b2, const at::Tensor& h, const at::Tensor& y, bool relu1, bool relu2) {
  for (const at::Tensor* t : {&x, &W1, &W2, &h, &y}) check_gpu(*t, "linear2 operand", at::kFloat);
  const int64_t M = x.size(0), K = x.size(1), H = W1.size(0), O = W2.size(0);
  TORCH_CHECK(x.dim() == 2 && W1.dim() == 2 && W1.size(1) == K && W2.dim() == 2 && W2.size(1) == H &&
                  h.numel() == M * H && y.numel() == M * O && linear2_fits(M, K, H, O),
              "dgt: linear2_fwd shapes: x [M, K], W1 [H, K], W2 [O, H], h [M, H], y [M, O], M * H <= 4096");
  c10::DeviceGuard guard(x.device());
  DGT_CHECK_HIP(dgt::linear2_fwd(x.data_ptr<float>(), W1.data_ptr<float>(), opt_f32(b1, "b1", H), W2.data_ptr<float>(),
                                 opt_f32(b2, "b2", O), h.data_ptr<float>(), y.data_ptr<float>(), (int)M, (int)K, (int)H,
                                 (int)O, relu1, relu2, stream_of(x)));
}

void linear2_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& W1, const at::Tensor& h,
                 const at::Tensor& W2, const std::optional<at::Tensor>& y, const std::optional<at::Tensor>& dx,
                 const at::Tensor& dW1, const std::optional<at::Tensor>& db1, const at::Tensor& dW2,
                 const std::optional<at::Tensor>& db2, bool relu1, bool acc1, bool acc2) {
  for (const at::Tensor* t : {&dy, &x, &W1, &h, &W2, &dW1, &dW2}) check_gpu(*t, "linear2 operand", at::kFloat);
  const int64_t M = x.size(0), K = x.size(1), H = W1.size(0), O = W2.size(0);
  TORCH_CHECK(x.dim() == 2 && W1.dim() == 2 && W1.size(1) == K && W2.dim() == 2 && W2.size(1) == H &&
                  h.numel() == M * H && dy.numel() == M * O && dW1.sizes() == W1.sizes() &&
                  dW2.sizes() == W2.sizes() && linear2_fits(M, K, H, O),
              "dgt: linear2_bwd shapes: dy [M, O], x [M, K], W1 / dW1 [H, K], h [M, H], W2 / dW2 [O, H]");
  c10::DeviceGuard guard(x.device());
  DGT_CHECK_HIP(dgt::linear2_bwd(dy.data_ptr<float>(), x.data_ptr<float>(), W1.data_ptr<float>(), h.data_ptr<float>(),
                                 W2.data_ptr<float>(), opt_f32(y, "y", M * O), opt_f32(dx, "dx", M * K),
                                 dW1.data_ptr<float>(), opt_f32(db1, "db1", H), dW2.data_ptr<float>(),
                                 opt_f32(db2, "db2", O), (int)M, (int)K, (int)H, (int)O, relu1, acc1, acc2,
                                 stream_of(x)));
}

void linear_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& W, const std::optional<at::Tensor>& y,
                const std::optional<at::Tensor>& dx, const at::Tensor& dW, const std::optional<at::Tensor>& db,
                bool accumulate) {
  check_gpu(dy, "dy", at::kFloat);
  check_gpu(x, "x", at::kFloat);
  check_gpu(W, "W", at::kFloat);
  check_gpu(dW, "dW", at::kFloat);
  const int64_t M = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && W.size(1) == K && dy.dim() == 2 && dy.size(0) == M && dy.size(1) == N &&
                  dW.sizes() == W.sizes(),
              "dgt: linear_bwd shapes: dy [M, N], x [M, K], W / dW [N, K]");
  auto opt = [&](const std::optional<at::Tensor>& t, const char* name, int64_t numel) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    check_gpu(*t, name, at::kFloat);
    TORCH_CHECK(t->numel() == numel, "dgt: linear_bwd ", name, " has ", t->numel(), " elements, expected ", numel);
    return t->data_ptr<float>();
  };
  const float* yp = opt(y, "y", M * N);
  float* dxp = opt(dx, "dx", M * K);
  float* dbp = opt(db, "db", N);
  c10::DeviceGuard guard(x.device());
  DGT_CHECK_HIP(dgt::linear_bwd(dy.data_ptr<float>(), x.data_ptr<float>(), W.data_ptr<float>(), yp, dxp,
                                dW.data_ptr<float>(), dbp, (int)M, (int)N, (int)K, accumulate,
                                stream_of(x)));
}

std::pair<float*, int*> sk_workspace(const at::Tensor& like, hipStream_t stream, int64_t slab_floats,
                                     int64_t flag_ints);  // (below, with the bf16 split-K's)

// Exact-fp32 MFMA GEMM (gemm_f32.hip): C[M, N] (+)= epi(A . B) with A [M, K] (la 0) or [K, M] (la 1),
// B [N, K] (lb 0) or [K, N] (lb 1), all contiguous; one launch (K splits inside the workgroup).
void gemm_f32(const at::Tensor& A, const at::Tensor& B, const std::optional<at::Tensor>& maskA,
              const std::optional<at::Tensor>& bias, const at::Tensor& C, int64_t la, int64_t lb, bool relu,
              bool accumulate, const std::optional<at::Tensor>& rowsum, const std::optional<at::Tensor>& maskC) {
  check_gpu(A, "A", at::kFloat);
  check_gpu(B, "B", at::kFloat);
  check_gpu(C, "C", at::kFloat);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && (la == 0 || la == 1) && (lb == 0 || lb == 1),
              "dgt: gemm_f32 takes 2-D operands and layouts 0 / 1");
  const int64_t M = la == 0 ? A.size(0) : A.size(1), K = la == 0 ? A.size(1) : A.size(0);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1), Kb = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == Kb && C.size(0) == M && C.size(1) == N, "dgt: gemm_f32 shapes: A ", A.sizes(), " (layout ", la,
              "), B ", B.sizes(), " (layout ", lb, "), C ", C.sizes());
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "dgt: gemm_f32 dims must fit in int32");
  dgt::GemmF32Args a{};
  a.A = A.data_ptr<float>();
  a.B = B.data_ptr<float>();
  if (maskA.has_value() && maskA->defined()) {
    check_gpu(*maskA, "maskA", at::kFloat);
    TORCH_CHECK(maskA->sizes() == A.sizes(), "dgt: gemm_f32 maskA must have A's shape");
    a.maskA = maskA->data_ptr<float>();
  }
  if (bias.has_value() && bias->defined()) {
    check_gpu(*bias, "bias", at::kFloat);
    TORCH_CHECK(bias->numel() == N, "dgt: gemm_f32 bias must have N elements");
    a.bias = bias->data_ptr<float>();
  }
  a.C = C.data_ptr<float>();
  if (rowsum.has_value() && rowsum->defined()) {
    check_gpu(*rowsum, "rowsum", at::kFloat);
    TORCH_CHECK(rowsum->numel() == M && rowsum->is_contiguous(), "dgt: gemm_f32 rowsum must have M elements");
    a.rowsum = rowsum->data_ptr<float>();
  }
  if (maskC.has_value() && maskC->defined()) {
    check_gpu(*maskC, "maskC", at::kFloat);
    TORCH_CHECK(maskC->sizes() == C.sizes() && maskC->is_contiguous(), "dgt: gemm_f32 maskC must be C-shaped, contiguous");
    a.maskC = maskC->data_ptr<float>();
  }
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = A.size(1);
  a.ldb = B.size(1);
  a.ldc = N;
  a.relu = relu ? 1 : 0;
  a.accumulate = accumulate ? 1 : 0;
  if (M == 0 || N == 0) return;
  c10::DeviceGuard guard(A.device());
  if (K == 0) {  // an empty sum: the epilogue of zero
    at::Tensor z = at::zeros_like(C);
    if (a.bias) z.add_(*bias);
    if (relu) z.clamp_min_(0.f);
    if (a.maskC) z.mul_(maskC->gt(0.f));
    if (accumulate) C.add_(z); else C.copy_(z);
    if (a.rowsum && !accumulate) rowsum->zero_();
    return;
  }
  // DGT_F32_CFG (A/B knob, read once): force a tile configuration (dgt::GemmF32Cfg)
  static const int force_cfg = [] {
    const char* e = std::getenv("DGT_F32_CFG");
    return e && *e ? std::atoi(e) : -1;
  }();
  // DGT_F32_SPLIT (A/B knob, read once): 0 / 1 = no cross-workgroup split-K, n > 1 = at most n
  static const int force_split = [] {
    const char* e = std::getenv("DGT_F32_SPLIT");
    return e && *e ? std::atoi(e) : -1;
  }();
  const dgt::GemmF32Plan plan = dgt::gemm_f32_plan(a.M, a.N, a.K, force_cfg);
  const hipStream_t stream = stream_of(A);
  a.split = a.rowsum ? 1 : dgt::gemm_f32_split(a.M, a.N, a.K, plan, force_split);
  if (a.split > 1) {
    const int64_t tiles = ((M + 63) / 64) * ((N + 63) / 64);
    std::tie(a.sk_slab, a.sk_flags) = sk_workspace(A, stream, tiles * a.split * 64 * 64, tiles);
  }
  DGT_CHECK_HIP(dgt::gemm_f32(a, (int)la, (int)lb, plan, stream));
}

// db[n] (+)= sum_m dy[m][n] (* 1[y[m][n] > 0]), deterministic two-pass column sum
void colsum_f32(const at::Tensor& dy, const std::optional<at::Tensor>& y, const at::Tensor& db, bool accumulate) {
  check_gpu(dy, "dy", at::kFloat);
  check_gpu(db, "db", at::kFloat);
  TORCH_CHECK(dy.dim() == 2 && db.numel() == dy.size(1), "dgt: colsum_f32 shapes: dy [M, N], db [N]");
  const float* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_gpu(*y, "y", at::kFloat);
    TORCH_CHECK(y->sizes() == dy.sizes(), "dgt: colsum_f32 mask must have dy's shape");
    yp = y->data_ptr<float>();
  }
  const int M = (int)dy.size(0), N = (int)dy.size(1);
  if (N == 0) return;
  c10::DeviceGuard guard(dy.device());
  if (M == 0) {
    if (!accumulate) db.zero_();
    return;
  }
  const int slices = dgt::colsum_f32_slices(M, N);
  at::Tensor part = at::empty({(int64_t)slices * N}, dy.options());
  DGT_CHECK_HIP(dgt::colsum_f32(dy.data_ptr<float>(), yp, db.data_ptr<float>(), part.data_ptr<float>(), M, N, slices,
                                accumulate, stream_of(dy)));
}

void bce_logits(const at::Tensor& z, const at::Tensor& y, const at::Tensor& loss, const at::Tensor& dz,
                const std::optional<at::Tensor>& dz_lp, const std::optional<at::Tensor>& sum_into) {
  TORCH_CHECK(z.is_cuda() && z.is_contiguous() && (z.scalar_type() == at::kFloat || z.scalar_type() == at::kBFloat16),
              "dgt: bce_logits needs contiguous fp32 / bf16 GPU logits");
  check_gpu(y, "y", at::kFloat);
  check_gpu(loss, "loss", at::kFloat);
  check_gpu(dz, "dz", at::kFloat);
  TORCH_CHECK(y.numel() == z.numel() && dz.numel() == z.numel() && loss.numel() == 1 && z.numel() > 0,
              "dgt: bce_logits size mismatch");
  void* lp = nullptr;
  if (dz_lp.has_value()) {
    check_gpu(*dz_lp, "dz_lp", at::kBFloat16);
    TORCH_CHECK(dz_lp->numel() == z.numel(), "dgt: bce_logits dz_lp size mismatch");
    lp = dz_lp->data_ptr();
  }
  double* acc = nullptr;
  if (sum_into.has_value()) {
    check_gpu(*sum_into, "sum_into", at::kDouble);
    TORCH_CHECK(sum_into->numel() == 1, "dgt: bce_logits sum_into must hold one fp64 value");
    acc = sum_into->data_ptr<double>();
  }
  c10::DeviceGuard guard(z.device());
  DGT_CHECK_HIP(dgt::bce_logits(z.data_ptr(), dtype_code(z.scalar_type()), y.data_ptr<float>(), z.numel(),
                                loss.data_ptr<float>(), dz.data_ptr<float>(), lp, acc, stream_of(z)));
}

std::vector<at::Tensor> gather_rows(const at::Tensor& idx, at::TensorList srcs) {
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(),
              "dgt: gather_rows needs a contiguous 1-D int64 GPU index");
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= dgt::kMaxGather, "dgt: gather_rows takes 1..", dgt::kMaxGather,
              " tensors");
  const int64_t n = srcs[0].dim() > 0 ? srcs[0].size(0) : 0;
  dgt::GatherArgs a{};
  a.idx = reinterpret_cast<const long long*>(idx.data_ptr<int64_t>());
  a.n_rows = n;
  a.count = (int)srcs.size();
  std::vector<at::Tensor> outs;
  for (size_t t = 0; t < srcs.size(); ++t) {
    const at::Tensor& s = srcs[t];
    TORCH_CHECK(s.device() == idx.device() && s.is_contiguous() && s.dim() >= 1 && s.size(0) == n,
                "dgt: gather_rows tensors must be contiguous, on the index's device, with the same row count");
    const int64_t row_bytes = n > 0 ? s.numel() / n * (int64_t)s.element_size() : 0;
    TORCH_CHECK(row_bytes % 4 == 0 && row_bytes / 4 < (1 << 30), "dgt: gather_rows rows must be whole 4-byte words");
    auto sizes = s.sizes().vec();
    sizes[0] = idx.numel();
    outs.push_back(at::empty(sizes, s.options()));
    a.src[t] = s.data_ptr();
    a.dst[t] = outs.back().data_ptr();
    a.row_words[t] = (int)(row_bytes / 4);
    if (row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(a.src[t]) % 16 == 0) a.vec_mask |= 1 << t;
  }
  if (idx.numel() == 0 || n == 0 || outs[0].numel() == 0) {
    TORCH_CHECK(idx.numel() == 0, "dgt: gather_rows from an empty tensor");
    return outs;
  }
  c10::DeviceGuard guard(idx.device());
  DGT_CHECK_HIP(dgt::gather_rows(a, (int)idx.numel(), stream_of(idx)));
  return outs;
}

void tiny_mlp_grad(const at::Tensor& X, const at::Tensor& Y, const at::Tensor& plan, const at::Tensor& counts,
                   int64_t step, const at::Tensor& params, const at::Tensor& grad, const at::Tensor& loss_acc,
                   int64_t n_features, int64_t hidden) {
  TORCH_CHECK(dgt::tiny_mlp_supported((int)n_features, (int)hidden), "dgt: no fused kernel for F=", n_features,
              " H=", hidden);
  check_gpu(X, "X", at::kFloat);
  check_gpu(Y, "Y", at::kFloat);
  check_gpu(plan, "plan", at::kInt);
  check_gpu(counts, "counts", at::kInt);
  check_gpu(params, "params", at::kFloat);
  check_gpu(grad, "grad", at::kFloat);
  check_gpu(loss_acc, "loss_acc", at::kDouble);
  const int64_t pp = dgt::tiny_mlp_padded_numel((int)n_features, (int)hidden);
  TORCH_CHECK(params.numel() >= pp && grad.numel() >= pp, "dgt: flat buffers need ", pp, " elements");
  TORCH_CHECK(plan.dim() == 2 && plan.size(1) <= 16 && step >= 0 && step < plan.size(0), "dgt: bad plan/step");
  TORCH_CHECK(X.dim() == 2 && X.size(1) == n_features, "dgt: X must be [N, ", n_features, "]");
  c10::DeviceGuard guard(X.device());
  dgt::TinyGradArgs a;
  a.X = X.data_ptr<float>();
  a.Y = Y.data_ptr<float>();
  a.plan = plan.data_ptr<int>();
  a.counts = counts.data_ptr<int>();
  a.step = (int)step;
  a.bmax = (int)plan.size(1);
  a.params = params.data_ptr<float>();
  a.grad = grad.data_ptr<float>();
  a.loss_acc = loss_acc.data_ptr<double>();
  DGT_CHECK_HIP(dgt::tiny_mlp_grad((int)n_features, (int)hidden, a, stream_of(X)));
}

// ------------------------------------------------------------------------------ Adam
dgt::AdamFlatArgs adam_args(const at::Tensor& master, const std::optional<at::Tensor>& param_lp,
                            const at::Tensor& grad, const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq,
                            double lr, double beta1, double beta2, double eps, double weight_decay, bool adamw,
                            int64_t step, double grad_scale, const std::optional<at::Tensor>& grad_scale_dev,
                            const std::optional<at::Tensor>& step_dev,
                            const std::optional<at::Tensor>& step_ticket = std::nullopt) {
  check_gpu(master, "master", at::kFloat);
  check_gpu(exp_avg, "exp_avg", at::kFloat);
  check_gpu(exp_avg_sq, "exp_avg_sq", at::kFloat);
  TORCH_CHECK(grad.is_cuda() && grad.is_contiguous(), "dgt: grad must be a contiguous GPU tensor");
  const int64_t n = master.numel();
  TORCH_CHECK(n % 4 == 0, "dgt: flat buffers must be padded to a multiple of 4 elements");
  // the kernels move float4 (fp32) and 4 x 16-bit groups: slices must start on such a group
  auto al = [](const void* p, int b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; };
  TORCH_CHECK(al(master.data_ptr(), 16) && al(exp_avg.data_ptr(), 16) && al(exp_avg_sq.data_ptr(), 16),
              "dgt: adam_flat fp32 buffers must be 16-byte aligned (slice offsets a multiple of 4)");
  TORCH_CHECK(al(grad.data_ptr(), 4 * (int)grad.element_size()),
              "dgt: adam_flat grad must be aligned to a 4-element group");
  TORCH_CHECK(grad.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n, "dgt: flat size mismatch");
  const bool dev_step = step_dev.has_value() && step_dev->defined();
  TORCH_CHECK(dev_step || step >= 1, "dgt: adam step must be >= 1");
  dgt::AdamFlatArgs a{};
  a.master = master.data_ptr<float>();
  a.param_lp = nullptr;
  a.lp_dtype = dgt::kF32;
  if (param_lp.has_value() && param_lp->defined()) {
    TORCH_CHECK(param_lp->is_cuda() && param_lp->is_contiguous() && param_lp->numel() == n, "dgt: bad param_lp");
    TORCH_CHECK(al(param_lp->data_ptr(), 4 * (int)param_lp->element_size()),
                "dgt: adam_flat param_lp must be aligned to a 4-element group");
    a.param_lp = param_lp->data_ptr();
    a.lp_dtype = dtype_code(param_lp->scalar_type());
  }
  a.grad = grad.data_ptr();
  a.grad_dtype = dtype_code(grad.scalar_type());
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.n = n;
  a.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
  const double bc1 = 1.0 - std::pow(beta1, (double)std::max<int64_t>(step, 1));
  const double bc2 = 1.0 - std::pow(beta2, (double)std::max<int64_t>(step, 1));
  a.step_size_neg = (float)(-(lr / bc1));
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.grad_scale = (float)grad_scale;
  a.grad_scale_dev = nullptr;
  if (grad_scale_dev.has_value() && grad_scale_dev->defined()) {
    check_gpu(*grad_scale_dev, "grad_scale_dev", at::kFloat);
    a.grad_scale_dev = grad_scale_dev->data_ptr<float>();
  }
  a.step_dev = nullptr;
  a.lr_d = lr;
  a.beta1_d = beta1;
  a.beta2_d = beta2;
  a.step_ticket = nullptr;
  if (dev_step) {
    check_gpu(*step_dev, "step_dev", at::kLong);
    a.step_dev = reinterpret_cast<long long*>(step_dev->data_ptr<int64_t>());
  }
  if (step_ticket.has_value() && step_ticket->defined()) {
    TORCH_CHECK(dev_step, "dgt: adam_flat step_ticket needs step_dev");
    check_gpu(*step_ticket, "step_ticket", at::kInt);
    a.step_ticket = reinterpret_cast<unsigned*>(step_ticket->data_ptr<int32_t>());
  }
  return a;
}

void adam_flat(const at::Tensor& master, const std::optional<at::Tensor>& param_lp, const at::Tensor& grad,
               const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq, double lr, double beta1, double beta2,
               double eps, double weight_decay, bool adamw, int64_t step, double grad_scale,
               const std::optional<at::Tensor>& grad_scale_dev, const std::optional<at::Tensor>& step_dev,
               const std::optional<at::Tensor>& step_ticket) {
  const dgt::AdamFlatArgs a = adam_args(master, param_lp, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps,
                                        weight_decay, adamw, step, grad_scale, grad_scale_dev, step_dev, step_ticket);
  c10::DeviceGuard guard(master.device());
  DGT_CHECK_HIP(dgt::adam_flat(a, stream_of(master)));
}

void step_increment(const at::Tensor& counter) {
  check_gpu(counter, "counter", at::kLong);
  c10::DeviceGuard guard(counter.device());
  DGT_CHECK_HIP(dgt::step_increment(reinterpret_cast<long long*>(counter.data_ptr<int64_t>()), stream_of(counter)));
}

// ------------------------------------------------------------------------------ one-shot all-reduce
void oneshot_allreduce(const at::Tensor& inp, const at::Tensor& out, double scale, c10::ArrayRef<int64_t> data_ptrs,
                       int64_t rank, int64_t world_size, int64_t stride,
                       int64_t seq, int64_t timeout_ticks, const at::Tensor& status, int64_t reps) {
  check_gpu(inp, "inp", at::kFloat);
  check_gpu(out, "out", at::kFloat);
  check_gpu(status, "status", at::kInt);
  TORCH_CHECK(inp.numel() == out.numel() && inp.numel() % 4 == 0 && inp.numel() <= stride,
              "dgt: one-shot all-reduce needs equal sizes, a multiple of 4 and <= mailbox stride");
  c10::DeviceGuard guard(inp.device());
  dgt::Exchange ex = make_exchange(data_ptrs, rank, world_size, stride, seq, timeout_ticks);
  DGT_CHECK_HIP(dgt::oneshot_allreduce(inp.data_ptr<float>(), out.data_ptr<float>(), inp.numel(), (float)scale, ex,
                                       status.data_ptr<int>(), stream_of(inp), (int)reps));
}

// ------------------------------------------------------------------------------ bf16 GEMM + MLP helpers
void check_2d(const at::Tensor& t, const char* name, at::ScalarType dt, int64_t r, int64_t c) {
  check_gpu(t, name, dt);
  TORCH_CHECK(t.dim() == 2 && t.size(0) == r && t.size(1) == c, "dgt: ", name, " must be [", r, ", ", c, "], got ",
              t.sizes());
  // the kernels move whole 16-byte rows pieces (staged GEMM epilogue, vector loads)
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "dgt: ", name, " must be 16-byte aligned");
}

// Workspace of the split-K GEMM (gemm.hip, variant 9): per (device, stream), so launches that may
// run concurrently never share a partial slab or a ticket.  Tensors from the caching allocator (a
// first use inside a graph capture allocates from the graph's pool; the map keeps it alive); the
// ticket words start at zero and every launch leaves them at zero.  The map is never destroyed: its
// tensors must not be freed into the caching allocator during static destruction at exit.
struct SkWorkspace {
  at::Tensor slab, flags;
  at::Tensor bt;  // B^T of a [K, N] operand run as NT (gemm_nt_kn_transposes)
};
std::mutex g_sk_mu;
auto* g_sk_ws = new std::map<std::pair<int, hipStream_t>, SkWorkspace>();

std::pair<float*, int*> sk_workspace(const at::Tensor& like, hipStream_t stream, int64_t slab_floats,
                                     int64_t flag_ints) {
  std::lock_guard<std::mutex> lock(g_sk_mu);
  SkWorkspace& w = (*g_sk_ws)[{(int)like.device().index(), stream}];
  if (!w.slab.defined() || w.slab.numel() < slab_floats || w.flags.numel() < flag_ints) {
    const int64_t sf = std::max<int64_t>(slab_floats, w.slab.defined() ? w.slab.numel() : 0);
    const int64_t fi = std::max<int64_t>(flag_ints, w.flags.defined() ? w.flags.numel() : 0);
    w.slab = at::empty({sf}, like.options().dtype(at::kFloat));
    w.flags = at::zeros({fi}, like.options().dtype(at::kInt));
  }
  return {w.slab.data_ptr<float>(), w.flags.data_ptr<int>()};
}

void attach_sk_workspace(dgt::GemmArgs& g, const at::Tensor& like, hipStream_t stream, int64_t slab_floats,
                         int64_t flag_ints) {
  std::tie(g.sk_slab, g.sk_flags) = sk_workspace(like, stream, slab_floats, flag_ints);
  static const int xs = [] {
    const char* e = std::getenv("DGT_GEMM_SK_XS");
    return (e && *e) ? std::atoi(e) : 1;
  }();
  g.sk_xs = xs;
}

void gemm_nt(const at::Tensor& A, const at::Tensor& B, const std::optional<at::Tensor>& C,
             const std::optional<at::Tensor>& CT, const std::optional<at::Tensor>& bias,
             const std::optional<at::Tensor>& mask, int64_t epi, double alpha, int64_t variant,
             const std::optional<at::Tensor>& colsum) {
  TORCH_CHECK(!(epi & dgt::kEpiBKN) || (variant != 2 && variant != 8),
              "dgt: a [K, N] B operand runs on the 128x128 kernels only");
  TORCH_CHECK(variant >= 0 && variant <= 11,
              "dgt: gemm_nt variant must be 0 (auto), 1 (128x128, 2 stages), 2 (256x256), 3 (4 with front-loaded "
              "fragment reads), 4 (128x128, 4 stages, 8 waves), 5 (software-pipelined reads), 6 / 7 (register "
              "prefetch, 2 / 4 K-tiles), 8 (256x256 with cross-phase fragment prefetch), 9 (256x128 split-K 2) or "
              "10 (128x128 split-K for small grids) or 11 (256x256 split-K 2); the round-2 variants live in git history "
              "(commit c0371a5)");
  const bool b_kn = (epi & dgt::kEpiBKN) != 0;
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(b_kn ? 0 : 1),
              b_kn ? "dgt: gemm_nt with kEpiBKN needs A[M,K], B[K,N]" : "dgt: gemm_nt needs A[M,K], B[N,K]");
  const int64_t M = A.size(0), N = B.size(b_kn ? 1 : 0), K = A.size(1);
  for (const at::Tensor* t : {&A, &B}) {  // rows may be strided (column blocks of a wider matrix)
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16, "dgt: gemm_nt operands must be bf16 GPU tensors");
    TORCH_CHECK(t->stride(1) == 1 && t->stride(0) >= t->size(1) && t->stride(0) % 8 == 0,
                "dgt: gemm_nt operand rows must be unit-stride with a 16-byte aligned row stride");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "dgt: gemm_nt operand must be 16-byte aligned");
  }
  TORCH_CHECK(M % 128 == 0 && N % 128 == 0 && K % 64 == 0, "dgt: gemm_nt needs M, N % 128 == 0 and K % 64 == 0 (got ",
              M, "x", N, "x", K, ")");
  dgt::GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.A = A.data_ptr();
  g.B = B.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = (int)A.stride(0);
  g.ldb = (int)B.stride(0);
  g.alpha = (float)alpha;
  if (C.has_value() && C->defined()) {
    check_2d(*C, "C", (epi & dgt::kEpiOutF32) ? at::kFloat : at::kBFloat16, M, N);
    g.C = C->data_ptr();
    g.ldc = (int)N;
  } else {
    TORCH_CHECK(!(epi & dgt::kEpiOutF32) && !(epi & dgt::kEpiAccumulate) && (epi & dgt::kEpiStoreT),
                "dgt: gemm_nt without C must store C^T");
  }
  if (epi & dgt::kEpiStoreT) {
    TORCH_CHECK(CT.has_value() && CT->defined(), "dgt: kEpiStoreT needs CT");
    check_2d(*CT, "CT", at::kBFloat16, N, M);
    g.CT = CT->data_ptr();
    g.ldct = (int)M;
  }
  if (epi & dgt::kEpiBias) {
    TORCH_CHECK(bias.has_value() && bias->defined() && bias->numel() == N, "dgt: bias must have N elements");
    const bool bf = bias->scalar_type() == at::kBFloat16;
    check_gpu(*bias, "bias", bf ? at::kBFloat16 : at::kFloat);
    TORCH_CHECK(bias->is_contiguous(), "dgt: bias must be contiguous");
    g.bias = bias->data_ptr();
    g.bias_bf16 = bf ? 1 : 0;  // a bf16 module's bias as it is: no per-call fp32 copy
  }
  if (epi & dgt::kEpiMask) {
    TORCH_CHECK(mask.has_value() && mask->defined(), "dgt: kEpiMask needs mask");
    check_2d(*mask, "mask", at::kBFloat16, M, N);
    g.mask = mask->data_ptr();
    g.ldmask = (int)N;
  }
  if (colsum.has_value() && colsum->defined()) {  // bias-gradient partials of the (masked) output
    TORCH_CHECK((epi & dgt::kEpiStoreT) && (epi & dgt::kEpiBKN) && (epi & dgt::kEpiMask) && variant != 2,
                "dgt: colsum is formed by the [K, N] dgrad epilogue (mask + C^T) of the 128x128 kernels");
    check_2d(*colsum, "colsum", at::kFloat, M / 128, N);
    g.colsum = colsum->data_ptr<float>();
    epi |= dgt::kEpiColSum;
  }
  c10::DeviceGuard guard(A.device());
  if (variant == 2 || variant == 8)
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0, "dgt: the 256x256 gemm needs M, N % 256 == 0, K % 128 == 0");
  const hipStream_t stream = stream_of(A);
  if (dgt::gemm_nt_kn_transposes(g, (int)epi, (int)variant)) {
    // B [K, N] -> B^T [N, K] in this stream's workspace, then the NT product (256 x 256 kernels)
    void* bt = nullptr;
    {
      std::lock_guard<std::mutex> lock(g_sk_mu);
      SkWorkspace& w = (*g_sk_ws)[{(int)A.device().index(), stream}];
      if (!w.bt.defined() || w.bt.numel() < K * N) w.bt = at::empty({K * N}, A.options());
      bt = w.bt.data_ptr();
    }
    DGT_CHECK_HIP(dgt::transpose_bf16(g.B, bt, (int)K, (int)N, stream));
    g.B = bt;
    g.ldb = (int)K;
    epi &= ~(int64_t)dgt::kEpiBKN;
  }
  const int spk256 = dgt::gemm_nt_uses_spk256(g, (int)epi, (int)variant);
  TORCH_CHECK(variant != 11 || spk256, "dgt: the 256x256 split-K mode (variant 11) needs M, N % 256 == 0, K % 256 == 0, "
              "an [N, K] B and a bf16 (staged) epilogue without column sums");
  const int skn = spk256 ? 0 : dgt::gemm_nt_uses_skn(g, (int)epi, (int)variant);
  TORCH_CHECK(variant != 10 || skn > 0,
              "dgt: the 128x128 split-K mode (variant 10) needs a bf16 (staged) epilogue and a grid of at most 128 "
              "tiles with at least 16 K-tiles");
  if (spk256) {
    const int64_t tiles = (int64_t)(M / 256) * (N / 256);
    attach_sk_workspace(g, A, stream, tiles * 2 * 256 * 256, tiles);
  } else if (skn > 0) {
    g.skn_split = skn;
    const int64_t tiles = (int64_t)(M / 128) * (N / 128);
    attach_sk_workspace(g, A, stream, tiles * skn * 128 * 128, tiles);
  } else if (dgt::gemm_nt_uses_sk(g, (int)epi, (int)variant)) {
    TORCH_CHECK(dgt::gemm_nt_sk_fits(g, (int)epi),
                "dgt: the split-K gemm (variant 9) needs M % 256 == 0, N % 128 == 0, K % 128 == 0, a multiple of 8 "
                "256x128 tiles and a bf16 (staged) epilogue");
    const int64_t tiles = (int64_t)(M / 256) * (N / 128);
    attach_sk_workspace(g, A, stream, tiles * 512 * 128, tiles * 4);
  }
  DGT_CHECK_HIP(dgt::gemm_nt(g, (int)epi, stream, (int)variant));
}

// wgrad + Adam in one launch: the weight gradient alpha * A . B^T ([M, N], never stored) updates the
// fp32 master / exp_avg / exp_avg_sq [M, N] and the bf16 compute copy param_lp [M, N] in place.
void gemm_nt_adam(const at::Tensor& A, const at::Tensor& B, const at::Tensor& master, const at::Tensor& exp_avg,
                  const at::Tensor& exp_avg_sq, const at::Tensor& param_lp, int64_t step, double lr, double beta1,
                  double beta2, double eps, double weight_decay, bool adamw, double grad_scale, int64_t variant) {
  TORCH_CHECK(((variant >= 0 && variant <= 5) || variant == 8) && step >= 1,
              "dgt: gemm_nt_adam needs variant 0 .. 5 or 8 and step >= 1");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "dgt: gemm_nt_adam needs A[M,K], B[N,K]");
  const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
  for (const at::Tensor* t : {&A, &B}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16, "dgt: gemm_nt_adam operands must be bf16 GPU tensors");
    TORCH_CHECK(t->stride(1) == 1 && t->stride(0) >= t->size(1) && t->stride(0) % 8 == 0,
                "dgt: gemm_nt_adam operand rows must be unit-stride with a 16-byte aligned row stride");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "dgt: gemm_nt_adam operand must be 16-byte aligned");
  }
  TORCH_CHECK(M % 128 == 0 && N % 128 == 0 && K % 64 == 0, "dgt: gemm_nt_adam needs M, N % 128 == 0 and K % 64 == 0");
  check_2d(master, "master", at::kFloat, M, N);
  check_2d(exp_avg, "exp_avg", at::kFloat, M, N);
  check_2d(exp_avg_sq, "exp_avg_sq", at::kFloat, M, N);
  check_2d(param_lp, "param_lp", at::kBFloat16, M, N);
  for (const at::Tensor* t : {&master, &exp_avg, &exp_avg_sq, &param_lp})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "dgt: gemm_nt_adam state must be 16-byte aligned");
  if (variant == 2 || variant == 8)
    TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && K % 128 == 0, "dgt: the 256x256 gemm needs M, N % 256 == 0, K % 128 == 0");
  dgt::GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.A = A.data_ptr();
  g.B = B.data_ptr();
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = (int)A.stride(0);
  g.ldb = (int)B.stride(0);
  g.ldc = (int)N;
  g.alpha = (float)grad_scale;
  g.adam.master = master.data_ptr<float>();
  g.adam.m = exp_avg.data_ptr<float>();
  g.adam.v = exp_avg_sq.data_ptr<float>();
  g.adam.lp = param_lp.data_ptr();
  g.adam.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
  const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
  g.adam.step_size_neg = (float)(-(lr / bc1));
  g.adam.bc2_sqrt = (float)std::sqrt(bc2);
  static const int adam_nt = [] {  // nontemporal optimizer-state streams (A/B: DGT_ADAM_EPI_NT=0)
    const char* e = std::getenv("DGT_ADAM_EPI_NT");
    return e ? std::atoi(e) : 1;
  }();
  g.adam_nt = adam_nt;
  c10::DeviceGuard guard(A.device());
  DGT_CHECK_HIP(dgt::gemm_nt(g, dgt::kEpiAdam, stream_of(A), (int)variant));
}

void transpose_bf16(const at::Tensor& in, const at::Tensor& out) {
  TORCH_CHECK(in.dim() == 2, "dgt: transpose needs a 2-d tensor");
  check_2d(in, "in", at::kBFloat16, in.size(0), in.size(1));
  check_2d(out, "out", at::kBFloat16, in.size(1), in.size(0));
  c10::DeviceGuard guard(in.device());
  DGT_CHECK_HIP(dgt::transpose_bf16(in.data_ptr(), out.data_ptr(), (int)in.size(0), (int)in.size(1), stream_of(in)));
}

void rowsum_bf16(const at::Tensor& in, const at::Tensor& out, bool accumulate) {
  TORCH_CHECK(in.dim() == 2 && in.size(1) % 8 == 0, "dgt: rowsum needs [rows, cols % 8 == 0]");
  check_2d(in, "in", at::kBFloat16, in.size(0), in.size(1));
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "dgt: rowsum out must be fp32 or bf16");
  check_gpu(out, "out", out.scalar_type());
  TORCH_CHECK(out.numel() == in.size(0), "dgt: rowsum out must have one entry per row");
  c10::DeviceGuard guard(in.device());
  DGT_CHECK_HIP(dgt::rowsum_bf16(in.data_ptr(), out.data_ptr(), out.scalar_type() == at::kBFloat16 ? 1 : 0,
                                 (int)in.size(0), (int)in.size(1), accumulate ? 1 : 0, stream_of(in)));
}

// skinny bf16 head Linear(K, N <= 4): z = a . W^T + b
void skinny_fwd_bf16(const at::Tensor& a, const at::Tensor& W, const std::optional<at::Tensor>& b,
                     const at::Tensor& z) {
  TORCH_CHECK(a.dim() == 2 && W.dim() == 2 && W.size(1) == a.size(1), "dgt: skinny_fwd needs a [M, K], W [N, K]");
  const int64_t M = a.size(0), K = a.size(1), N = W.size(0);
  TORCH_CHECK(N >= 1 && N <= 4 && K % 8 == 0, "dgt: skinny_fwd needs N <= 4, K % 8 == 0");
  check_2d(a, "a", at::kBFloat16, M, K);
  check_2d(W, "W", at::kBFloat16, N, K);
  check_gpu(z, "z", at::kBFloat16);
  TORCH_CHECK(z.numel() == M * N, "dgt: skinny_fwd z must be [M, N]");
  const void* bp = nullptr;
  if (b.has_value() && b->defined()) {
    check_gpu(*b, "b", at::kBFloat16);
    TORCH_CHECK(b->numel() == N, "dgt: skinny_fwd bias must have N elements");
    bp = b->data_ptr();
  }
  c10::DeviceGuard guard(a.device());
  DGT_CHECK_HIP(dgt::skinny_fwd_bf16(a.data_ptr(), W.data_ptr(), bp, z.data_ptr(), (int)M, (int)N, (int)K,
                                     stream_of(a)));
}

// its backward: g = (dz . W) * 1[a > 0] (mask) and g^T; dW / db accumulate in fp32
void skinny_bwd_bf16(const at::Tensor& dz, const at::Tensor& a, const at::Tensor& W, bool mask, const at::Tensor& g,
                     const std::optional<at::Tensor>& gT, const at::Tensor& dW, const at::Tensor& db,
                     bool accumulate, const std::optional<at::Tensor>& bias_part,
                     const std::optional<at::Tensor>& dw_part) {
  const int64_t M = a.size(0), K = a.size(1), N = W.size(0);
  TORCH_CHECK(a.dim() == 2 && W.dim() == 2 && W.size(1) == K && N >= 1 && N <= 4 && M % 64 == 0 && K % 64 == 0,
              "dgt: skinny_bwd needs a [M, K], W [N <= 4, K], M, K % 64 == 0");
  check_gpu(dz, "dz", at::kBFloat16);
  TORCH_CHECK(dz.numel() == M * N, "dgt: skinny_bwd dz must be [M, N]");
  check_2d(a, "a", at::kBFloat16, M, K);
  check_2d(W, "W", at::kBFloat16, N, K);
  check_2d(g, "g", at::kBFloat16, M, K);
  void* gTp = nullptr;
  if (gT.has_value() && gT->defined()) {
    check_2d(*gT, "gT", at::kBFloat16, K, M);
    gTp = gT->data_ptr();
  }
  const bool bf = dW.scalar_type() == at::kBFloat16;  // the bucket's bf16 gradient views, or fp32
  check_gpu(dW, "dW", bf ? at::kBFloat16 : at::kFloat);
  check_gpu(db, "db", bf ? at::kBFloat16 : at::kFloat);
  TORCH_CHECK(dW.numel() == N * K && db.numel() == N, "dgt: skinny_bwd dW [N, K] and db [N] (one dtype)");
  TORCH_CHECK(dW.is_contiguous(), "dgt: skinny_bwd dW must be contiguous");
  c10::DeviceGuard guard(a.device());
  float* bp = nullptr;  // caller-owned [M / 64, K] column sums of g (the layer below's bias partials)
  if (bias_part.has_value() && bias_part->defined()) {
    check_2d(*bias_part, "bias_part", at::kFloat, M / 64, K);
    bp = bias_part->data_ptr<float>();
  }
  at::Tensor ws;  // per-row-tile dW partials: the caller's (reduced by it later) or this call's scratch
  void* dwp = dW.data_ptr();
  if (dw_part.has_value() && dw_part->defined()) {
    check_2d(*dw_part, "dw_part", at::kFloat, M / 64, N * K);
    ws = *dw_part;
    dwp = nullptr;
  } else {
    ws = at::empty({M / 64, N, K}, a.options().dtype(at::kFloat));
  }
  DGT_CHECK_HIP(dgt::skinny_bwd_bf16(dz.data_ptr(), a.data_ptr(), W.data_ptr(), mask ? 1 : 0, g.data_ptr(), gTp,
                                     dwp, db.data_ptr(), bf ? 1 : 0, accumulate ? 1 : 0,
                                     ws.data_ptr<float>(), (int)M, (int)N, (int)K, stream_of(a), bp));
}

// skinny fp32 Linear(K, N <= 4) (the fp32 engine's MLP head): z = act(a . W^T + b)
void skinny_f32_fwd(const at::Tensor& a, const at::Tensor& W, const std::optional<at::Tensor>& b, const at::Tensor& z,
                    bool relu) {
  TORCH_CHECK(a.dim() == 2 && W.dim() == 2 && W.size(1) == a.size(1), "dgt: skinny_f32_fwd needs a [M, K], W [N, K]");
  const int64_t M = a.size(0), K = a.size(1), N = W.size(0);
  TORCH_CHECK(N >= 1 && N <= 4 && K % 4 == 0 && M > 0, "dgt: skinny_f32_fwd needs N <= 4, K % 4 == 0");
  check_2d(a, "a", at::kFloat, M, K);
  check_2d(W, "W", at::kFloat, N, K);
  check_gpu(z, "z", at::kFloat);
  TORCH_CHECK(z.numel() == M * N, "dgt: skinny_f32_fwd z must be [M, N]");
  const float* bp = nullptr;
  if (b.has_value() && b->defined()) {
    check_gpu(*b, "b", at::kFloat);
    TORCH_CHECK(b->numel() == N, "dgt: skinny_f32_fwd bias must have N elements");
    bp = b->data_ptr<float>();
  }
  c10::DeviceGuard guard(a.device());
  DGT_CHECK_HIP(dgt::skinny_f32_fwd(a.data_ptr<float>(), W.data_ptr<float>(), bp, z.data_ptr<float>(), (int)M, (int)N,
                                    (int)K, relu ? 1 : 0, stream_of(a)));
}

// its backward: g = dz * 1[y > 0] (y given), dx = (g . W) * 1[a > 0] (mask), dW / db (+)= in fixed order
void skinny_f32_bwd(const at::Tensor& dz, const std::optional<at::Tensor>& y, const at::Tensor& a, const at::Tensor& W,
                    bool mask, const std::optional<at::Tensor>& dx, const at::Tensor& dW,
                    const std::optional<at::Tensor>& db, bool accumulate) {
  const int64_t M = a.size(0), K = a.size(1), N = W.size(0);
  TORCH_CHECK(a.dim() == 2 && W.dim() == 2 && W.size(1) == K && N >= 1 && N <= 4 && M % 64 == 0 && K % 32 == 0 && M > 0,
              "dgt: skinny_f32_bwd needs a [M, K], W [N <= 4, K], M % 64 == 0, K % 32 == 0");
  check_gpu(dz, "dz", at::kFloat);
  TORCH_CHECK(dz.numel() == M * N, "dgt: skinny_f32_bwd dz must be [M, N]");
  check_2d(a, "a", at::kFloat, M, K);
  check_2d(W, "W", at::kFloat, N, K);
  const float* yp = nullptr;
  if (y.has_value() && y->defined()) {
    check_gpu(*y, "y", at::kFloat);
    TORCH_CHECK(y->numel() == M * N, "dgt: skinny_f32_bwd y must be [M, N]");
    yp = y->data_ptr<float>();
  }
  float* dxp = nullptr;
  if (dx.has_value() && dx->defined()) {
    check_2d(*dx, "dx", at::kFloat, M, K);
    dxp = dx->data_ptr<float>();
  }
  check_gpu(dW, "dW", at::kFloat);
  TORCH_CHECK(dW.numel() == N * K && reinterpret_cast<uintptr_t>(dW.data_ptr()) % 16 == 0,
              "dgt: skinny_f32_bwd dW must be [N, K], 16-byte aligned");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    check_gpu(*db, "db", at::kFloat);
    TORCH_CHECK(db->numel() == N, "dgt: skinny_f32_bwd db must have N elements");
    dbp = db->data_ptr<float>();
  }
  c10::DeviceGuard guard(a.device());
  at::Tensor ws = at::empty({M / 64, N, K}, a.options());
  DGT_CHECK_HIP(dgt::skinny_f32_bwd(dz.data_ptr<float>(), yp, a.data_ptr<float>(), W.data_ptr<float>(), mask ? 1 : 0,
                                    dxp, dW.data_ptr<float>(), dbp, accumulate ? 1 : 0, ws.data_ptr<float>(), (int)M,
                                    (int)N, (int)K, stream_of(a)));
}

void mlp_head(const at::Tensor& a, const at::Tensor& w, const at::Tensor& b0, const at::Tensor& y,
              const at::Tensor& dz, const at::Tensor& dw, const at::Tensor& db, const at::Tensor& loss_acc,
              const at::Tensor& g, const at::Tensor& gT, const std::optional<at::Tensor>& dw_part,
              const std::optional<at::Tensor>& bias_part) {
  TORCH_CHECK(a.dim() == 2, "dgt: head activation must be 2-d");
  const int64_t B = a.size(0), D = a.size(1);
  TORCH_CHECK(B % 64 == 0 && D % 64 == 0, "dgt: head needs B, D % 64 == 0");
  check_2d(a, "a", at::kBFloat16, B, D);
  check_gpu(w, "w", at::kFloat);
  check_gpu(b0, "b0", at::kFloat);
  check_gpu(y, "y", at::kFloat);
  check_gpu(dz, "dz", at::kFloat);
  check_gpu(dw, "dw", at::kFloat);
  check_gpu(db, "db", at::kFloat);
  check_gpu(loss_acc, "loss_acc", at::kDouble);
  TORCH_CHECK(w.numel() == D && dw.numel() == D && y.numel() == B && dz.numel() == B, "dgt: head size mismatch");
  check_2d(g, "g", at::kBFloat16, B, D);
  check_2d(gT, "gT", at::kBFloat16, D, B);
  dgt::HeadArgs h;
  h.a = a.data_ptr();
  h.w = w.data_ptr<float>();
  h.b0 = b0.data_ptr<float>();
  h.y = y.data_ptr<float>();
  h.B = (int)B;
  h.D = (int)D;
  h.dz = dz.data_ptr<float>();
  h.dw = dw.data_ptr<float>();
  h.db = db.data_ptr<float>();
  h.loss_acc = loss_acc.data_ptr<double>();
  h.g = g.data_ptr();
  h.gT = gT.data_ptr();
  c10::DeviceGuard guard(a.device());
  // stream-ordered workspace from the caching allocator (reused in place on later calls)
  at::Tensor scratch = at::empty({B + (B / 64) * D}, dz.options());
  h.scratch = scratch.data_ptr<float>();
  h.dw_part = nullptr;
  h.bias_part = nullptr;
  // caller-owned partials (reduced later by partials_reduce_multi, so never in this call's scratch)
  if (dw_part.has_value() && dw_part->defined()) {
    check_2d(*dw_part, "dw_part", at::kFloat, B / 64, D);
    h.dw_part = dw_part->data_ptr<float>();
  }
  if (bias_part.has_value() && bias_part->defined()) {
    check_2d(*bias_part, "bias_part", at::kFloat, B / 64, D);
    h.bias_part = bias_part->data_ptr<float>();
  }
  DGT_CHECK_HIP(dgt::mlp_head(h, stream_of(a)));
}

// out_s (+)= sum over t of part_s[t] for every segment, in one launch (out fp32 or bf16; accumulate[s]
// adds to it instead of storing); with
// `grads` given, also the Adam step of master / exp_avg / exp_avg_sq on the outs' elements (their
// offsets inside `grads`), as adam_flat would over that region
void partials_reduce_multi(at::TensorList parts, at::TensorList outs, const std::optional<at::Tensor>& grads,
                           const std::optional<at::Tensor>& master, const std::optional<at::Tensor>& exp_avg,
                           const std::optional<at::Tensor>& exp_avg_sq, int64_t step, double lr, double beta1,
                           double beta2, double eps, double weight_decay, bool adamw, double grad_scale,
                           at::OptionalIntArrayRef accumulate) {
  TORCH_CHECK(parts.size() == outs.size() && parts.size() >= 1 && (int)parts.size() <= dgt::kMaxReduceSegs,
              "dgt: partials_reduce_multi needs 1..", dgt::kMaxReduceSegs, " (part, out) pairs");
  TORCH_CHECK(!accumulate.has_value() || accumulate->size() == parts.size(),
              "dgt: partials_reduce_multi accumulate needs one flag per segment");
  dgt::ReduceSegs r;
  std::memset(&r, 0, sizeof(r));
  r.count = (int)parts.size();
  for (size_t s = 0; s < parts.size(); ++s) {
    const at::Tensor &p = parts[s], &o = outs[s];
    TORCH_CHECK(p.dim() == 2 && p.is_contiguous() && o.is_contiguous() && o.numel() == p.size(1) && p.size(1) % 4 == 0,
                "dgt: partials_reduce_multi segment ", s, ": part [tiles, n] (n % 4 == 0) and a contiguous out [n]");
    check_gpu(p, "part", at::kFloat);
    const bool bf = o.scalar_type() == at::kBFloat16;
    check_gpu(o, "out", bf ? at::kBFloat16 : at::kFloat);
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(o.data_ptr()) % (bf ? 8 : 16) == 0,
                "dgt: partials_reduce_multi parts must be 16-byte, outs 16 (fp32) / 8 (bf16) byte aligned");
    r.part[s] = p.data_ptr<float>();
    r.out[s] = o.data_ptr();
    r.flags[s] = (bf ? 1 : 0) | ((accumulate.has_value() && (*accumulate)[s]) ? 2 : 0);
    r.tiles[s] = (int)p.size(0);
    r.n[s] = (int)p.size(1);
  }
  dgt::ReduceAdam ad;
  std::memset(&ad, 0, sizeof(ad));
  if (grads.has_value() && grads->defined()) {
    TORCH_CHECK(master.has_value() && exp_avg.has_value() && exp_avg_sq.has_value() && step >= 1,
                "dgt: partials_reduce_multi's Adam needs master, exp_avg, exp_avg_sq and step >= 1");
    for (const at::Tensor* t : {&*grads, &*master, &*exp_avg, &*exp_avg_sq}) {
      check_gpu(*t, "adam region", at::kFloat);
      TORCH_CHECK(t->is_contiguous() && t->numel() == grads->numel() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "dgt: partials_reduce_multi's Adam region tensors must be contiguous, equal-sized, 16-byte aligned");
    }
    const float* gb = grads->data_ptr<float>();
    for (int s = 0; s < r.count; ++s) {
      const float* o = static_cast<const float*>(r.out[s]);
      TORCH_CHECK(r.flags[s] == 0 && o >= gb && o + r.n[s] <= gb + grads->numel(),
                  "dgt: partials_reduce_multi with Adam: every out must be a stored fp32 slice of grads");
    }
    ad.on = 1;
    ad.grads = gb;
    ad.master = master->data_ptr<float>();
    ad.m = exp_avg->data_ptr<float>();
    ad.v = exp_avg_sq->data_ptr<float>();
    ad.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
    const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
    ad.step_size_neg = (float)(-(lr / bc1));
    ad.bc2_sqrt = (float)std::sqrt(bc2);
    ad.grad_scale = (float)grad_scale;
  }
  c10::DeviceGuard guard(parts[0].device());
  DGT_CHECK_HIP(dgt::partials_reduce_multi(r, ad, stream_of(parts[0])));
}

// ------------------------------------------------------------------------------ IPC runtime
// kind: 0 = coarse-grained (hipMalloc), 1 = uncached (no cache holds a line: peers' xGMI writes
// are seen by the next poll), 2 = fine-grained (cacheable, kept coherent by the fabric)
int64_t ipc_alloc(int64_t nbytes, int64_t kind, int64_t device) {
  TORCH_CHECK(nbytes > 0, "dgt: ipc_alloc needs a positive size");
  TORCH_CHECK(kind >= 0 && kind <= 2, "dgt: ipc_alloc kind must be 0 (coarse), 1 (uncached) or 2 (fine-grained)");
  c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  void* p = nullptr;
  if (kind == 1) {
    DGT_CHECK_HIP(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached));
  } else if (kind == 2) {
    DGT_CHECK_HIP(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocFinegrained));
  } else {
    DGT_CHECK_HIP(hipMalloc(&p, (size_t)nbytes));
  }
  DGT_CHECK_HIP(hipMemset(p, 0, (size_t)nbytes));
  DGT_CHECK_HIP(hipDeviceSynchronize());
  return reinterpret_cast<int64_t>(p);
}

at::Tensor ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  DGT_CHECK_HIP(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  at::Tensor out = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}

int64_t ipc_open(const at::Tensor& handle, int64_t device) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == sizeof(hipIpcMemHandle_t),
              "dgt: ipc_open needs a CPU uint8 tensor of ", sizeof(hipIpcMemHandle_t), " bytes");
  c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  DGT_CHECK_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void ipc_close(int64_t ptr) { DGT_CHECK_HIP(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr))); }
void ipc_free(int64_t ptr) { DGT_CHECK_HIP(hipFree(reinterpret_cast<void*>(ptr))); }

void memset_device(int64_t ptr, int64_t value, int64_t nbytes) {
  DGT_CHECK_HIP(hipMemset(reinterpret_cast<void*>(ptr), (int)value, (size_t)nbytes));
}

bool can_access_peer(int64_t dev, int64_t peer) {
  int ok = 0;
  DGT_CHECK_HIP(hipDeviceCanAccessPeer(&ok, (int)dev, (int)peer));
  return ok != 0;
}

}  // namespace

TORCH_LIBRARY(dgt, m) {
  m.def(
      "gemm_nt_adam(Tensor A, Tensor B, Tensor(a!) master, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, "
      "Tensor(d!) param_lp, int step, float lr, float beta1, float beta2, float eps, float weight_decay, bool adamw, "
      "float grad_scale, int variant=0) -> ()",
      &gemm_nt_adam);
  m.def("tiny_mlp_supported(int f, int h) -> bool", &tiny_mlp_supported);
  m.def("tiny_mlp_padded_numel(int f, int h) -> int", &tiny_mlp_padded_numel);
  m.def("tiny_mlp_exchange_floats(int f, int h) -> int", &tiny_mlp_exchange_floats);
  m.def(
      "tiny_mlp_train(Tensor X, Tensor Y, Tensor plan, Tensor counts, Tensor(a!) params, Tensor(b!) exp_avg, "
      "Tensor(c!) exp_avg_sq, Tensor(d!) loss_acc, Tensor(e!) status, int n_features, int hidden, float lr, "
      "float beta1, float beta2, float eps, float weight_decay, bool adamw, int adam_step0, int[] data_ptrs, "
      "int rank, int world_size, int stride, int seq_base, int timeout_ticks, int corrupt_step=-1, "
      "Tensor(f!)? workspace=None, int zero1=0, int line=3, int xsum=0) -> ()",
      &tiny_mlp_train);
  m.def(
      "tiny_launcher_create(Tensor X, Tensor Y, Tensor(a!) params, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, "
      "Tensor(d!) loss_acc, Tensor(e!) status, int n_features, int hidden, float lr, float beta1, float beta2, "
      "float eps, float weight_decay, bool adamw, int[] data_ptrs, int rank, int world_size, int stride, "
      "int timeout_ticks, int corrupt_step, int zero1=0, int line=3, int xsum=0) -> int",
      &tiny_launcher_create);
  m.def("tiny_launcher_destroy(int handle) -> ()", &tiny_launcher_destroy);
  m.def(
      "tiny_xch_stress(int n_features, int hidden, int[] data_ptrs, int rank, int world_size, int stride, "
      "int seq_base, int timeout_ticks, int line, int n_steps, Tensor(a!) status, Tensor(b!) errors) -> ()",
      &tiny_xch_stress);
  m.def(
      "tiny_mlp_grad(Tensor X, Tensor Y, Tensor plan, Tensor counts, int step, Tensor params, Tensor(a!) grad, "
      "Tensor(b!) loss_acc, int n_features, int hidden) -> ()",
      &tiny_mlp_grad);
  m.def(
      "adam_flat(Tensor(a!) master, Tensor(b!)? param_lp, Tensor grad, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, "
      "float lr, float beta1, float beta2, float eps, float weight_decay, bool adamw, int step, float grad_scale, "
      "Tensor? grad_scale_dev, Tensor(e!)? step_dev=None, Tensor(f!)? step_ticket=None) -> ()",
      &adam_flat);
  m.def("step_increment(Tensor(a!) counter) -> ()", &step_increment);
  m.def("bce_logits(Tensor z, Tensor y, Tensor(a!) loss, Tensor(b!) dz, Tensor(c!)? dz_lp=None, Tensor(d!)? sum_into=None) -> ()", &bce_logits);
  m.def("gather_rows(Tensor idx, Tensor[] srcs) -> Tensor[]", &gather_rows);
  m.def("linear_fwd(Tensor x, Tensor W, Tensor? b, Tensor(a!) y, bool relu) -> ()", &linear_fwd);
  m.def("linear2_fwd(Tensor x, Tensor W1, Tensor? b1, Tensor W2, Tensor? b2, Tensor(a!) h, Tensor(b!) y, bool relu1, "
        "bool relu2) -> ()",
        &linear2_fwd);
  m.def("linear2_bwd(Tensor dy, Tensor x, Tensor W1, Tensor h, Tensor W2, Tensor? y, Tensor(a!)? dx, Tensor(b!) dW1, "
        "Tensor(c!)? db1, Tensor(d!) dW2, Tensor(e!)? db2, bool relu1, bool acc1, bool acc2) -> ()",
        &linear2_bwd);
  m.def("gemm_f32(Tensor A, Tensor B, Tensor? maskA, Tensor? bias, Tensor(a!) C, int la, int lb, bool relu=False, "
        "bool accumulate=False, Tensor(b!)? rowsum=None, Tensor? maskC=None) -> ()",
        &gemm_f32);
  m.def("colsum_f32(Tensor dy, Tensor? y, Tensor(a!) db, bool accumulate=False) -> ()", &colsum_f32);
  m.def("linear_bwd(Tensor dy, Tensor x, Tensor W, Tensor? y, Tensor(a!)? dx, Tensor(b!) dW, Tensor(c!)? db, "
        "bool accumulate=False) -> ()",
        &linear_bwd);
  m.def(
      "oneshot_allreduce(Tensor inp, Tensor(a!) out, float scale, int[] data_ptrs, int rank, "
      "int world_size, int stride, int seq, int timeout_ticks, Tensor(b!) status, int reps=1) -> ()",
      &oneshot_allreduce);
  m.def(
      "gemm_nt(Tensor A, Tensor B, Tensor(a!)? C, Tensor(b!)? CT, Tensor? bias, Tensor? mask, int epi, "
      "float alpha, int variant=0, Tensor(c!)? colsum=None) -> ()",
      &gemm_nt);
  m.def("transpose_bf16(Tensor inp, Tensor(a!) out) -> ()", &transpose_bf16);
  m.def("rowsum_bf16(Tensor inp, Tensor(a!) out, bool accumulate) -> ()", &rowsum_bf16);
  m.def("skinny_fwd_bf16(Tensor a, Tensor W, Tensor? b, Tensor(a!) z) -> ()", &skinny_fwd_bf16);
  m.def("skinny_f32_fwd(Tensor a, Tensor W, Tensor? b, Tensor(a!) z, bool relu=False) -> ()", &skinny_f32_fwd);
  m.def(
      "skinny_f32_bwd(Tensor dz, Tensor? y, Tensor a, Tensor W, bool mask, Tensor(a!)? dx, Tensor(b!) dW, "
      "Tensor(c!)? db, bool accumulate=False) -> ()",
      &skinny_f32_bwd);
  m.def(
      "skinny_bwd_bf16(Tensor dz, Tensor a, Tensor W, bool mask, Tensor(a!) g, Tensor(b!)? gT, Tensor(c!) dW, "
      "Tensor(d!) db, bool accumulate=True, Tensor(e!)? bias_part=None, Tensor(f!)? dw_part=None) -> ()",
      &skinny_bwd_bf16);
  m.def(
      "mlp_head(Tensor a, Tensor w, Tensor b0, Tensor y, Tensor(a!) dz, Tensor(b!) dw, Tensor(c!) db, "
      "Tensor(d!) loss_acc, Tensor(e!) g, Tensor(f!) gT, Tensor(g!)? dw_part=None, Tensor(h!)? bias_part=None) -> ()",
      &mlp_head);
  m.def(
      "partials_reduce_multi(Tensor[] parts, Tensor(a!)[] outs, Tensor? grads=None, Tensor(b!)? master=None, "
      "Tensor(c!)? exp_avg=None, Tensor(d!)? exp_avg_sq=None, int step=1, float lr=0., float beta1=0.9, "
      "float beta2=0.999, float eps=1e-8, float weight_decay=0., bool adamw=False, float grad_scale=1., "
      "int[]? accumulate=None) -> ()",
      &partials_reduce_multi);
  m.def("ipc_alloc(int nbytes, int kind, int device) -> int", &ipc_alloc);
  m.def("ipc_handle(int ptr) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle, int device) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
  m.def("ipc_free(int ptr) -> ()", &ipc_free);
  m.def("memset_device(int ptr, int value, int nbytes) -> ()", &memset_device);
  m.def("can_access_peer(int dev, int peer) -> bool", &can_access_peer);
}

// The same functions as a Python extension module (``distributed_gpu_test_amd._C``, loaded by
// ops/_ext.py fast()): a pybind11 call unpacks its tensors directly, where a ``torch.ops.dgt`` call
// goes through the boxed dispatcher (an IValue stack per call) -- ~2-3 us of host time per call on
// the MI355X box, paid several times per step by the host-bound engine paths (gather, Linear chain,
// loss, Adam).  Only the hot eager-path ops; everything else stays on torch.ops.dgt.

// ---------------------------------------------------------------- captured kernels, launched directly
// A HIP graph replay costs ~10 us of device time on this stack whatever it holds, against ~4-5 us for
// one kernel launched directly (profiles/r5_graph_launch_cost.txt).  A graph that captured only a
// chain of kernels can therefore run cheaper as the same kernels re-launched with the captured
// arguments, in capture order, on the current stream: the graph keeps owning the argument storage
// (torch.cuda.CUDAGraph(keep_graph=True)), so the launches read exactly what a replay would.
struct DirectNode {
  const void* func;
  dim3 grid, block;
  unsigned shmem;
  void** params;
};

struct DirectLaunch {
  std::vector<DirectNode> nodes;
  int device = 0;
  void launch() const {
    hipStream_t st = at::hip::getCurrentHIPStreamMasqueradingAsCUDA(device).stream();
    for (const DirectNode& n : nodes) DGT_CHECK_HIP(hipLaunchKernel(n.func, n.grid, n.block, n.params, n.shmem, st));
  }
};

// The kernels of ``graph`` in dependency order, or nullptr when the graph holds anything else (a copy,
// memset, event or child-graph node, a fork or join, arguments passed through ``extra``, or a function
// the runtime does not know as a launchable kernel).
std::unique_ptr<DirectLaunch> direct_plan(uintptr_t graph_handle, int device) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph_handle);
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess || n == 0 || n > 64) return nullptr;
  std::vector<hipGraphNode_t> all(n);
  if (hipGraphGetNodes(g, all.data(), &n) != hipSuccess) return nullptr;
  // a linear chain: one root, every node at most one dependency and one dependent
  hipGraphNode_t cur = nullptr;
  for (hipGraphNode_t node : all) {
    size_t deps = 0;
    if (hipGraphNodeGetDependencies(node, nullptr, &deps) != hipSuccess || deps > 1) return nullptr;
    if (deps == 0) {
      if (cur != nullptr) return nullptr;
      cur = node;
    }
  }
  auto plan = std::make_unique<DirectLaunch>();
  plan->device = device;
  while (cur != nullptr) {
    hipGraphNodeType type;
    if (hipGraphNodeGetType(cur, &type) != hipSuccess || type != hipGraphNodeTypeKernel) return nullptr;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(cur, &kp) != hipSuccess || kp.extra != nullptr || kp.func == nullptr) return nullptr;
    hipFuncAttributes attr;
    if (hipFuncGetAttributes(&attr, kp.func) != hipSuccess) return nullptr;
    plan->nodes.push_back({kp.func, kp.gridDim, kp.blockDim, kp.sharedMemBytes, kp.kernelParams});
    size_t outs = 0;
    if (hipGraphNodeGetDependentNodes(cur, nullptr, &outs) != hipSuccess || outs > 1) return nullptr;
    hipGraphNode_t next = nullptr;
    if (outs == 1 && hipGraphNodeGetDependentNodes(cur, &next, &outs) != hipSuccess) return nullptr;
    cur = outs == 1 ? next : nullptr;
  }
  if (plan->nodes.size() != n) return nullptr;
  return plan;
}

namespace dgt {
void bucket_launcher_submit(int64_t h, int64_t bi);  // bucket_launcher.cpp
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "dgt hot-path ops without the dispatcher (same C++ functions as torch.ops.dgt)";
  m.def("gather_rows", [](const at::Tensor& idx, const std::vector<at::Tensor>& srcs) { return gather_rows(idx, srcs); });
  m.def("bce_logits", &bce_logits);
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_bwd", &linear_bwd);
  m.def("linear2_fwd", &linear2_fwd);
  m.def("linear2_bwd", &linear2_bwd);
  m.def("adam_flat", &adam_flat);
  m.def("bucket_launcher_submit", &dgt::bucket_launcher_submit);
  pybind11::class_<DirectLaunch>(m, "DirectLaunch")
      .def("__call__", &DirectLaunch::launch)
      .def_property_readonly("kernels", [](const DirectLaunch& d) { return d.nodes.size(); });
  m.def("graph_direct_plan", [](uintptr_t graph, int device) -> pybind11::object {
    auto p = direct_plan(graph, device);
    if (!p) return pybind11::none();
    return pybind11::cast(std::move(p));
  });
}
