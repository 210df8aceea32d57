// torch.ops.dgt.* bindings for the MI355X kernels and the IPC runtime.
// Host-only translation unit: validates shapes/devices, picks the current HIP stream, and calls
// the launch functions declared in dgt_kernels.h.  Every op fails loudly on a non-GPU tensor.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <cstring>
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

dgt::Exchange make_exchange(c10::ArrayRef<int64_t> data_ptrs, c10::ArrayRef<int64_t> flag_ptrs, int64_t rank,
                            int64_t world_size, int64_t stride, int64_t seq_base, int64_t timeout_ticks) {
  dgt::Exchange ex;
  std::memset(&ex, 0, sizeof(ex));
  TORCH_CHECK(world_size >= 1 && world_size <= dgt::kMaxRanks, "dgt: world_size must be in [1, 8], got ", world_size);
  TORCH_CHECK(rank >= 0 && rank < world_size, "dgt: bad rank ", rank);
  ex.rank = (int)rank;
  ex.world_size = (int)world_size;
  ex.stride = (int)stride;
  ex.seq_base = seq_base;
  ex.timeout_ticks = timeout_ticks;
  if (world_size > 1) {
    TORCH_CHECK((int64_t)data_ptrs.size() == world_size && (int64_t)flag_ptrs.size() == world_size,
                "dgt: need one mailbox pointer per rank");
    for (int64_t i = 0; i < world_size; ++i) {
      TORCH_CHECK(data_ptrs[i] != 0 && flag_ptrs[i] != 0, "dgt: null mailbox pointer for rank ", i);
      ex.data[i] = reinterpret_cast<float*>(data_ptrs[i]);
      ex.flags[i] = reinterpret_cast<unsigned*>(flag_ptrs[i]);
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

void tiny_mlp_train(const at::Tensor& X, const at::Tensor& Y, const at::Tensor& plan, const at::Tensor& counts,
                    const at::Tensor& params, const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq,
                    const at::Tensor& loss_acc, const at::Tensor& status, int64_t n_features, int64_t hidden,
                    double lr, double beta1, double beta2, double eps, double weight_decay, bool adamw,
                    int64_t adam_step0, c10::ArrayRef<int64_t> data_ptrs, c10::ArrayRef<int64_t> flag_ptrs,
                    int64_t rank, int64_t world_size, int64_t stride, int64_t seq_base, int64_t timeout_ticks) {
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
  a.loss_acc = loss_acc.data_ptr<double>();
  a.status = status.data_ptr<int>();
  a.ex = make_exchange(data_ptrs, flag_ptrs, rank, world_size, stride, seq_base, timeout_ticks);
  a.stamps = nullptr;
  if (world_size > 1) TORCH_CHECK(stride >= pp, "dgt: mailbox stride ", stride, " < ", pp);
  if (a.n_steps == 0) return;
  DGT_CHECK_HIP(dgt::tiny_mlp_train((int)n_features, (int)hidden, a, stream_of(X)));
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
void adam_flat(const at::Tensor& master, const std::optional<at::Tensor>& param_lp, const at::Tensor& grad,
               const at::Tensor& exp_avg, const at::Tensor& exp_avg_sq, double lr, double beta1, double beta2,
               double eps, double weight_decay, bool adamw, int64_t step, double grad_scale,
               const std::optional<at::Tensor>& grad_scale_dev) {
  check_gpu(master, "master", at::kFloat);
  check_gpu(exp_avg, "exp_avg", at::kFloat);
  check_gpu(exp_avg_sq, "exp_avg_sq", at::kFloat);
  TORCH_CHECK(grad.is_cuda() && grad.is_contiguous(), "dgt: grad must be a contiguous GPU tensor");
  const int64_t n = master.numel();
  TORCH_CHECK(n % 4 == 0, "dgt: flat buffers must be padded to a multiple of 4 elements");
  TORCH_CHECK(grad.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n, "dgt: flat size mismatch");
  TORCH_CHECK(step >= 1, "dgt: adam step must be >= 1");
  c10::DeviceGuard guard(master.device());
  dgt::AdamFlatArgs a;
  a.master = master.data_ptr<float>();
  a.param_lp = nullptr;
  a.lp_dtype = dgt::kF32;
  if (param_lp.has_value() && param_lp->defined()) {
    TORCH_CHECK(param_lp->is_cuda() && param_lp->is_contiguous() && param_lp->numel() == n, "dgt: bad param_lp");
    a.param_lp = param_lp->data_ptr();
    a.lp_dtype = dtype_code(param_lp->scalar_type());
  }
  a.grad = grad.data_ptr();
  a.grad_dtype = dtype_code(grad.scalar_type());
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.n = n;
  a.hp = make_hyper(lr, beta1, beta2, eps, weight_decay, adamw);
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  a.step_size_neg = (float)(-(lr / bc1));
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.grad_scale = (float)grad_scale;
  a.grad_scale_dev = nullptr;
  if (grad_scale_dev.has_value() && grad_scale_dev->defined()) {
    check_gpu(*grad_scale_dev, "grad_scale_dev", at::kFloat);
    a.grad_scale_dev = grad_scale_dev->data_ptr<float>();
  }
  DGT_CHECK_HIP(dgt::adam_flat(a, stream_of(master)));
}

// ------------------------------------------------------------------------------ one-shot all-reduce
void oneshot_allreduce(const at::Tensor& inp, const at::Tensor& out, double scale, c10::ArrayRef<int64_t> data_ptrs,
                       c10::ArrayRef<int64_t> flag_ptrs, int64_t rank, int64_t world_size, int64_t stride,
                       int64_t seq, int64_t timeout_ticks, const at::Tensor& status) {
  check_gpu(inp, "inp", at::kFloat);
  check_gpu(out, "out", at::kFloat);
  check_gpu(status, "status", at::kInt);
  TORCH_CHECK(inp.numel() == out.numel() && inp.numel() % 4 == 0 && inp.numel() <= stride,
              "dgt: one-shot all-reduce needs equal sizes, a multiple of 4 and <= mailbox stride");
  c10::DeviceGuard guard(inp.device());
  dgt::Exchange ex = make_exchange(data_ptrs, flag_ptrs, rank, world_size, stride, seq, timeout_ticks);
  DGT_CHECK_HIP(dgt::oneshot_allreduce(inp.data_ptr<float>(), out.data_ptr<float>(), inp.numel(), (float)scale, ex,
                                       status.data_ptr<int>(), stream_of(inp)));
}

// ------------------------------------------------------------------------------ IPC runtime
int64_t ipc_alloc(int64_t nbytes, bool uncached, int64_t device) {
  TORCH_CHECK(nbytes > 0, "dgt: ipc_alloc needs a positive size");
  c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  void* p = nullptr;
  if (uncached) {
    DGT_CHECK_HIP(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached));
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
  m.def("tiny_mlp_supported(int f, int h) -> bool", &tiny_mlp_supported);
  m.def("tiny_mlp_padded_numel(int f, int h) -> int", &tiny_mlp_padded_numel);
  m.def(
      "tiny_mlp_train(Tensor X, Tensor Y, Tensor plan, Tensor counts, Tensor(a!) params, Tensor(b!) exp_avg, "
      "Tensor(c!) exp_avg_sq, Tensor(d!) loss_acc, Tensor(e!) status, int n_features, int hidden, float lr, "
      "float beta1, float beta2, float eps, float weight_decay, bool adamw, int adam_step0, int[] data_ptrs, "
      "int[] flag_ptrs, int rank, int world_size, int stride, int seq_base, int timeout_ticks) -> ()",
      &tiny_mlp_train);
  m.def(
      "tiny_mlp_grad(Tensor X, Tensor Y, Tensor plan, Tensor counts, int step, Tensor params, Tensor(a!) grad, "
      "Tensor(b!) loss_acc, int n_features, int hidden) -> ()",
      &tiny_mlp_grad);
  m.def(
      "adam_flat(Tensor(a!) master, Tensor(b!)? param_lp, Tensor grad, Tensor(c!) exp_avg, Tensor(d!) exp_avg_sq, "
      "float lr, float beta1, float beta2, float eps, float weight_decay, bool adamw, int step, float grad_scale, "
      "Tensor? grad_scale_dev) -> ()",
      &adam_flat);
  m.def(
      "oneshot_allreduce(Tensor inp, Tensor(a!) out, float scale, int[] data_ptrs, int[] flag_ptrs, int rank, "
      "int world_size, int stride, int seq, int timeout_ticks, Tensor(b!) status) -> ()",
      &oneshot_allreduce);
  m.def("ipc_alloc(int nbytes, bool uncached, int device) -> int", &ipc_alloc);
  m.def("ipc_handle(int ptr) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle, int device) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
  m.def("ipc_free(int ptr) -> ()", &ipc_free);
  m.def("memset_device(int ptr, int value, int nbytes) -> ()", &memset_device);
  m.def("can_access_peer(int dev, int peer) -> bool", &can_access_peer);
}
