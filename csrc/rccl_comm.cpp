// Native RCCL communicator: collectives enqueued directly on the caller's current HIP
// stream, with no process-group bookkeeping in between, so a whole training step — kernels AND the
// gradient all-reduce — can be captured into one HIP graph and replayed.  The communicator is
// bootstrapped over the existing torch.distributed group: rank 0 creates the ncclUniqueId, the
// Python side broadcasts its 128 bytes, every rank calls ncclCommInitRank.
//
// Links against the librccl.so that PyTorch-ROCm already loads (same soname), so RCCL state is
// shared with ProcessGroupNCCL's copy of the library rather than duplicated.
// Reference: deepspeed.init_distributed() at train.py:59 and the all-reduce inside backward at train.py:113.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <cstring>

namespace {

#define DGT_CHECK_NCCL(expr)                                                                    \
  do {                                                                                          \
    ncclResult_t r_ = (expr);                                                                   \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", ncclGetErrorString(r_), " in ", #expr);       \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "dgt.rccl: unsupported dtype ", t);
  }
}

ncclRedOp_t to_op(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: TORCH_CHECK(false, "dgt.rccl: bad reduce op ", op);
  }
}

hipStream_t cur(const at::Tensor& t) {
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

ncclComm_t comm_of(int64_t h) {
  TORCH_CHECK(h != 0, "dgt.rccl: null communicator");
  return reinterpret_cast<ncclComm_t>(h);
}

void check(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "dgt.rccl: tensors must be contiguous GPU tensors");
}

at::Tensor rccl_unique_id() {
  ncclUniqueId id;
  DGT_CHECK_NCCL(ncclGetUniqueId(&id));
  at::Tensor out = at::empty({(int64_t)sizeof(id)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &id, sizeof(id));
  return out;
}

int64_t rccl_comm_init(const at::Tensor& id, int64_t rank, int64_t world, int64_t device) {
  TORCH_CHECK(!id.is_cuda() && id.numel() == (int64_t)sizeof(ncclUniqueId), "dgt.rccl: bad unique id");
  ncclUniqueId uid;
  std::memcpy(&uid, id.contiguous().data_ptr(), sizeof(uid));
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  ncclComm_t comm;
  DGT_CHECK_NCCL(ncclCommInitRank(&comm, (int)world, uid, (int)rank));
  return reinterpret_cast<int64_t>(comm);
}

void rccl_comm_destroy(int64_t h) { DGT_CHECK_NCCL(ncclCommDestroy(comm_of(h))); }

int64_t rccl_version() {
  int v = 0;
  DGT_CHECK_NCCL(ncclGetVersion(&v));
  return v;
}

void rccl_all_reduce(int64_t h, const at::Tensor& t, int64_t op) {
  check(t);
  DGT_CHECK_NCCL(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_op(op), comm_of(h),
                               cur(t)));
}

void rccl_reduce_scatter(int64_t h, const at::Tensor& out, const at::Tensor& in, int64_t op) {
  check(out);
  check(in);
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "dgt.rccl: dtype mismatch");
  DGT_CHECK_NCCL(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(out.scalar_type()), to_op(op),
                                   comm_of(h), cur(out)));
}

void rccl_all_gather(int64_t h, const at::Tensor& out, const at::Tensor& in) {
  check(out);
  check(in);
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "dgt.rccl: dtype mismatch");
  DGT_CHECK_NCCL(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_of(h),
                               cur(out)));
}

void rccl_broadcast(int64_t h, const at::Tensor& t, int64_t root) {
  check(t);
  DGT_CHECK_NCCL(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), (int)root, comm_of(h),
                               cur(t)));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(dgt, m) {
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_comm_init(Tensor id, int rank, int world, int device) -> int", &rccl_comm_init);
  m.def("rccl_comm_destroy(int comm) -> ()", &rccl_comm_destroy);
  m.def("rccl_version() -> int", &rccl_version);
  m.def("rccl_all_reduce(int comm, Tensor(a!) t, int op) -> ()", &rccl_all_reduce);
  m.def("rccl_reduce_scatter(int comm, Tensor(a!) out, Tensor inp, int op) -> ()", &rccl_reduce_scatter);
  m.def("rccl_all_gather(int comm, Tensor(a!) out, Tensor inp) -> ()", &rccl_all_gather);
  m.def("rccl_broadcast(int comm, Tensor(a!) t, int root) -> ()", &rccl_broadcast);
}
