// Native gradient-bucket launcher: the engine's per-layer bucket collectives issued from a C++ thread.
//
// Reference: the gradient all-reduce inside model_engine.backward (train.py:113), SURVEY X6 / HC1 /
// HC7; the Python side is distributed_gpu_test_amd/parallel/reducer.py.
//
// The engine's fused Linear chains report each layer's gradient complete from inside their backward
// (ops/linear.py grad_ready), and the layer's bucket should go out over xGMI right then, beside the
// backward of the layers below.  Issuing that collective from the thread that enqueues backward costs
// the compute stream its next kernels for as long as the launch takes (ProcessGroupNCCL's bookkeeping,
// RCCL's enqueue, the wire cast: 40-60 us of host per bucket, profiles/r6_reducer_host_cost.json),
// and a Python launcher thread shares the interpreter lock with it.  So the backward thread only
// records a HIP event on its stream and queues (bucket, event) here (a few microseconds); this
// launcher's own thread, which never touches Python, makes a side stream wait for the event, widens
// bf16 gradients onto the fp32 wire buffer there (comm.hip widen_bf16_f32) and enqueues the bucket's
// ncclAllReduce (ZeRO-0) or ncclReduceScatter into this rank's shard (ZeRO-1/2) on the same side
// stream, on the framework's native communicator (rccl_comm.cpp).  One thread issues every
// collective in submission order, so every rank issues the same sequence.  finish() waits until the
// queue is drained, then makes the caller's stream wait for the side stream: the optimizer reads
// the reduced buffer after that.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dgt_kernels.h"

namespace {

struct Bucket {
  int64_t off;        // element offset in the gradient / wire buffers
  int64_t numel;      // padded length (a multiple of world for ZeRO)
  int64_t shard_off;  // element offset of this rank's shard in the shard buffer (ZeRO)
};

struct Launcher {
  ncclComm_t comm = nullptr;
  int device = 0;
  int stage = 0;
  int world = 1;
  void* grad = nullptr;
  void* wire = nullptr;  // == grad when no cast
  void* shard = nullptr;
  bool widen = false;    // bf16 gradients -> fp32 wire
  ncclDataType_t wire_t = ncclFloat32;
  size_t wire_elem = 4;
  std::vector<Bucket> buckets;
  hipStream_t side = nullptr;
  bool own_side = false;
  hipEvent_t join_ev = nullptr;
  std::vector<hipEvent_t> free_events;
  std::mutex mu;
  std::condition_variable cv, idle_cv;
  std::deque<std::pair<int, hipEvent_t>> q;
  int busy = 0;
  bool stop = false;
  std::string error;
  std::thread th;
  int64_t launched = 0;
  bool failed = false;  // (worker-thread local copy of "an earlier launch failed")

  void run() {
    hipSetDevice(device);
    for (;;) {
      std::pair<int, hipEvent_t> item;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;  // stop
        item = q.front();
        q.pop_front();
        ++busy;
        failed = !error.empty();
      }
      std::string err;
      if (!failed) err = issue(item.first, item.second);
      {
        std::lock_guard<std::mutex> lk(mu);
        // the wait above captured the event's recorded state: it may be recorded again
        free_events.push_back(item.second);
        if (!err.empty() && error.empty()) error = err;
        --busy;
        ++launched;
      }
      idle_cv.notify_all();
    }
  }

  std::string issue(int bi, hipEvent_t ev) {
    const Bucket& b = buckets[bi];
    if (hipStreamWaitEvent(side, ev, 0) != hipSuccess) return "hipStreamWaitEvent failed";
    char* wbase = static_cast<char*>(wire) + b.off * (int64_t)wire_elem;
    if (widen) {
      const char* g = static_cast<const char*>(grad) + b.off * 2;
      if (dgt::widen_bf16_f32(g, reinterpret_cast<float*>(wbase), b.numel, side) != hipSuccess)
        return "widen_bf16_f32 launch failed";
    }
    ncclResult_t r;
    if (stage == 0) {
      r = ncclAllReduce(wbase, wbase, (size_t)b.numel, wire_t, ncclSum, comm, side);
    } else {
      char* out = static_cast<char*>(shard) + b.shard_off * (int64_t)wire_elem;
      r = ncclReduceScatter(wbase, out, (size_t)(b.numel / world), wire_t, ncclSum, comm, side);
    }
    if (r != ncclSuccess) return std::string("RCCL error ") + ncclGetErrorString(r);
    return std::string();
  }
};

}  // namespace

namespace dgt {

static Launcher* launcher_of(int64_t h) {
  TORCH_CHECK(h != 0, "dgt.bucket_launcher: null handle");
  return reinterpret_cast<Launcher*>(h);
}

static ncclDataType_t nccl_type(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    default: TORCH_CHECK(false, "dgt.bucket_launcher: unsupported wire dtype ", t);
  }
}

// offsets / numels / shard_offsets: int64 CPU tensors, one entry per bucket
int64_t bucket_launcher_create(int64_t comm, const at::Tensor& grad, const at::Tensor& wire,
                               const c10::optional<at::Tensor>& shard, const at::Tensor& offsets,
                               const at::Tensor& numels, const at::Tensor& shard_offsets, int64_t stage,
                               int64_t world, int64_t side_stream) {
  TORCH_CHECK(comm != 0, "dgt.bucket_launcher: null communicator");
  TORCH_CHECK(grad.is_cuda() && wire.is_cuda() && grad.is_contiguous() && wire.is_contiguous(),
              "dgt.bucket_launcher: contiguous GPU buffers");
  TORCH_CHECK(grad.numel() == wire.numel(), "dgt.bucket_launcher: gradient and wire buffers differ in length");
  const bool same = grad.data_ptr() == wire.data_ptr();
  TORCH_CHECK(same || (grad.scalar_type() == at::kBFloat16 && wire.scalar_type() == at::kFloat),
              "dgt.bucket_launcher: the wire is the gradient buffer itself or its fp32 copy of bf16 gradients");
  TORCH_CHECK(stage == 0 || (shard.has_value() && shard->is_cuda() && shard->scalar_type() == wire.scalar_type()),
              "dgt.bucket_launcher: ZeRO needs a shard buffer of the wire dtype");
  auto off = offsets.to(at::kLong).contiguous(), num = numels.to(at::kLong).contiguous(),
       soff = shard_offsets.to(at::kLong).contiguous();
  TORCH_CHECK(off.numel() == num.numel() && soff.numel() == num.numel(), "dgt.bucket_launcher: bucket table sizes");
  auto* L = new Launcher();
  L->comm = reinterpret_cast<ncclComm_t>(comm);
  L->device = grad.device().index();
  L->stage = (int)stage;
  L->world = (int)world;
  L->grad = grad.data_ptr();
  L->wire = wire.data_ptr();
  L->shard = stage ? shard->data_ptr() : nullptr;
  L->widen = !same;
  L->wire_t = nccl_type(wire.scalar_type());
  L->wire_elem = wire.element_size();
  const int64_t* po = off.data_ptr<int64_t>();
  const int64_t* pn = num.data_ptr<int64_t>();
  const int64_t* ps = soff.data_ptr<int64_t>();
  for (int64_t i = 0; i < num.numel(); ++i) {
    TORCH_CHECK(po[i] >= 0 && pn[i] > 0 && po[i] + pn[i] <= grad.numel(), "dgt.bucket_launcher: bucket ", i,
                " outside the buffer");
    TORCH_CHECK(stage == 0 || pn[i] % world == 0, "dgt.bucket_launcher: ZeRO bucket not a multiple of world");
    L->buckets.push_back({po[i], pn[i], ps[i]});
  }
  hipSetDevice(L->device);
  // The side stream is the caller's (a stream of torch's pool, ``side_stream``): two streams that share a
  // hardware queue run strictly in turn (GPU_MAX_HW_QUEUES queues per process, streams assigned round
  // robin), and a stream created here landed on the compute stream's queue
  // (profiles/r6_engine_overlap_trace_v3.txt); a stream of another priority class gets a queue of its
  // own but put the device in a mode where every kernel ran ~2x longer (profiles/r6_reducer_launch_ab.txt).
  // A CU-masked stream made here would get a queue of its own too -- and, as a fifth queue, the same
  // slowdown.  So the caller picks a stream of torch's pool measured to run beside the compute stream
  // (accelerator.py concurrent_stream); side_stream == 0 falls back to a plain stream made here.
  if (side_stream != 0) {
    L->side = reinterpret_cast<hipStream_t>(side_stream);
    L->own_side = false;
  } else {
    TORCH_CHECK(hipStreamCreateWithFlags(&L->side, hipStreamNonBlocking) == hipSuccess, "hipStreamCreate failed");
    L->own_side = true;
  }
  TORCH_CHECK(hipEventCreateWithFlags(&L->join_ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
  L->th = std::thread([L] { L->run(); });
  return reinterpret_cast<int64_t>(L);
}

// Queue bucket bi: its gradients are complete at the current point of the caller's current stream.
void bucket_launcher_submit(int64_t h, int64_t bi) {
  Launcher* L = launcher_of(h);
  TORCH_CHECK(bi >= 0 && bi < (int64_t)L->buckets.size(), "dgt.bucket_launcher: bad bucket ", bi);
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    if (!L->free_events.empty()) {
      ev = L->free_events.back();
      L->free_events.pop_back();
    }
  }
  if (ev == nullptr)
    TORCH_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
  hipStream_t cur = at::hip::getCurrentHIPStreamMasqueradingAsCUDA(L->device).stream();
  TORCH_CHECK(hipEventRecord(ev, cur) == hipSuccess, "hipEventRecord failed");
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->q.emplace_back((int)bi, ev);
  }
  L->cv.notify_one();
}

// Every submitted bucket issued; the caller's current stream then waits for their collectives.
void bucket_launcher_finish(int64_t h) {
  Launcher* L = launcher_of(h);
  std::string err;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    L->idle_cv.wait(lk, [&] { return L->q.empty() && L->busy == 0; });
    err.swap(L->error);
  }
  TORCH_CHECK(err.empty(), "dgt.bucket_launcher: ", err);
  hipStream_t cur = at::hip::getCurrentHIPStreamMasqueradingAsCUDA(L->device).stream();
  TORCH_CHECK(hipEventRecord(L->join_ev, L->side) == hipSuccess, "hipEventRecord failed");
  TORCH_CHECK(hipStreamWaitEvent(cur, L->join_ev, 0) == hipSuccess, "hipStreamWaitEvent failed");
}

int64_t bucket_launcher_launched(int64_t h) {
  Launcher* L = launcher_of(h);
  std::lock_guard<std::mutex> lk(L->mu);
  return L->launched;
}

void bucket_launcher_destroy(int64_t h) {
  Launcher* L = launcher_of(h);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv.notify_all();
  if (L->th.joinable()) L->th.join();
  hipSetDevice(L->device);
  hipStreamSynchronize(L->side);
  for (hipEvent_t e : L->free_events) hipEventDestroy(e);
  for (auto& it : L->q) hipEventDestroy(it.second);
  hipEventDestroy(L->join_ev);
  if (L->own_side) hipStreamDestroy(L->side);
  delete L;
}

}  // namespace dgt

TORCH_LIBRARY_FRAGMENT(dgt, m) {
  using namespace dgt;
  m.def("bucket_launcher_create(int comm, Tensor grad, Tensor wire, Tensor? shard, Tensor offsets, Tensor numels, "
        "Tensor shard_offsets, int stage, int world, int side_stream) -> int", &bucket_launcher_create);
  m.def("bucket_launcher_submit(int handle, int bucket) -> ()", &bucket_launcher_submit);
  m.def("bucket_launcher_finish(int handle) -> ()", &bucket_launcher_finish);
  m.def("bucket_launcher_launched(int handle) -> int", &bucket_launcher_launched);
  m.def("bucket_launcher_destroy(int handle) -> ()", &bucket_launcher_destroy);
}
