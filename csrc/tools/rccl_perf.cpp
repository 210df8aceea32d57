// rccl_perf — collective bus-bandwidth sweep over the GPUs of one node (rccl-tests equivalent;
// rccl-tests is not shipped in the ROCm image).  One process drives every visible GPU through
// ncclCommInitAll, exactly like `all_reduce_perf -g N`, so no launcher or MPI is needed.
//
//   rccl_perf [-o all_reduce|reduce_scatter|all_gather|broadcast|alltoall] [-d float|bf16|half]
//             [-b MINBYTES] [-e MAXBYTES] [-f FACTOR] [-g NGPUS] [-n ITERS] [-w WARMUP] [-c 0|1] [-j]
//
// Columns follow rccl-tests: size, count, type, time (us), algbw, busbw (GB/s), #wrong.
// busbw = algbw x 2(n-1)/n for all_reduce, x (n-1)/n for reduce_scatter / all_gather / alltoall,
// x 1 for broadcast.  -j prints one JSON object per size instead of the table.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(cmd)                                                                     \
  do {                                                                                    \
    hipError_t e = (cmd);                                                                 \
    if (e != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(2);                                                                            \
    }                                                                                     \
  } while (0)
#define NCCLCHECK(cmd)                                                                      \
  do {                                                                                      \
    ncclResult_t r = (cmd);                                                                 \
    if (r != ncclSuccess) {                                                                 \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r), __FILE__, __LINE__); \
      exit(3);                                                                              \
    }                                                                                       \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void count_wrong(const float* p, size_t n, float want, unsigned long long* wrong) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    local += fabsf(p[i] - want) > 1e-3f * fabsf(want) ? 1 : 0;
  if (local) atomicAdd(wrong, local);
}

struct Opts {
  std::string op = "all_reduce";
  std::string dtype = "float";
  size_t minb = 8, maxb = 256u << 20;
  int factor = 2, ngpus = 0, iters = 20, warmup = 5, check = 1, json = 0;
};

static size_t elem_size(const std::string& t) { return t == "float" ? 4 : 2; }
static ncclDataType_t nccl_type(const std::string& t) {
  if (t == "bf16") return ncclBfloat16;
  if (t == "half") return ncclFloat16;
  return ncclFloat32;
}

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(1); }
      return argv[++i];
    };
    if (a == "-o") o.op = next();
    else if (a == "-d") o.dtype = next();
    else if (a == "-b") o.minb = strtoull(next(), nullptr, 10);
    else if (a == "-e") o.maxb = strtoull(next(), nullptr, 10);
    else if (a == "-f") o.factor = atoi(next());
    else if (a == "-g") o.ngpus = atoi(next());
    else if (a == "-n") o.iters = atoi(next());
    else if (a == "-w") o.warmup = atoi(next());
    else if (a == "-c") o.check = atoi(next());
    else if (a == "-j") o.json = 1;
    else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 1; }
  }
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (o.ngpus <= 0 || o.ngpus > ndev) o.ngpus = ndev;
  const int n = o.ngpus;
  if (n < 1) { fprintf(stderr, "no GPUs\n"); return 2; }
  if (o.dtype != "float") o.check = 0;  // the fill / verify kernels are fp32-only
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  NCCLCHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  int ver = 0;
  ncclGetVersion(&ver);

  const size_t es = elem_size(o.dtype);
  const bool grows = o.op == "all_gather";  // recv = n x send
  const bool shrinks = o.op == "reduce_scatter";
  std::vector<void*> sendb(n), recvb(n);
  std::vector<hipStream_t> streams(n);
  std::vector<unsigned long long*> wrong(n);
  const size_t max_elems = o.maxb / es;
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(devs[i]));
    HIPCHECK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&sendb[i], o.maxb));
    HIPCHECK(hipMalloc(&recvb[i], grows ? o.maxb * n : o.maxb));
    HIPCHECK(hipMalloc(&wrong[i], sizeof(unsigned long long)));
  }
  if (!o.json) {
    printf("# rccl_perf: %s  %s  ngpus=%d  RCCL %d\n", o.op.c_str(), o.dtype.c_str(), n, ver);
    printf("# %12s %12s %8s %10s %10s %10s %8s\n", "size(B)", "count", "type", "time(us)", "algbw", "busbw",
           "#wrong");
  }
  for (size_t bytes = o.minb; bytes <= o.maxb; bytes *= o.factor) {
    size_t count = bytes / es;  // elements per rank in the send buffer (rccl-tests "count")
    if (shrinks || o.op == "alltoall") count = count / n * n;
    if (count == 0) continue;
    const size_t recv_count = shrinks ? count / n : count;
    auto launch = [&]() {
      NCCLCHECK(ncclGroupStart());
      for (int i = 0; i < n; ++i) {
        if (o.op == "all_reduce")
          NCCLCHECK(ncclAllReduce(sendb[i], recvb[i], count, nccl_type(o.dtype), ncclSum, comms[i], streams[i]));
        else if (o.op == "reduce_scatter")
          NCCLCHECK(ncclReduceScatter(sendb[i], recvb[i], recv_count, nccl_type(o.dtype), ncclSum, comms[i],
                                      streams[i]));
        else if (o.op == "all_gather")
          NCCLCHECK(ncclAllGather(sendb[i], recvb[i], count, nccl_type(o.dtype), comms[i], streams[i]));
        else if (o.op == "broadcast")
          NCCLCHECK(ncclBroadcast(sendb[i], recvb[i], count, nccl_type(o.dtype), 0, comms[i], streams[i]));
        else if (o.op == "alltoall")
          NCCLCHECK(ncclAllToAll(sendb[i], recvb[i], count / n, nccl_type(o.dtype), comms[i], streams[i]));
        else { fprintf(stderr, "unknown op %s\n", o.op.c_str()); exit(1); }
      }
      NCCLCHECK(ncclGroupEnd());
    };
    if (o.check) {
      for (int i = 0; i < n; ++i) {
        HIPCHECK(hipSetDevice(devs[i]));
        hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, streams[i], (float*)sendb[i], count, (float)(i + 1));
      }
    }
    for (int w = 0; w < o.warmup; ++w) launch();
    for (int i = 0; i < n; ++i) { HIPCHECK(hipSetDevice(devs[i])); HIPCHECK(hipStreamSynchronize(streams[i])); }
    std::vector<hipEvent_t> e0(n), e1(n);
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(devs[i]));
      HIPCHECK(hipEventCreate(&e0[i]));
      HIPCHECK(hipEventCreate(&e1[i]));
      HIPCHECK(hipEventRecord(e0[i], streams[i]));
    }
    for (int it = 0; it < o.iters; ++it) launch();
    double worst_ms = 0.0;
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(devs[i]));
      HIPCHECK(hipEventRecord(e1[i], streams[i]));
      HIPCHECK(hipEventSynchronize(e1[i]));
      float ms = 0.f;
      HIPCHECK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      if (ms > worst_ms) worst_ms = ms;
      HIPCHECK(hipEventDestroy(e0[i]));
      HIPCHECK(hipEventDestroy(e1[i]));
    }
    const double us = worst_ms * 1e3 / o.iters;
    const double data_bytes = (double)count * es;  // rccl-tests: algbw = size / time
    const double algbw = data_bytes / (us * 1e-6) / 1e9;
    double factor = 1.0;
    if (o.op == "all_reduce") factor = 2.0 * (n - 1) / n;
    else if (o.op != "broadcast") factor = (double)(n - 1) / n;
    const double busbw = algbw * factor;
    unsigned long long bad = 0;
    if (o.check && o.op == "all_reduce") {
      const float want = n * (n + 1) / 2.0f;
      for (int i = 0; i < n; ++i) {
        HIPCHECK(hipSetDevice(devs[i]));
        HIPCHECK(hipMemsetAsync(wrong[i], 0, sizeof(unsigned long long), streams[i]));
        hipLaunchKernelGGL(count_wrong, dim3(256), dim3(256), 0, streams[i], (const float*)recvb[i], recv_count,
                           want, wrong[i]);
        unsigned long long h = 0;
        HIPCHECK(hipMemcpyAsync(&h, wrong[i], sizeof(h), hipMemcpyDeviceToHost, streams[i]));
        HIPCHECK(hipStreamSynchronize(streams[i]));
        bad += h;
      }
    }
    if (o.json)
      printf("{\"op\": \"%s\", \"dtype\": \"%s\", \"ngpus\": %d, \"bytes\": %zu, \"count\": %zu, \"time_us\": %.3f, "
             "\"algbw_GBps\": %.3f, \"busbw_GBps\": %.3f, \"wrong\": %llu}\n",
             o.op.c_str(), o.dtype.c_str(), n, (size_t)data_bytes, count, us, algbw, busbw, bad);
    else
      printf("  %12zu %12zu %8s %10.2f %10.2f %10.2f %8llu\n", (size_t)data_bytes, count, o.dtype.c_str(), us, algbw,
             busbw, bad);
    fflush(stdout);
    if (bytes > SIZE_MAX / o.factor) break;
  }
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(devs[i]));
    HIPCHECK(hipFree(sendb[i]));
    HIPCHECK(hipFree(recvb[i]));
    HIPCHECK(hipFree(wrong[i]));
    NCCLCHECK(ncclCommDestroy(comms[i]));
  }
  (void)max_elems;
  return 0;
}
