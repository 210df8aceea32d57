// Minibatch gather for the device-resident dataset loader (data.py SyntheticDataset, bench.py's
// engine loop): the rows a sampler picked, copied out of every tensor of the dataset (x and y) in
// ONE launch instead of one index_select per tensor -- on the generic engine's host-bound step
// (reference train.py:107-112: next batch, .to(device), forward) each launch is ~4-5 us of host time.
// One workgroup per (output row, tensor) pair walks the row in 16-byte words when the row allows it,
// else in 4-byte words.  An index outside [0, n_rows) yields a zero row and sets *bad (checked by the
// host binding only on request, so the step stays sync-free).
#include "dgt_common.h"
#include "dgt_kernels.h"

namespace dgt {

__global__ __launch_bounds__(256) void gather_rows_kernel(GatherArgs a) {
  const int row = blockIdx.x, t = blockIdx.y;
  const long long src_row = a.idx[row];
  const bool ok = src_row >= 0 && src_row < a.n_rows;
  if (!ok && threadIdx.x == 0 && a.bad) a.bad[0] = 1;
  const int words = a.row_words[t];
  if ((a.vec_mask >> t) & 1) {
    const uint4* s = reinterpret_cast<const uint4*>(a.src[t]) + (ok ? src_row : 0) * (words / 4);
    uint4* d = reinterpret_cast<uint4*>(a.dst[t]) + (long long)row * (words / 4);
    for (int i = threadIdx.x; i < words / 4; i += blockDim.x) d[i] = ok ? s[i] : make_uint4(0, 0, 0, 0);
  } else {
    const unsigned* s = static_cast<const unsigned*>(a.src[t]) + (ok ? src_row : 0) * words;
    unsigned* d = static_cast<unsigned*>(a.dst[t]) + (long long)row * words;
    for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = ok ? s[i] : 0u;
  }
}

hipError_t gather_rows(const GatherArgs& a, int n_out, hipStream_t stream) {
  if (a.count < 1 || a.count > kMaxGather || n_out < 1) return hipErrorInvalidValue;
  int maxw = 1;
  for (int t = 0; t < a.count; ++t) maxw = a.row_words[t] > maxw ? a.row_words[t] : maxw;
  const int vec = maxw / 4 > 0 ? maxw / 4 : 1;
  const int threads = vec >= 256 ? 256 : (vec + 63) / 64 * 64;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(n_out, a.count), dim3(threads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace dgt
