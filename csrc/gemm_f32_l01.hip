// Exact-fp32 MFMA GEMM, operand layouts A MK / B KN (gemm_f32.hip).
#include "gemm_f32_kernel.h"

namespace dgt {
hipError_t gemm_f32_l01(const GemmF32Args& a, const GemmF32Plan& p, bool vec, hipStream_t stream) {
  return f32g::dispatch<0, 1>(a, p, vec, stream);
}
}  // namespace dgt
