// kernels_util.hip -- the measurement kernels of the bench line (no part of the DSP path).
//
//   k_copy16   the HBM copy ceiling of k_rdx's bytes in the same process (bench.py
//              copy_ceiling): one 16-byte nontemporal load and store per thread over a grid
//              of one thread per 16 bytes (DESIGN.md 4.0.1 part A's shape: the fastest copy
//              of these bytes probed on MI355X, 2.63 ms for 17.2 GB).
#include <hip/hip_runtime.h>

#include "fmcw_internal.h"

namespace fmcw {

typedef float f4v_ __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy16(const f4v_* __restrict__ src, f4v_* __restrict__ dst, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

hipError_t launch_copy16(const void* src, void* dst, int64_t bytes, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
    return hipErrorInvalidValue;
  const int64_t n16 = bytes >> 4, blocks = (n16 + 255) / 256;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_copy16, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const f4v_*>(src),
                     static_cast<f4v_*>(dst), n16);
  return hipGetLastError();
}

}  // namespace fmcw
