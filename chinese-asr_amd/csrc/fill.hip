// Fill kernels used instead of hipMemsetAsync inside stream-captured regions: replays of
// graphs holding captured memset nodes produced corrupted results under the HIP runtime
// torch ships (ROCm 7.0), while kernel-only graphs replay correctly (tools/debug_replay.py).
#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

__global__ void fill_u32_kernel(uint32_t* __restrict__ p, uint32_t v, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void fill_u8_kernel(uint8_t* __restrict__ p, uint8_t v, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

hipError_t fill_u32(void* p, uint32_t v, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(fill_u32_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<uint32_t*>(p), v, n);
  return hipGetLastError();
}

hipError_t fill_u8(void* p, uint8_t v, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(fill_u8_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<uint8_t*>(p), v, n);
  return hipGetLastError();
}

}  // namespace casr
