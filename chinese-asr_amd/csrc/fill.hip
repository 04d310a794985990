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

// Several fills / copies in one launch (blockIdx.y = segment): the small per-call resets of the
// recurrence hand-off buffers and of the decode state, and the copies of a decode graph's outputs
// to the caller's buffers, were one launch each (≈5 µs apiece on the profile's timeline).
__global__ void fill_multi_kernel(FillList fl) {
  const FillSeg sg = fl.seg[blockIdx.y];
  const size_t step = (size_t)gridDim.x * blockDim.x;
  if (sg.bytes == 4) {
    uint32_t* p = reinterpret_cast<uint32_t*>(sg.p);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.count; i += step) p[i] = sg.v;
  } else {
    uint8_t* p = reinterpret_cast<uint8_t*>(sg.p);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.count; i += step) p[i] = (uint8_t)sg.v;
  }
}

hipError_t fill_multi(const FillList& fl, hipStream_t s) {
  if (fl.n <= 0 || fl.n > FILL_MAX_SEG) return hipErrorInvalidValue;
  size_t mx = 0;
  for (int i = 0; i < fl.n; ++i) mx = std::max(mx, fl.seg[i].count);
  if (mx == 0) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<size_t>((mx + 255) / 256, 1024);
  hipLaunchKernelGGL(fill_multi_kernel, dim3(blocks, fl.n), dim3(256), 0, s, fl);
  return hipGetLastError();
}

__global__ void copy_multi_kernel(CopyList cl) {
  const CopySeg sg = cl.seg[blockIdx.y];
  const size_t step = (size_t)gridDim.x * blockDim.x;
  const bool w4 = ((reinterpret_cast<uintptr_t>(sg.dst) | reinterpret_cast<uintptr_t>(sg.src) | sg.bytes) & 3) == 0;
  if (w4) {
    uint32_t* d = reinterpret_cast<uint32_t*>(sg.dst);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(sg.src);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.bytes / 4; i += step) d[i] = q[i];
  } else {
    uint8_t* d = reinterpret_cast<uint8_t*>(sg.dst);
    const uint8_t* q = reinterpret_cast<const uint8_t*>(sg.src);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < sg.bytes; i += step) d[i] = q[i];
  }
}

hipError_t copy_multi(const CopyList& cl, hipStream_t s) {
  if (cl.n <= 0 || cl.n > FILL_MAX_SEG) return hipErrorInvalidValue;
  size_t mx = 0;
  for (int i = 0; i < cl.n; ++i) mx = std::max(mx, cl.seg[i].bytes / 4 + 1);
  const unsigned blocks = (unsigned)std::min<size_t>((mx + 255) / 256, 1024);
  hipLaunchKernelGGL(copy_multi_kernel, dim3(blocks, cl.n), dim3(256), 0, s, cl);
  return hipGetLastError();
}

// CASR_OPT_DIAG_COLD: stream a buffer larger than every cache level through the L2s, so the next
// launch finds neither its L2 lines nor its Infinity-Cache lines (a sum no input can make equal
// to the sentinel keeps the loads live; nothing is ever stored)
__global__ void flush_caches_kernel(const float4* __restrict__ p, size_t n, float* __restrict__ never) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234567.f && never) never[0] = acc;
}

hipError_t flush_caches(const void* buf, size_t bytes, hipStream_t s) {
  hipLaunchKernelGGL(flush_caches_kernel, dim3(4096), dim3(256), 0, s, reinterpret_cast<const float4*>(buf),
                     bytes / 16, nullptr);
  return hipGetLastError();
}

}  // namespace casr
