// Isolation probe for the exit crash under rocprofv3 (cooperative launch): one
// trivial kernel, launched with hipLaunchCooperativeKernel (argv[1] = "coop") or an ordinary
// launch ("plain"), synchronised, device memory freed, then a normal exit.  Nothing of the casr
// library is involved.  Run: rocprofv3 --kernel-trace --stats -d DIR -o run -- ./coop_exit_probe coop
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void touch(int* p) { p[blockIdx.x * blockDim.x + threadIdx.x] = (int)threadIdx.x; }

int main(int argc, char** argv) {
  const bool coop = argc > 1 && std::strcmp(argv[1], "coop") == 0;
  int* d = nullptr;
  if (hipMalloc(&d, 256 * 512 * sizeof(int)) != hipSuccess) return 2;
  hipError_t e;
  if (coop) {
    void* args[] = {&d};
    e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(touch), dim3(256), dim3(512), args, 0, nullptr);
  } else {
    hipLaunchKernelGGL(touch, dim3(256), dim3(512), 0, nullptr, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipFree(d);
  std::printf("%s launch: %s\n", coop ? "cooperative" : "plain", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
