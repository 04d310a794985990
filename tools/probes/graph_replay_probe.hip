// Minimal probe: does a stream-captured hipGraph replay correctly in this process?
// Variants: small vs large by-value kernel args; replay on the capture stream vs another
// stream; many nodes.  Prints one line per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Big {
  int* out;
  int pad[24];
  int val;
};

__global__ void k_small(int* out, int i, int v) { if (threadIdx.x == 0) out[i] = v; }
__global__ void k_big(Big b, int i) { if (threadIdx.x == 0) b.out[i] = b.val + b.pad[3]; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static int run(bool big, bool other_stream, int nodes) {
  int* d; CK(hipMalloc(&d, nodes * sizeof(int)));
  hipStream_t cap, xs; CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking));
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeRelaxed));
  for (int i = 0; i < nodes; ++i) {
    if (big) { Big b{}; b.out = d; b.val = 1000 + i; b.pad[3] = 7; hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, cap, b, i); }
    else hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, cap, d, i, 1000 + i + 7);
  }
  hipGraph_t g; CK(hipStreamEndCapture(cap, &g));
  hipGraphExec_t ex; CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  hipStream_t ls = other_stream ? xs : cap;
  int bad[3] = {0, 0, 0};
  std::vector<int> h(nodes);
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemsetAsync(d, 0, nodes * sizeof(int), ls));
    CK(hipGraphLaunch(ex, ls));
    CK(hipStreamSynchronize(ls));
    CK(hipMemcpy(h.data(), d, nodes * sizeof(int), hipMemcpyDeviceToHost));
    for (int i = 0; i < nodes; ++i) bad[rep] += h[i] != 1000 + i + 7;
  }
  printf("big=%d other_stream=%d nodes=%d bad per replay: %d %d %d\n", big, other_stream, nodes, bad[0], bad[1], bad[2]);
  CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g)); CK(hipFree(d));
  return 0;
}

extern "C" int graph_probe() {
  int rv = 0, dv = 0;
  hipRuntimeGetVersion(&rv); hipDriverGetVersion(&dv);
  printf("hip runtime %d driver %d\n", rv, dv);
  for (int big = 0; big < 2; ++big)
    for (int os = 0; os < 2; ++os)
      for (int n : {4, 300}) if (run(big, os, n)) return 1;
  return 0;
}

int main() { return graph_probe(); }
