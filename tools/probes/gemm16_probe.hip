// Standalone timing + bitwise check of the s16x3 input-projection kernels (gemm16.hip) at the
// bench shape (M = 256 x 266 rows, N = 2048, Kp = 768 / 512).  Diagnostic only.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../chinese-asr_amd/csrc \
//         gemm16_probe.hip -o gemm16_probe && ./gemm16_probe
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../chinese-asr_amd/csrc/gemm16.hip"
using namespace casr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static uint16_t f2h(float x) {
  _Float16 h = (_Float16)x;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

// s16 row image: per 32-k tile [32 hi | 32 lo] halves
static void make_image(std::vector<uint16_t>& img, int rows, int Kp, int K, unsigned seed, float scale) {
  img.assign((size_t)rows * Kp * 2, 0);
  unsigned s = seed;
  auto rnd = [&] {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f;
  };
  for (int r = 0; r < rows; ++r)
    for (int k = 0; k < K; ++k) {
      const float x = rnd() * scale;
      const _Float16 hi = (_Float16)x;
      const float lo = (x - (float)hi) * 2048.0f;
      uint16_t* t = img.data() + ((size_t)r * Kp + (k / 32) * 32) * 2;
      t[k % 32] = f2h(x);
      t[32 + k % 32] = f2h(lo);
    }
}

int main() {
  const int M = 256 * 266, N = 2048;
  for (int Kp : {768, 512}) {
    const int K = Kp == 768 ? 720 : 512;
    std::vector<uint16_t> a, w;
    make_image(a, M, Kp, K, 1u, 3.0f);
    make_image(w, N, Kp, K, 2u, 0.05f);
    std::vector<float> bias(N);
    for (int i = 0; i < N; ++i) bias[i] = 0.001f * (i % 97) - 0.05f;
    float *dA, *dW, *dB, *dC0, *dC1;
    CK(hipMalloc(&dA, a.size() * 2));
    CK(hipMalloc(&dW, w.size() * 2));
    CK(hipMalloc(&dB, N * 4));
    CK(hipMalloc(&dC0, (size_t)M * N * 4));
    CK(hipMalloc(&dC1, (size_t)M * N * 4));
    CK(hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dW, w.data(), w.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, bias.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dC0, 0, (size_t)M * N * 4));
    CK(hipMemset(dC1, 0xFF, (size_t)M * N * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[6] = {"bias_kernel<4>", "persist", "p:no-dma", "p:no-mfma", "p:no-stores", "p:dma-only"};
    float* outs[6] = {dC0, dC1, dC1, dC1, dC1, dC1};
    for (int rep = 0; rep < 3; ++rep)
      for (int v = 0; v < 6; ++v) {
        const int NB = N / G16_N, NM = (M + G16_M - 1) / G16_M;
        int NG = 1;
        while (NG < 8 && NB % (NG * 2) == 0 && (size_t)(NB / NG) * G16_N * Kp * 4 > (3u << 20)) NG *= 2;
        const Order16 order{NB, NM, NG};
        const int iters = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) {
          if (v == 0)
            hipLaunchKernelGGL(gemm16_bias_kernel<4>, dim3(order.blocks()), dim3(512), 0, 0, dA, dW, dB, outs[v], M,
                               N, Kp, order);
          else if (v == 1)
            hipLaunchKernelGGL(gemm16_persist_kernel<0>, dim3(256), dim3(512), 0, 0, dA, dW, dB, outs[v], M, N, Kp,
                               order, order.blocks(), Kp / G16_K);
          else if (v == 2)
            hipLaunchKernelGGL(gemm16_persist_kernel<1>, dim3(256), dim3(512), 0, 0, dA, dW, dB, outs[v], M, N, Kp,
                               order, order.blocks(), Kp / G16_K);
          else if (v == 3)
            hipLaunchKernelGGL(gemm16_persist_kernel<2>, dim3(256), dim3(512), 0, 0, dA, dW, dB, outs[v], M, N, Kp,
                               order, order.blocks(), Kp / G16_K);
          else if (v == 4)
            hipLaunchKernelGGL(gemm16_persist_kernel<4>, dim3(256), dim3(512), 0, 0, dA, dW, dB, outs[v], M, N, Kp,
                               order, order.blocks(), Kp / G16_K);
          else
            hipLaunchKernelGGL(gemm16_persist_kernel<6>, dim3(256), dim3(512), 0, 0, dA, dW, dB, outs[v], M, N, Kp,
                               order, order.blocks(), Kp / G16_K);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double flop = 2.0 * M * N * (double)Kp * 3;
        printf("Kp %d %-16s %8.1f us  %6.0f TF/s f16\n", Kp, names[v], 1000.0 * ms / iters, flop / (ms / iters * 1e-3) / 1e12);
      }
    // the bitwise check needs the persist result: rerun it last
    hipLaunchKernelGGL(gemm16_persist_kernel<0>, dim3(256), dim3(512), 0, 0, dA, dW, dB, dC1, M, N, Kp,
                       Order16{N / G16_N, (M + G16_M - 1) / G16_M, 2}, Order16{N / G16_N, (M + G16_M - 1) / G16_M, 2}.blocks(), Kp / G16_K);
    CK(hipDeviceSynchronize());
    std::vector<float> c0((size_t)M * N), c1((size_t)M * N);
    CK(hipMemcpy(c0.data(), dC0, c0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c1.data(), dC1, c1.size() * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < c0.size(); ++i)
      if (memcmp(&c0[i], &c1[i], 4) != 0) {
        if (diff < 5) printf("  diff at %zu (row %zu col %zu): %g vs %g\n", i, i / N, i % N, c0[i], c1[i]);
        ++diff;
      }
    printf("Kp %d: %zu of %zu outputs differ bitwise\n", Kp, diff, c0.size());
    hipFree(dA);
    hipFree(dW);
    hipFree(dB);
    hipFree(dC0);
    hipFree(dC1);
  }
  return 0;
}
