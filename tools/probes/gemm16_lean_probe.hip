// Standalone bitwise check and interleaved timing of the lean ping-pong input projection
// (gemm16.hip gemm16_pp_lean_kernel, round 6) against gemm16_pp_kernel<…, KM = true>, on
// 16-k-block-major images at the bench shape (M = 256 x 266, N = 2048; Kp = 768 with K = 720, and
// Kp = 512) and at a ragged M.  Diagnostic only.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../chinese-asr_amd/csrc \
//         gemm16_lean_probe.hip -o gemm16_lean_probe && ./gemm16_lean_probe [reps]
#include <cstdio>
#include <cstdlib>
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

// a random s16 image, 16-k-block major: [Kp / 16][rows][16 hi | 16 lo] halves, zero past K
static void make_km(std::vector<uint16_t>& km, int rows, int Kp, int K, unsigned seed, float scale) {
  km.assign((size_t)rows * Kp * 2, 0);
  unsigned s = seed;
  for (int r = 0; r < rows; ++r)
    for (int k = 0; k < K; ++k) {
      s = s * 1664525u + 1013904223u;
      const float x = (((s >> 8) & 0xFFFF) / 32768.0f - 1.0f) * scale;
      const _Float16 hi = (_Float16)x;
      const float lo = (x - (float)hi) * 2048.0f;
      uint16_t* o = km.data() + ((size_t)(k / 16) * rows + r) * 32;
      o[k % 16] = f2h(x);
      o[16 + k % 16] = f2h(lo);
    }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 4;
  int G = 0;
  CK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, 0));
  const int N = 2048;
  for (int Kp : {768, 512}) {
    const int K = Kp == 768 ? 720 : 512, nk16 = (K + 15) / 16;
    for (int M : {256 * 266, 37 * 266 + 5}) {
      std::vector<uint16_t> a, w;
      make_km(a, M, Kp, K, 1u + M, 3.0f);
      make_km(w, N, Kp, K, 2u, 0.05f);
      std::vector<float> bias(N);
      for (int i = 0; i < N; ++i) bias[i] = 0.001f * (i % 97) - 0.05f;
      float *dA, *dW, *dB, *dC0, *dC1;
      CK(hipMalloc(&dA, a.size() * 2));
      CK(hipMalloc(&dW, w.size() * 2));
      CK(hipMalloc(&dB, N * 4));
      CK(hipMalloc(&dC0, (size_t)M * N * 4 + 4096));
      CK(hipMalloc(&dC1, (size_t)M * N * 4 + 4096));
      CK(hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dW, w.data(), w.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dB, bias.data(), N * 4, hipMemcpyHostToDevice));
      const int NB = N / G16_N, NM = (M + G16_M - 1) / G16_M;
      int NG = 1;
      while (NG < 8 && NB % (NG * 2) == 0 && (size_t)(NB / NG) * G16_N * Kp * 4 > (3u << 20)) NG *= 2;
      const Order16 o{NB, NM, NG};
      const int grid = std::min(o.blocks(), G);
      auto run_pp = [&](float* C) {
        hipLaunchKernelGGL((gemm16_pp_kernel<0, 1, 0, 0, true>), dim3(grid), dim3(512), 0, 0, dA, dW, dB, C, M, N, Kp, o,
                           o.blocks(), nk16, M);
      };
      auto run_lean = [&](float* C) {
        hipLaunchKernelGGL(gemm16_pp_lean_kernel, dim3(grid), dim3(512), 0, 0, dA, dW, dB, C, M, N, o, o.blocks(), nk16, M);
      };
      CK(hipMemset(dC0, 0xFF, (size_t)M * N * 4 + 4096));
      run_pp(dC0);
      CK(hipDeviceSynchronize());
      std::vector<float> c0((size_t)M * N + 1024), c1((size_t)M * N + 1024);
      CK(hipMemcpy(c0.data(), dC0, c0.size() * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (int r = 0; r < reps; ++r) {
        CK(hipMemset(dC1, 0xFF, (size_t)M * N * 4 + 4096));
        run_lean(dC1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(c1.data(), dC1, c1.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < c1.size(); ++i)
          if (memcmp(&c0[i], &c1[i], 4) != 0) {
            if (bad < 3) printf("  rep %d diff at %zu: %g vs %g\n", r, i, c0[i], c1[i]);
            ++bad;
          }
      }
      printf("Kp %d M %d: lean vs pp-km: %zu differing words (outputs + guard words) over %d reps\n", Kp, M, bad, reps);
      fflush(stdout);
      if (M == 256 * 266) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int rep = 0; rep < 5; ++rep)
          for (int v = 0; v < 2; ++v) {
            const int iters = 10;
            CK(hipEventRecord(e0));
            for (int i = 0; i < iters; ++i) {
              if (v) run_lean(dC1);
              else run_pp(dC1);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double flop = 2.0 * M * N * (double)(16 * nk16) * 3;
            printf("Kp %d %-8s %8.1f us  %6.0f TF/s f16\n", Kp, v ? "lean" : "pp:km", 1000.0 * ms / iters,
                   flop / (ms / iters * 1e-3) / 1e12);
          }
        fflush(stdout);
      }
      CK(hipFree(dA));
      CK(hipFree(dW));
      CK(hipFree(dB));
      CK(hipFree(dC0));
      CK(hipFree(dC1));
    }
  }
  return 0;
}
