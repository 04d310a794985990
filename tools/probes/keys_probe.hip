// Standalone timing of the s16x3 keys GEMM forms (encoder.hip): keys16_kernel (W_enc in registers,
// 16-row items through an LDS ring) against gemm_nt_kernel<KeysEpi, true> (128 x 128 tiles), at the
// bench shape (B = 256, Tp = 266, C = 512, A = 128), outputs compared bit for bit.  Diagnostic only.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../chinese-asr_amd/csrc \
//         keys_probe.hip ../../chinese-asr_amd/casr/_obj/*.o -o keys_probe   (the product objects
//         resolve encoder.hip's external references; this file's copy of the kernels is the probe's)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "casr_common.h"
#include "casr_internal.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

using namespace casr;

static uint16_t f2h(float x) {
  _Float16 h = (_Float16)x;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

// s16 row image [rows][K] words of [32 hi | 32 lo] halves per 32-k tile
static void make_image(std::vector<uint16_t>& img, int rows, int K, unsigned seed, float scale) {
  img.assign((size_t)rows * K * 2, 0);
  unsigned s = seed;
  for (int r = 0; r < rows; ++r)
    for (int k = 0; k < K; ++k) {
      s = s * 1664525u + 1013904223u;
      const float x = (((s >> 8) & 0xFFFF) / 32768.0f - 1.0f) * scale;
      const _Float16 hi = (_Float16)x;
      uint16_t* t = img.data() + ((size_t)r * K + (k / 32) * 32) * 2;
      t[k % 32] = f2h(x);
      t[32 + k % 32] = f2h((x - (float)hi) * 2048.0f);
    }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256, Tp = 266, Tq = (Tp + 3) & ~3, M = B * Tp;
  std::vector<uint16_t> a, w;
  make_image(a, M, C, 7u, 1.0f);
  make_image(w, A, C, 9u, 0.05f);
  std::vector<float> bias(A);
  for (int i = 0; i < A; ++i) bias[i] = 0.01f * (i % 13);
  float *dA, *dW, *dB, *dK0, *dK1;
  const size_t kn = (size_t)2 * B * A * Tq;
  CK(hipMalloc(&dA, a.size() * 2));
  CK(hipMalloc(&dW, w.size() * 2));
  CK(hipMalloc(&dB, A * 4));
  CK(hipMalloc(&dK0, kn * 4));
  CK(hipMalloc(&dK1, kn * 4));
  CK(hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, w.data(), w.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, bias.data(), A * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dK0, 0, kn * 4));
  CK(hipMemset(dK1, 0, kn * 4));
  CK(launch_keys_s16(dA, B, Tp, dW, dB, dK0, 0, 0));
  CK(launch_keys_s16(dA, B, Tp, dW, dB, dK1, 0, 1));
  CK(hipDeviceSynchronize());
  std::vector<float> k0(kn), k1(kn);
  CK(hipMemcpy(k0.data(), dK0, kn * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(k1.data(), dK1, kn * 4, hipMemcpyDeviceToHost));
  size_t diff = 0;
  for (int half = 0; half < 2; ++half)
    for (int b = 0; b < B; ++b)
      for (int c = 0; c < A; ++c)
        for (int t = 0; t < Tp; ++t) {
          const size_t i = (size_t)half * B * A * Tq + ((size_t)b * A + c) * Tq + t;
          if (memcmp(&k0[i], &k1[i], 4) != 0) ++diff;
        }
  printf("B %d: keys16 vs tiles: %zu differing of %zu\n", B, diff, (size_t)2 * B * A * Tp);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    for (int form = 0; form < 2; ++form) {
      const int iters = 20;
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) CK(launch_keys_s16(dA, B, Tp, dW, dB, form ? dK1 : dK0, 0, form));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("rep %d %-8s %7.1f us\n", rep, form ? "keys16" : "tiles", 1000.f * ms / iters);
    }
  return 0;
}
