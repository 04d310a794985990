// The 16-lane log-mel kernel (frontend.hip log_mel_q16_kernel, round 5) against the one-wave-per-frame
// kernel at B = 256 x 8 s and on a ragged batch: bitwise comparison and HIP-event timing.  Diagnostic.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I chinese-asr_amd/csrc \
//     tools/probes/logmel_q16_probe.hip -o tools/probes/logmel_q16_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "frontend.hip"

using namespace casr;

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main() {
  const int B = 256, N = 8 * 16000, T = frontend_frames(N);
  std::vector<float> w((size_t)B * N);
  uint64_t st = 88172645463325252ull;
  for (auto& x : w) {  // xorshift + Box-Muller: 0.1 x standard normal
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    const double u1 = ((st >> 11) + 1.0) / 9007199254740993.0;
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    const double u2 = (st >> 11) / 9007199254740992.0;
    x = (float)(0.1 * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2));
  }
  FrontendConst hc;
  build_frontend_const(&hc);
  float *wav, *o0, *o1;
  int *nsd, *fr, *err;
  FrontendConst* k;
  CK(hipMalloc(&wav, w.size() * 4));
  CK(hipMalloc(&o0, (size_t)B * T * 80 * 4));
  CK(hipMalloc(&o1, (size_t)B * T * 80 * 4));
  CK(hipMalloc(&nsd, B * 4));
  CK(hipMalloc(&fr, B * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&k, sizeof hc));
  CK(hipMemcpy(wav, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(k, &hc, sizeof hc, hipMemcpyHostToDevice));
  CK(hipMemset(err, 0, 4));
  for (int ragged = 0; ragged < 2; ++ragged) {
    std::vector<int> ns(B, N);
    if (ragged)
      for (int b = 0; b < B; ++b) ns[b] = 513 + (int)((b * 2654435761u) % (unsigned)(N - 513));
    CK(hipMemcpy(nsd, ns.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMemset(o0, 0xFF, (size_t)B * T * 80 * 4));
    CK(hipMemset(o1, 0x7F, (size_t)B * T * 80 * 4));
    CK(launch_log_mel(wav, nsd, B, N, T, 0.97f, k, o0, fr, err, nullptr, 0));
    CK(launch_log_mel(wav, nsd, B, N, T, 0.97f, k, o1, fr, err, nullptr, 1));
    CK(hipDeviceSynchronize());
    std::vector<float> h0((size_t)B * T * 80), h1(h0.size());
    CK(hipMemcpy(h0.data(), o0, h0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), o1, h1.size() * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    double mx = 0;
    for (size_t i = 0; i < h0.size(); ++i)
      if (std::memcmp(&h0[i], &h1[i], 4) != 0) {
        ++diff;
        mx = std::fmax(mx, std::fabs((double)h0[i] - h1[i]));
      }
    std::printf("%s: %zu of %zu outputs differ (max |d| %.3g)\n", ragged ? "ragged" : "B = 256 x 8 s", diff, h0.size(), mx);
  }
  std::vector<int> ns(B, N);
  CK(hipMemcpy(nsd, ns.data(), B * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    for (int form = 0; form < 2; ++form) {
      const int it = 20;
      CK(hipEventRecord(e0, nullptr));
      for (int i = 0; i < it; ++i) CK(launch_log_mel(wav, nsd, B, N, T, 0.97f, k, form ? o1 : o0, fr, err, nullptr, form));
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("form %d (%s): %.1f us\n", form, form ? "16 lanes per frame" : "one wave per frame", 1000.f * ms / it);
    }
  int he = 0;
  CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
  std::printf("device flags %d\n", he);
  return 0;
}
