// Log-mel kernel variants at B = 256 x 8 s (diagnostic probe, not shipped): frames per wave.  Times
// each variant with HIP events and compares its output with variant 0 (the shipped default).  Round
// 4 also measured, with a templated copy of the kernel (profiles/r04/logmel/variants_r04g.txt): the
// filter weights in registers (adopted: 7 % faster, same bits) and the stage 0 -> 1 exchange by
// v_permlane16/32_swap (5 % faster, but hipcc then contracts the complex products differently: up to
// 8e-3 in log-mel against the LDS form, so not adopted).  With -DFE_NI and FE_SRC pointing at a copy
// of frontend.hip whose kernel takes a second template parameter NI (frames in flight per wave,
// interleaved through every stage) it also times NI = 2 and 4: 191 / 215 us against 181 us for
// the default (profiles/r04/logmel/variants_ni_r04j.txt; 146 / 207 VGPRs), so not adopted.  With
// -DFE_LB and a copy whose second parameter is the __launch_bounds__ minimum waves per SIMD, 5 and 6
// waves: 253 / 412 us (36 / 51 VGPRs spilled; variants_lb_r04o.txt), not adopted.  Build:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I chinese-asr_amd/csrc -DFE_SRC=<file> \
//     tools/probes/logmel_variants.hip -o tools/probes/logmel_variants
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#ifndef FE_SRC
#define FE_SRC "frontend.hip"
#endif
#include FE_SRC

using namespace casr;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                          \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

#if defined(FE_NI) || defined(FE_LB)  // a kernel source with a second template parameter
                                     // (frames in flight, or the minimum waves per SIMD)
#define FE_KERNEL(FPW, NI) log_mel_kernel<FPW, NI>
#else
#define FE_KERNEL(FPW, NI) log_mel_kernel<FPW>
#endif

template <int FPW, int NI = 1>
static float run(const char* name, const float* wav, const int* ns, int B, int N, int T, const FrontendConst* k,
                 float* out, int* fr, int* err, const std::vector<float>* ref, std::vector<float>* keep) {
  constexpr int FPB = 4 * FPW;
  dim3 grid((T + FPB - 1) / FPB, B);
  auto go = [&] { hipLaunchKernelGGL((FE_KERNEL(FPW, NI)), grid, dim3(256), 0, nullptr, wav, ns, N, T, 0.97f, k, out, fr, err); };
  go();
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int it = 20;
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < it; ++i) go();
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<float> h((size_t)B * T * 80);
  (void)hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
  double md = 0.0;
  size_t ndiff = 0;
  if (ref)
    for (size_t i = 0; i < h.size(); ++i) {
      const double d = std::fabs((double)h[i] - (*ref)[i]);
      md = d > md ? d : md;
      ndiff += h[i] != (*ref)[i];
    }
  if (keep) *keep = h;
  std::printf("%-34s %8.1f us   max|diff| vs v0 %.3g  (%zu of %zu differ)\n", name, 1000.f * ms / it, md, ndiff, h.size());
  return ms / it;
}

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
  std::vector<int> ns(B, N);
  FrontendConst hc;
  build_frontend_const(&hc);
  float *wav, *out;
  int *nsd, *fr, *err;
  FrontendConst* k;
  CK(hipMalloc(&wav, w.size() * 4));
  CK(hipMalloc(&out, (size_t)B * T * 80 * 4));
  CK(hipMalloc(&nsd, B * 4));
  CK(hipMalloc(&fr, B * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&k, sizeof hc));
  CK(hipMemcpy(wav, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(nsd, ns.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(k, &hc, sizeof hc, hipMemcpyHostToDevice));
  CK(hipMemset(err, 0, 4));
  std::vector<float> ref;
  std::printf("B = %d, %d samples, %d frames\n", B, N, T);
  run<8>("v0 FPW 8 (default)", wav, nsd, B, N, T, k, out, fr, err, nullptr, &ref);
  run<4>("v1 FPW 4", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<16>("v2 FPW 16", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
#ifdef FE_LB  // log_mel_kernel<FPW, MINW>: __launch_bounds__(256, MINW)
  run<8, 5>("v3 FPW 8, 5 waves per SIMD", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<8, 6>("v4 FPW 8, 6 waves per SIMD", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<16, 5>("v5 FPW 16, 5 waves per SIMD", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<16, 6>("v6 FPW 16, 6 waves per SIMD", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
#endif
#ifdef FE_NI
  run<8, 2>("v3 FPW 8, 2 frames in flight", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<16, 2>("v4 FPW 16, 2 frames in flight", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<8, 4>("v5 FPW 8, 4 frames in flight", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
  run<8, 1>("v6 FPW 8 (NI template, 1)", wav, nsd, B, N, T, k, out, fr, err, &ref, nullptr);
#endif
  int he = 0;
  (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
  std::printf("device flags %d\n", he);
  return 0;
}
