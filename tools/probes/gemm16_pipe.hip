// Input-projection experiment (diagnostic probe, not shipped): the persistent s16x3 kernel with
// 16-deep half stages on a 4-slot LDS ring (three halves in flight: 96 KB, against one 64 KB stage
// now) and the fragments of half p + 1 read from LDS into a second register set while the MFMAs of
// half p run, so the LDS latency after each barrier is no longer exposed.  Same operands and the
// same MFMA order per accumulator as gemm16_bias_kernel<4> (k tile, then its two 16-deep halves,
// then w_hi 2^11 / w_lo / a_lo), so the outputs must be bitwise equal; the probe checks all of them.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../chinese-asr_amd/csrc \
//         gemm16_pipe.hip -o gemm16_pipe && ./gemm16_pipe
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

namespace {
// a half slot: 256 A rows then 256 W rows of 16 words (64 B: logical chunks hi 2ks, hi 2ks + 1,
// lo 2ks, lo 2ks + 1 of the row's 32-k tile), logical chunk j of row r at j ^ ((r >> 2) & 3)
constexpr int HP_ROWW = 16, HP_OP = 256 * HP_ROWW, HP_SLOT = 2 * HP_OP, HP_NS = 4;
constexpr int HP_LDS = HP_NS * HP_SLOT + 2 * G16_N;  // 4 slots + two bias slots (129 KB)
constexpr int HP_EPI_STORES = 32;                    // float4 stores per thread per tile

template <int VM>
__device__ __forceinline__ void hp_vm_wait() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
}

__global__ __launch_bounds__(512, 2) void gemm16_pipe_kernel(const float* __restrict__ A16,
                                                            const float* __restrict__ W16,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ Cout, int M, int N, int Kp,
                                                            Order16 order, int total, int nk) {
  __shared__ __attribute__((aligned(16))) float lds[HP_LDS];
  constexpr int NT = 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;
  const int r32 = lane & 31, hsel = lane >> 5;
  const int G = gridDim.x, H = 2 * nk;
  float* const bias_lds = lds + HP_NS * HP_SLOT;

  auto next_tile = [&](int L, int& n, int& m) {
    while (L < total && !order.tile(L, n, m)) L += G;
    return L;
  };
  // the tiles of this workgroup, (n, m) of the current one and the next
  int n0, m0, n1 = 0, m1 = 0;
  int L0 = next_tile(blockIdx.x, n0, m0);
  if (L0 >= total) return;
  int L1 = next_tile(L0 + G, n1, m1);
  int ntl = 1;
  for (int L = L1, a, b; L < total; L = next_tile(L + G, a, b)) ++ntl;
  const int P = ntl * H;  // halves of this workgroup

  // DMA of half p (tile i = p / H: the current (i == cur) or the next one) into slot p % 4: wave
  // w stages A rows and W rows 32w .. 32w + 31, 16 rows per instruction (lane: row lane >> 2,
  // physical chunk lane & 3); wave 0 adds the tile's bias with its half 0
  auto dma = [&](int p, int n, int m, int tpar) {
    const int hh = p % H, kt = hh >> 1, ks = hh & 1;
    float* slot = lds + (p % HP_NS) * HP_SLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wave * 32 + j * 16 + (lane >> 2), pc = lane & 3, lc = pc ^ ((row >> 2) & 3);
      const int gc = lc < 2 ? 2 * ks + lc : 4 + 2 * ks + (lc - 2);
      const int k0 = kt * G16_K + gc * 4;
      lds_dma16(A16 + (size_t)min(m * G16_M + row, M - 1) * Kp + k0, slot + (wave * 32 + j * 16) * HP_ROWW);
      lds_dma16(W16 + (size_t)min(n * G16_N + row, N - 1) * Kp + k0, slot + HP_OP + (wave * 32 + j * 16) * HP_ROWW);
    }
    if (hh == 0 && wave == 0) lds_dma16(bias + min(n * G16_N + lane * 4, N - 4), bias_lds + tpar * G16_N);
  };
  // A fragments of a half: read one phase ahead (two register sets); the W fragments (4 reads)
  // at the start of their own phase
  struct Frag {
    f16x8 ah[4], al[4];
  };
  struct WFrag {
    f16x8 wh[NT], wl[NT];
  };
  auto read_w = [&](int p, WFrag& f) {
    const float* slot = lds + (p % HP_NS) * HP_SLOT;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = wn * 32 * NT + t * 32 + r32, sw = (row >> 2) & 3;
      f.wh[t] = *reinterpret_cast<const f16x8*>(slot + HP_OP + row * HP_ROWW + ((hsel ^ sw) << 2));
      f.wl[t] = *reinterpret_cast<const f16x8*>(slot + HP_OP + row * HP_ROWW + (((2 + hsel) ^ sw) << 2));
    }
  };
  auto read = [&](int p, Frag& f) {
    const float* slot = lds + (p % HP_NS) * HP_SLOT;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm) {
      const int row = wm * 128 + tm * 32 + r32, sw = (row >> 2) & 3;
      f.ah[tm] = *reinterpret_cast<const f16x8*>(slot + row * HP_ROWW + ((hsel ^ sw) << 2));
      f.al[tm] = *reinterpret_cast<const f16x8*>(slot + row * HP_ROWW + (((2 + hsel) ^ sw) << 2));
    }
  };
  f32x16 acc[4][NT];
  const _Float16 two11 = (_Float16)2048.0f;
  auto mfma = [&](const Frag& f, const WFrag& w) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f16x8 w1 = w.wh[t] * two11;
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[tm], w1, acc[tm][t], 0, 0, 0);
        acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[tm], w.wl[t], acc[tm][t], 0, 0, 0);
        acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.al[tm], w.wh[t], acc[tm][t], 0, 0, 0);
      }
    }
  };
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto zero = [&] {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  };
  // the (n, m) of half q: the current tile or (q in the next tile) the next one
  int cur = 0, tpar = 0;  // tile index of n0/m0 and its bias slot
  auto dma_at = [&](int q) {
    if (q >= P) return;
    if (q / H == cur) dma(q, n0, m0, tpar);
    else dma(q, n1, m1, tpar ^ 1);
  };

  zero();
  dma_at(0);
  dma_at(1);
  dma_at(2);
  hp_vm_wait<8>();  // own half 0 landed (halves 1, 2: 8 instructions younger; wave 0's bias is older)
  barrier();
  Frag fa, fb;
  read(0, fa);
  int after_epi = -1;  // stores issued after the last DMA, or -1
  // one phase: wait for half p + 1 (own DMA), barrier (everyone's half p + 1 landed, everyone done
  // reading slot (p + 3) % 4), DMA half p + 3, read half p + 1 into the other set, MFMAs of half p
  auto phase = [&](int p, Frag& use, Frag& next) {
    if (p + 1 < P) {  // younger than half p + 1: half p + 2 (if any), then the epilogue's stores
      if (p + 2 >= P) hp_vm_wait<0>();
      else if (after_epi == HP_EPI_STORES) hp_vm_wait<4 + HP_EPI_STORES>();
      else if (after_epi >= 0) hp_vm_wait<0>();
      else hp_vm_wait<4>();
    }
    after_epi = -1;
    barrier();
    dma_at(p + 3);
    WFrag wf;
    read_w(p, wf);
    if (p + 1 < P) read(p + 1, next);
    mfma(use, wf);
  };
  for (int p = 0; p < P; p += 2) {
    phase(p, fa, fb);
    phase(p + 1, fb, fa);
    // p + 1 is the last half of tile `cur` (H is even): epilogue through slot (p + 1) % 4, eight
    // rounds of 32 rows, float4 stores + bias
    if ((p + 2) % H == 0) {
      float* slab = lds + ((p + 1) % HP_NS) * HP_SLOT;
      const float* bl = bias_lds + tpar * G16_N;
      const int c4 = tid & 63, r0 = tid >> 6;
      const int mrow0 = m0 * G16_M, col = n0 * G16_N + c4 * 4;
      int nst = 0;
      barrier();  // every wave is done with its MFMAs' operands and the slot's last reads
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (wm == (q >> 2)) {
          const int tm = q & 3;
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e)
              slab[((e & 3) + 8 * (e >> 2) + 4 * hsel) * G16_N + wn * 32 * NT + t * 32 + r32] = acc[tm][t][e] * S16_LO_INV;
        }
        barrier();
        const float4 b4 = *reinterpret_cast<const float4*>(bl + c4 * 4);
#pragma unroll
        for (int row = r0; row < 32; row += 8) {
          const int gr = mrow0 + q * 32 + row;
          const float4 v = *reinterpret_cast<const float4*>(slab + row * G16_N + c4 * 4);
          if (gr < M) {
            *reinterpret_cast<float4*>(Cout + (size_t)gr * N + col) =
                make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
            ++nst;
          }
        }
        barrier();
      }
      zero();
      after_epi = nst;
      ++cur;
      tpar ^= 1;
      n0 = n1;
      m0 = m1;
      if (L1 < total) L1 = next_tile(L1 + G, n1, m1);
    }
  }
}
}  // namespace

static uint16_t f2h(float x) {
  _Float16 h = (_Float16)x;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

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
  for (int Kp : {512, 768}) {
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
    const int NB = N / G16_N, NM = (M + G16_M - 1) / G16_M;
    int NG = 1;
    while (NG < 8 && NB % (NG * 2) == 0 && (size_t)(NB / NG) * G16_N * Kp * 4 > (3u << 20)) NG *= 2;
    const Order16 order{NB, NM, NG};
    const int nk = (K + G16_K - 1) / G16_K;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep)
      for (int v = 0; v < 2; ++v) {
        const int iters = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) {
          if (v == 0)
            hipLaunchKernelGGL(gemm16_persist_kernel<0>, dim3(256), dim3(512), 0, 0, dA, dW, dB, dC0, M, N, Kp, order,
                               order.blocks(), nk);
          else
            hipLaunchKernelGGL(gemm16_pipe_kernel, dim3(256), dim3(512), 0, 0, dA, dW, dB, dC1, M, N, Kp, order,
                               order.blocks(), nk);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("Kp %d %-10s %8.1f us\n", Kp, v == 0 ? "persist" : "pipe", 1000.0 * ms / iters);
      }
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
    printf("Kp %d: %zu of %zu outputs differ bitwise (pipe vs persist)\n", Kp, diff, c0.size());
    hipFree(dA);
    hipFree(dW);
    hipFree(dB);
    hipFree(dC0);
    hipFree(dC1);
  }
  return 0;
}
