// Ablation probe for the encoder input GEMM (diagnostics only, not part of the library).
// Same tiling as encoder.hip gemm_nt_kernel (128x128 tile, BK 32, 4 waves of 64x64, LDS staged,
// register double buffer); compile-time switches remove one ingredient at a time so the
// time each costs can be read off.  Results are garbage in the ablated variants.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/gemm_ablate.hip -o /tmp/gemm_ablate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32, LDK = BK + 4;

enum : int { F_NOBAR = 1, F_NOGLOB = 2, F_NOLDS = 4, F_NOEPI = 8, F_M32 = 16 };

template <int FL>
__global__ __launch_bounds__(256) void gemm(const float* __restrict__ A, const float* __restrict__ W, float* C,
                                            int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) float sm[2 * (BM + BN) * LDK];
  constexpr int ST = (BM + BN) * LDK;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int L = blockIdx.x, x = L & 7, j = L >> 3;  // NG = 2 tile order of encoder.hip
  const int nb = (x % 2) * 8 + (j % 8), mb = (j / 8) * 4 + (x / 2);
  if (mb * BM >= M) return;
  const int m0 = mb * BM, n0 = nb * BN, r = lane & 15, g = lane >> 4;
  f32x4 acc[4][4];
  f32x16 acc32[2][2];
  for (int i = 0; i < 4; ++i)
    for (int q = 0; q < 4; ++q) acc[i][q] = f32x4{0, 0, 0, 0};
  for (int i = 0; i < 2; ++i)
    for (int q = 0; q < 2; ++q)
      for (int e = 0; e < 16; ++e) acc32[i][q][e] = 0.f;
  float4 ra[4], rw[4];
  auto gload = [&](int k0) {
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, c4 = idx & 7;
      if (FL & F_NOGLOB) {
        ra[i] = make_float4(row, c4, k0, 1.f);
        rw[i] = ra[i];
      } else {
        ra[i] = *reinterpret_cast<const float4*>(A + (size_t)(m0 + row) * K + k0 + c4 * 4);
        rw[i] = *reinterpret_cast<const float4*>(W + (size_t)(n0 + row) * K + k0 + c4 * 4);
      }
    }
  };
  auto swrite = [&](int buf) {
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, c4 = idx & 7;
      *reinterpret_cast<float4*>(sm + buf * ST + row * LDK + c4 * 4) = ra[i];
      *reinterpret_cast<float4*>(sm + buf * ST + (BM + row) * LDK + c4 * 4) = rw[i];
    }
  };
  const int nk = K / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  float4 fa[4], fw[4];
  for (int i = 0; i < 4; ++i) fa[i] = fw[i] = make_float4(i, 1, 2, 3);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const float* as = sm + cur * ST;
    const float* ws = as + BM * LDK;
    if (FL & F_M32) {
      // v_mfma_f32_32x32x2_f32: lane l: A row l&31, k = 2*step + (l>>5); 16 k-steps of 2 per BK
      // k permutation: lane half h takes k = 16h + 4q + e (q = 0..3), float4 per q
      const int r32 = lane & 31, h = lane >> 5;
      for (int q = 0; q < 4; ++q) {
        float4 a[2], w[2];
        for (int tm = 0; tm < 2; ++tm)
          a[tm] = (FL & F_NOLDS) ? fa[tm] : *reinterpret_cast<const float4*>(as + (wm * 64 + tm * 32 + r32) * LDK + h * 16 + q * 4);
        for (int tn = 0; tn < 2; ++tn)
          w[tn] = (FL & F_NOLDS) ? fw[tn] : *reinterpret_cast<const float4*>(ws + (wn * 64 + tn * 32 + r32) * LDK + h * 16 + q * 4);
        for (int tm = 0; tm < 2; ++tm)
          for (int tn = 0; tn < 2; ++tn) {
            acc32[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm].x, w[tn].x, acc32[tm][tn], 0, 0, 0);
            acc32[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm].y, w[tn].y, acc32[tm][tn], 0, 0, 0);
            acc32[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm].z, w[tn].z, acc32[tm][tn], 0, 0, 0);
            acc32[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm].w, w[tn].w, acc32[tm][tn], 0, 0, 0);
          }
      }
    } else {
      for (int half = 0; half < 2; ++half) {
        float4 a[4], w[4];
        for (int tm = 0; tm < 4; ++tm)
          a[tm] = (FL & F_NOLDS) ? fa[tm] : *reinterpret_cast<const float4*>(as + (wm * 64 + tm * 16 + r) * LDK + g * 8 + half * 4);
        for (int tn = 0; tn < 4; ++tn)
          w[tn] = (FL & F_NOLDS) ? fw[tn] : *reinterpret_cast<const float4*>(ws + (wn * 64 + tn * 16 + r) * LDK + g * 8 + half * 4);
        for (int tm = 0; tm < 4; ++tm)
          for (int tn = 0; tn < 4; ++tn) {
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].x, w[tn].x, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].y, w[tn].y, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].z, w[tn].z, acc[tm][tn], 0, 0, 0);
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].w, w[tn].w, acc[tm][tn], 0, 0, 0);
          }
      }
    }
    if (kt + 1 < nk) swrite(cur ^ 1);
    if (!(FL & F_NOBAR)) __syncthreads();
  }
  if (FL & F_NOEPI) {
    float s = 0;
    for (int i = 0; i < 4; ++i)
      for (int q = 0; q < 4; ++q) s += acc[i][q][0] + acc[i][q][3];
    for (int i = 0; i < 2; ++i)
      for (int q = 0; q < 2; ++q) s += acc32[i][q][0] + acc32[i][q][15];
    if (s == 1234.5f) C[tid] = s;
    return;
  }
  if (FL & F_M32) {
    for (int tm = 0; tm < 2; ++tm)
      for (int tn = 0; tn < 2; ++tn)
        for (int v = 0; v < 16; ++v) {
          const int row = m0 + wm * 64 + tm * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
          const int col = n0 + wn * 64 + tn * 32 + (lane & 31);
          C[(size_t)row * N + col] = acc32[tm][tn][v];
        }
  } else {
    for (int tm = 0; tm < 4; ++tm)
      for (int tn = 0; tn < 4; ++tn)
        for (int e = 0; e < 4; ++e)
          C[(size_t)(m0 + wm * 64 + tm * 16 + g * 4 + e) * N + n0 + wn * 64 + tn * 16 + r] = acc[tm][tn][e];
  }
}

// LDS-DMA staging: global_load_lds_dwordx4 into lane-linear 128-B rows, source-side XOR swizzle
// chunk' = chunk ^ ((row >> 1) & 7), same XOR on the fragment reads.
template <int FL>
__global__ __launch_bounds__(256) void gemm_glds(const float* __restrict__ A, const float* __restrict__ W, float* C,
                                                 int M, int N, int K) {
  constexpr int TILE = 128 * 32;  // floats per operand tile (16 KB)
  __shared__ __attribute__((aligned(16))) float sm[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int L = blockIdx.x, x = L & 7, j = L >> 3;
  const int nb = (x % 2) * 8 + (j % 8), mb = (j / 8) * 4 + (x / 2);
  if (mb * BM >= M) return;
  const int m0 = mb * BM, n0 = nb * BN, r = lane & 15, g = lane >> 4;
  f32x4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int q = 0; q < 4; ++q) acc[i][q] = f32x4{0, 0, 0, 0};
  // wave w stages rows [32w, 32w+32) of A and of W: 4 instructions each (8 rows x 128 B)
  auto stage = [&](int buf, int k0) {
    for (int i = 0; i < 4; ++i) {
      const int row = wave * 32 + i * 8 + (lane >> 3), p = lane & 7, c = p ^ ((row >> 1) & 7);
      float* la = sm + buf * 2 * TILE + (wave * 32 + i * 8) * 32;
      float* lw = la + TILE;
      __builtin_amdgcn_global_load_lds(A + (size_t)(m0 + row) * K + k0 + c * 4, (__attribute__((address_space(3))) void*)la, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(W + (size_t)(n0 + row) * K + k0 + c * 4, (__attribute__((address_space(3))) void*)lw, 16, 0, 0);
    }
  };
  const int nk = K / BK;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const float* as = sm + cur * 2 * TILE;
    const float* ws = as + TILE;
    for (int half = 0; half < 2; ++half) {
      float4 a[4], w[4];
      const int c = g * 2 + half;  // logical 16-B chunk of k = 8g + 4 half
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 64 + tm * 16 + r;
        a[tm] = *reinterpret_cast<const float4*>(as + row * 32 + ((c ^ ((row >> 1) & 7)) << 2));
      }
      for (int tn = 0; tn < 4; ++tn) {
        const int row = wn * 64 + tn * 16 + r;
        w[tn] = *reinterpret_cast<const float4*>(ws + row * 32 + ((c ^ ((row >> 1) & 7)) << 2));
      }
      for (int tm = 0; tm < 4; ++tm)
        for (int tn = 0; tn < 4; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].x, w[tn].x, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].y, w[tn].y, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].z, w[tn].z, acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm].w, w[tn].w, acc[tm][tn], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  if (FL & F_NOEPI) {
    float s = 0;
    for (int i = 0; i < 4; ++i)
      for (int q = 0; q < 4; ++q) s += acc[i][q][0] + acc[i][q][3];
    if (s == 1234.5f) C[tid] = s;
    return;
  }
  for (int tm = 0; tm < 4; ++tm)
    for (int tn = 0; tn < 4; ++tn)
      for (int e = 0; e < 4; ++e)
        C[(size_t)(m0 + wm * 64 + tm * 16 + g * 4 + e) * N + n0 + wn * 64 + tn * 16 + r] = acc[tm][tn][e];
}

template <int FL>
double run_glds(const char* name, const float* A, const float* W, float* C, int M, int N, int K,
                std::vector<float>& h) {
  const int blocks = 8 * 8 * ((M / BM + 3) / 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(gemm_glds<FL>, dim3(blocks), dim3(256), 0, 0, A, W, C, M, N, K);
  (void)hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(gemm_glds<FL>, dim3(blocks), dim3(256), 0, 0, A, W, C, M, N, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  double err = -1;
  if (!(FL & F_NOEPI)) {
    std::vector<float> got((size_t)M * N);
    (void)hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost);
    err = 0;
    for (size_t i = 0; i < got.size(); i += 997) err = fmax(err, fabs(got[i] - h[i]));
  }
  printf("%-28s %9.1f us  %6.1f TF/s  maxerr %g\n", name, us, 2.0 * M * N * K / us / 1e6, err);
  return us;
}

template <int FL>
double run(const char* name, const float* A, const float* W, float* C, int M, int N, int K, const float* Cref,
           std::vector<float>& h) {
  const int NM = M / BM;
  const int blocks = 8 * 8 * ((NM + 3) / 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(gemm<FL>, dim3(blocks), dim3(256), 0, 0, A, W, C, M, N, K);
  (void)hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(gemm<FL>, dim3(blocks), dim3(256), 0, 0, A, W, C, M, N, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / reps;
  double err = -1;
  if (Cref) {  // correctness of the non-ablated variants against a reference run
    std::vector<float> got((size_t)M * N);
    (void)hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost);
    err = 0;
    for (size_t i = 0; i < got.size(); i += 997) err = fmax(err, fabs(got[i] - h[i]));
  }
  printf("%-28s %9.1f us  %6.1f TF/s  maxerr %g\n", name, us, 2.0 * M * N * K / us / 1e6, err);
  return us;
}

int main() {
  const int M = 68096, N = 2048, K = 512;
  std::vector<float> ha((size_t)M * K), hw((size_t)N * K);
  for (size_t i = 0; i < ha.size(); ++i) ha[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (float)((i * 40503u) % 1000) / 1000.f - 0.5f;
  float *A, *W, *C;
  (void)hipMalloc(&A, ha.size() * 4);
  (void)hipMalloc(&W, hw.size() * 4);
  (void)hipMalloc(&C, (size_t)M * N * 4);
  (void)hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(W, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> ref((size_t)M * N);
  run<0>("baseline 16x16x4", A, W, C, M, N, K, nullptr, ref);
  (void)hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost);
  run<F_M32>("mfma 32x32x2", A, W, C, M, N, K, C, ref);
  run<F_NOEPI>("no epilogue", A, W, C, M, N, K, nullptr, ref);
  run<F_NOBAR>("no barrier", A, W, C, M, N, K, nullptr, ref);
  run<F_NOGLOB>("no global loads", A, W, C, M, N, K, nullptr, ref);
  run<F_NOLDS>("no LDS reads", A, W, C, M, N, K, nullptr, ref);
  run<F_NOGLOB | F_NOLDS | F_NOBAR | F_NOEPI>("MFMA only", A, W, C, M, N, K, nullptr, ref);
  run<F_M32 | F_NOGLOB | F_NOLDS | F_NOBAR | F_NOEPI>("MFMA only 32x32x2", A, W, C, M, N, K, nullptr, ref);
  run<F_M32 | F_NOEPI>("32x32x2 no epilogue", A, W, C, M, N, K, nullptr, ref);
  run_glds<0>("glds (LDS-DMA) staging", A, W, C, M, N, K, ref);
  run_glds<F_NOEPI>("glds no epilogue", A, W, C, M, N, K, ref);
  return 0;
}
