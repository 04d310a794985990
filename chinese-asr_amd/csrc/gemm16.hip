// Encoder input projection on the f16 MFMA pipes, 256 x 256 tiles (RNN_RES.forward's
// nn.LSTM input GEMM, util.py:1258-1275; Gin = x . W_ih^T + b_ih + b_hh for both directions).
//
// Why a separate kernel from encoder.hip's 128 x 128 gemm_nt_kernel: s16x3 moves 4 B per operand
// element (hi + lo halves) but runs the products 16/3 x faster than f32 MFMA, so at 128 x 128
// the tile is bound by L2 -> LDS bytes (46 B/clk/CU needed against ~30 available,
// MI355X_MICROARCH.md "2,048 rows shared by every workgroup": 17-19 TB/s chip-wide).  A 256 x 256
// tile halves the bytes per flop (23 B/clk/CU).
//
// Register budget: 4 waves (one per SIMD, 512 registers each), each 128 x 128 = 16 tiles of
// v_mfma_f32_32x32x16_f16.  Two accumulator sets (hi.hi and cross terms) would need 512
// accumulator registers, so ONE accumulator holds the whole s16x3 sum scaled by 2^11:
//     acc = sum_k  a_hi (w_hi 2^11) + a_hi w_lo' + a_lo' w_hi        (x' = (x - x_hi) 2^11)
//     Gin = acc 2^-11 + bias
// w_hi 2^11 is formed in registers from the staged w_hi (v_pk_mul_f16 by 2048: exact while
// |w| < 32, which casr_pack_weights requires before it marks the s16 images valid).  Every
// product stays exact in f32; the cross terms share the accumulator's rounding, as in the
// exact-f32 chain.
//
// Staging: LDS-DMA (global_load_lds_dwordx4) of 256 rows x 128 B (one 32-k tile of an s16 row
// image: 32 hi | 32 lo halves) for A and W, two distinct stage buffers of 64 KB, 16-B chunk c of
// row r at c ^ ((r >> 1) & 7).  Grid: XCD-aware tile order (encoder.hip TileOrder rationale).
#include <stdlib.h>

#include <type_traits>

#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

namespace {

constexpr int G16_M = 256, G16_N = 256, G16_K = 32;  // tile rows, columns, k per stage
constexpr int G16_TILE = G16_M * G16_K;              // 4-B words per operand stage (32 KB)

struct Order16 {
  int NB, NM, NG;
  __host__ __device__ int blocks() const { return 8 * (NB / NG) * ((NM + 8 / NG - 1) / (8 / NG)); }
  __device__ bool tile(int L, int& n, int& m) const {
    const int x = L & 7, j = L >> 3, nbg = NB / NG;
    n = (x % NG) * nbg + (j % nbg);
    m = (j / nbg) * (8 / NG) + (x / NG);
    return m < NM;
  }
};

// WN: waves along N (2 -> 128 x 128 wave tiles, 4 -> 128 x 64); MH: 128-row halves of the tile
// (2: 256 x 256 with 2 WN waves; 1: 128 x 256 with WN waves, the half tiles that balance the
// persistent kernel's last round, launch_input_proj_s16_big)
template <int WN, int MH = 2>
__global__ __launch_bounds__(64 * MH * WN, WN* MH / 4) void gemm16_bias_kernel(const float* __restrict__ A16, const float* __restrict__ W16,
                                                          const float* __restrict__ bias, float* __restrict__ Cout,
                                                          int M, int N, int Kp, Order16 order) {
  constexpr int BM = 128 * MH, ATILE = BM * G16_K, NWV = MH * WN;
  __shared__ __attribute__((aligned(16))) float buf0[ATILE + G16_TILE];  // [A tile | W tile]
  __shared__ __attribute__((aligned(16))) float buf1[ATILE + G16_TILE];
  int nt, mt;
  if (!order.tile(blockIdx.x, nt, mt)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NT = 8 / WN;                 // 32-column MFMA tiles per wave
  const int wm = wave / WN, wn = wave % WN;  // wave tile: rows [128 wm, +128) x columns [32 NT wn, +32 NT)
  const int m0 = mt * BM, n0 = nt * G16_N;

  // wave tile 128 x 128 as 4 x 4 tiles of v_mfma_f32_32x32x16_f16 (16 accumulators each):
  // lane l holds A[row l&31][k = 16s + 8(l>>5) + j] and B[k][col l&31] (j = 0..7) for k-step s,
  // C/D col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5)
  f32x16 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int r32 = lane & 31, hsel = lane >> 5;

  // wave w stages A rows [RWA w, +RWA) and W rows [RWW w, +RWW): DMA instructions of 8 rows x 128 B
  constexpr int RWA = BM / NWV, RWW = G16_N / NWV;
  auto stage = [&](float* dst, int k0) {
#pragma unroll
    for (int i = 0; i < RWA / 8; ++i) {
      const int row = wave * RWA + i * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
      const int ar = min(m0 + row, M - 1);
      float* la = dst + (wave * RWA + i * 8) * G16_K;
      __builtin_amdgcn_global_load_lds(A16 + (size_t)ar * Kp + k0 + c * 4,
                                       (__attribute__((address_space(3))) void*)la, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RWW / 8; ++i) {
      const int row = wave * RWW + i * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
      const int wr = min(n0 + row, N - 1);
      float* lw = dst + ATILE + (wave * RWW + i * 8) * G16_K;
      __builtin_amdgcn_global_load_lds(W16 + (size_t)wr * Kp + k0 + c * 4,
                                       (__attribute__((address_space(3))) void*)lw, 16, 0, 0);
    }
  };
  const _Float16 two11 = (_Float16)2048.0f;
  auto compute = [&](const float* src) {
    const float* as = src;
    const float* ws = src + ATILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + hsel;  // 16-B chunk of this lane's 8 k (hi); lo is chunk 4 + ch
      f16x8 wh[NT], wl[NT], w1[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int row = wn * 32 * NT + t * 32 + r32, sw = (row >> 1) & 7;
        wh[t] = *reinterpret_cast<const f16x8*>(ws + row * G16_K + ((ch ^ sw) << 2));
        wl[t] = *reinterpret_cast<const f16x8*>(ws + row * G16_K + (((4 + ch) ^ sw) << 2));
        w1[t] = wh[t] * two11;
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 128 + tm * 32 + r32, sw = (row >> 1) & 7;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(as + row * G16_K + ((ch ^ sw) << 2));
        const f16x8 al = *reinterpret_cast<const f16x8*>(as + row * G16_K + (((4 + ch) ^ sw) << 2));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, w1[t], acc[tm][t], 0, 0, 0);
          if constexpr (kS16Cross) {
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, wl[t], acc[tm][t], 0, 0, 0);
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, wh[t], acc[tm][t], 0, 0, 0);
          }
        }
      }
    }
  };

  // Kp % 64 == 0: an even number of k tiles, so the loop body is straight-line (no exit between
  // the two halves: a branch around a compute block makes hipcc shuffle every accumulator)
  const int nk = Kp / G16_K;
  stage(buf0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    stage(buf1, (kt + 1) * G16_K);
    compute(buf0);
    __syncthreads();  // retires this wave's DMA into buf1 and everyone's reads of buf0
    if (kt + 2 < nk) stage(buf0, (kt + 2) * G16_K);
    compute(buf1);
    __syncthreads();
  }

  // epilogue: eight 32-row slabs staged through LDS (buf0), stored as whole 1 KB rows
  constexpr int LDC = G16_N + 4;
  static_assert(32 * LDC <= ATILE + G16_TILE, "slab fits one stage buffer");
  const int c4 = tid & 63, r0 = tid >> 6;  // 64 float4 per row, NWV rows per pass
  const int col = n0 + c4 * 4;
  const float4 b4 = col < N ? *reinterpret_cast<const float4*>(bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int p = 0; p < 4 * MH; ++p) {
    // slab p = rows [32p, 32p + 32) = tile tm = p & 3 of the waves with wm = p >> 2
    if (wm == (p >> 2)) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          buf0[((e & 3) + 8 * (e >> 2) + 4 * hsel) * LDC + wn * 32 * NT + t * 32 + r32] = acc[p & 3][t][e] * S16_LO_INV;
    }
    __syncthreads();
    if (col < N) {
#pragma unroll
      for (int row = r0; row < 32; row += NWV) {
        const int gr = m0 + p * 32 + row;
        if (gr >= M) break;
        const float4 v = *reinterpret_cast<const float4*>(buf0 + row * LDC + c4 * 4);
        *reinterpret_cast<float4*>(Cout + (size_t)gr * N + col) =
            make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
      }
    }
    __syncthreads();
  }
}

// ---- persistent form: one 512-thread workgroup per CU walks its tiles (the XCD-aware order
// above, tile L = blockIdx.x + i * gridDim.x, so a workgroup stays with its XCD's weight slices)
// and the stage pipeline runs on across tile boundaries:
//   * the first 32-k stage of the next tile is DMA'd during the last stage of the current one,
//     so the epilogue (slabs through the stage buffer just consumed, float4 stores to HBM)
//     overlaps that DMA, and the stores are never waited for: the stage waits count them
//     (vmcnt(G16P_EPI_STORES) retires the older DMA with the stores still in flight);
//   * the DMAs are issued from inline asm (lds_dma16) and ordered by counted s_waitcnt vmcnt +
//     raw s_barrier: no __syncthreads() (its fence drains vmcnt to 0), and hipcc inserts no wait
//     of its own for a DMA it cannot see;
//   * the bias of a tile arrives by one more DMA (1 KB, wave 0) into a slot beside the stages, so
//     the epilogue reads it from LDS (a global load there would make hipcc wait vmcnt(0)).
// Arithmetic (fragment order, MFMA order, accumulator scaling, bias add) is compute() of
// gemm16_bias_kernel<4>: both kernels give the same bits.
constexpr int G16P_STAGE = 2 * G16_TILE;                       // floats per stage: [A | W]
constexpr int G16P_LDS = 2 * G16P_STAGE + 2 * G16_N;           // two stages + two bias slots
constexpr int G16P_EPI_STORES = 32;                             // float4 stores per thread per tile
static_assert(G16P_LDS * 4 <= 160 * 1024, "stages + bias slots fit the LDS");

template <int I, int N, class F>
CASR_DEV void static_for16(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for16<I + 1, N>(f);
  }
}

template <int VM>
CASR_DEV void g16_vm_wait() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
}

// DIAG (tools/probes/gemm16_probe.hip only; results then wrong for 1, 2, 4): 1 = no k-loop DMA
// (stale LDS), 2 = no MFMA, 4 = no epilogue stores; 8 = iglp_opt(1) in the k loop, 16 = s_setprio 1
// for waves 4-7 (both measured within noise).  Round 2 also measured the next stage's DMA issued two
// instructions at a time between the first k-step's MFMA groups (faster in the probe, equal or
// slower inside the encoder); removed in round 3.
template <int DIAG = 0>
__global__ __launch_bounds__(512, 2) void gemm16_persist_kernel(const float* __restrict__ A16,
                                                             const float* __restrict__ W16,
                                                             const float* __restrict__ bias,
                                                             float* __restrict__ Cout, int M, int N, int Kp,
                                                             Order16 order, int total, int nk) {
  __shared__ __attribute__((aligned(16))) float lds[G16P_LDS];
  constexpr int WN = 4, NT = 2, RW = 32;  // 8 waves = 2 (M) x 4 (N) of 128 x 64; 32 staged rows per wave
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r32 = lane & 31, hsel = lane >> 5;
  const int G = gridDim.x;  // nk: 32-k stages to run (of the Kp / 32 in a row image)
  float* const bias_lds = lds + 2 * G16P_STAGE;

  // tiles of this workgroup: L = blockIdx.x + i G, skipping the order's empty slots
  auto next_tile = [&](int L, int& n, int& m) {
    while (L < total && !order.tile(L, n, m)) L += G;
    return L;
  };
  // DMA of stage (tile (n, m), k tile kt) into stage buffer `sb` (+ the tile's bias at kt = 0)
  // DMA slot q of a stage: rows i = q / 2 of this wave's share, A (q even) or W (q odd); the last
  // slot also brings the tile's bias at kt = 0
  constexpr int NQ = 2 * (RW / 8);
  auto stage_slot = [&](int sb, int n, int m, int kt, int tpar, auto Q) {
    constexpr int q = decltype(Q)::value, i = q >> 1;
    float* dst = lds + sb * G16P_STAGE;
    const int m0 = m * G16_M, n0 = n * G16_N, k0 = kt * G16_K;
    const int row = wave * RW + i * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
    float* la = dst + (wave * RW + i * 8) * G16_K;
    if constexpr ((q & 1) == 0) {
      lds_dma16(A16 + (size_t)min(m0 + row, M - 1) * Kp + k0 + c * 4, la);
    } else {
      lds_dma16(W16 + (size_t)min(n0 + row, N - 1) * Kp + k0 + c * 4, la + G16_TILE);
    }
    if constexpr (q == NQ - 1) {
      if (kt == 0 && wave == 0) lds_dma16(bias + min(n0 + lane * 4, N - 4), bias_lds + tpar * G16_N);
    }
  };
  auto stage = [&](int sb, int n, int m, int kt, int tpar) {
    static_for16<0, NQ>([&](auto Q) { stage_slot(sb, n, m, kt, tpar, Q); });
  };

  f32x16 acc[4][NT];
  const _Float16 two11 = (_Float16)2048.0f;
  if ((DIAG & 16) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  auto compute = [&](const float* src) {
    const float* as = src;
    const float* ws = src + G16_TILE;
    if constexpr ((DIAG & 8) != 0) __builtin_amdgcn_iglp_opt(1);
    static_for16<0, 2>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      const int ch = 2 * ks + hsel;
      f16x8 wh[NT], wl[NT], w1[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int row = wn * 32 * NT + t * 32 + r32, sw = (row >> 1) & 7;
        wh[t] = *reinterpret_cast<const f16x8*>(ws + row * G16_K + ((ch ^ sw) << 2));
        wl[t] = *reinterpret_cast<const f16x8*>(ws + row * G16_K + (((4 + ch) ^ sw) << 2));
        w1[t] = wh[t] * two11;
      }
      static_for16<0, 4>([&](auto TM) {
        constexpr int tm = decltype(TM)::value;
        const int row = wm * 128 + tm * 32 + r32, sw = (row >> 1) & 7;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(as + row * G16_K + ((ch ^ sw) << 2));
        const f16x8 al = *reinterpret_cast<const f16x8*>(as + row * G16_K + (((4 + ch) ^ sw) << 2));
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, w1[t], acc[tm][t], 0, 0, 0);
          if constexpr (kS16Cross) {
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, wl[t], acc[tm][t], 0, 0, 0);
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, wh[t], acc[tm][t], 0, 0, 0);
          }
        }
      });
    });
  };
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  int n, m;
  int L = next_tile(blockIdx.x, n, m);
  if (L >= total) return;
  int sb = 0, tpar = 0;
  stage(0, n, m, 0, 0);
  // the previous tile's epilogue stores issued after the DMA now waited for: all G16P_EPI_STORES
  // of them (a full tile; the row test is wave-uniform), or fewer (then wait for everything)
  int after_epi = 0;
  while (true) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    int n2 = n, m2 = m;
    const int L2 = next_tile(L + G, n2, m2);
    for (int kt = 0; kt < nk; ++kt) {
      if (after_epi == G16P_EPI_STORES) g16_vm_wait<G16P_EPI_STORES>();
      else g16_vm_wait<0>();
      after_epi = 0;
      barrier();  // everyone's DMA of this stage landed; everyone is done reading the other buffer
      auto issue = [&](auto Q) {
        if (DIAG & 1) return;
        if (kt + 1 < nk) stage_slot(sb ^ 1, n, m, kt + 1, tpar, Q);
        else if (L2 < total) stage_slot(sb ^ 1, n2, m2, 0, tpar ^ 1, Q);
      };
      static_for16<0, NQ>(issue);
      if (!(DIAG & 2)) compute(lds + sb * G16P_STAGE);
      sb ^= 1;
    }
    // epilogue through the stage buffer just consumed (sb ^ 1 now): four rounds of two 32-row
    // slabs (64 rows x 256 columns = the whole buffer; rows 1 KB apart and the two 32-lane halves
    // of a ds_write_b32 are separate LDS cycles, so no padding), float4 stores + bias
    float* slab = lds + (sb ^ 1) * G16P_STAGE;
    const float* bl = bias_lds + tpar * G16_N;
    const int c4 = tid & 63, r0 = tid >> 6;
    const int m0 = m * G16_M, col = n * G16_N + c4 * 4;
    int nst = 0;
    barrier();  // every wave is done reading the last stage
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (wm == (p >> 1)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tm = 2 * (p & 1) + h;
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e)
              slab[(h * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel) * G16_N + wn * 32 * NT + t * 32 + r32] =
                  acc[tm][t][e] * S16_LO_INV;
        }
      }
      barrier();
      const float4 b4 = *reinterpret_cast<const float4*>(bl + c4 * 4);
#pragma unroll
      for (int row = r0; row < 64; row += 8) {
        const int gr = m0 + p * 64 + row;
        const float4 v = *reinterpret_cast<const float4*>(slab + row * G16_N + c4 * 4);
        if ((DIAG & 4) && v.x == 12345.f) Cout[0] = b4.x;
        if (!(DIAG & 4) && gr < M) {  // wave-uniform (row = wave + 8 j); N % 256 == 0 (host check)
          *reinterpret_cast<float4*>(Cout + (size_t)gr * N + col) =
              make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
          ++nst;
        }
      }
      barrier();
    }
    if (L2 >= total) break;
    L = L2;
    n = n2;
    m = m2;
    tpar ^= 1;
    after_epi = nst;
  }
}

// ---- ping-pong form (round 5, CASR_OPT_GEMM16_PERSIST = 2): the persistent kernel's compute loop
// ran at ~2.3 us per 32-deep stage against ~1.5 us of MFMA (every wave of the CU
// read its fragments after the same barrier, then multiplied, so the SIMD's MFMA pipe idled through
// the LDS round trips).  Here the two wave groups (wm = 0: waves 0-3, wm = 1: waves 4-7; one wave of
// each per SIMD) run one barrier apart: each 16-deep stage is a LOAD section (the stage's 12
// fragment reads, the DMA of the stage three ahead, lgkmcnt(0)), a barrier, an MFMA section (24
// MFMAs), a barrier; with group 1 one barrier behind, one group's MFMA section always overlaps the
// other group's LOAD section on the same SIMD (cdna_hip_programming.md §5, the 256² 8-phase
// template's staggered wave groups).
//   * Stages are 16 k deep: [A 256 rows | W 256 rows] x 64 B (16 hi | 16 lo halves of the s16 row
//     image), a ring of four (128 KB), three stages in flight.  Chunk c (16 B) of row r sits at
//     c ^ ((r >> 2) & 3): conflict-free ds_read_b128 of 16 consecutive rows.
//   * Hazards, by barrier count (E_i = the i-th barrier release of a tile; group 0 enters its LOAD_j
//     after E_{2j-1}, group 1 after E_{2j}):
//       RAW: every wave waits (counted vmcnt) for its DMA of stage j + 1 before E_{2j+1}: group 0 after
//       MFMA_j, group 1 at the end of LOAD_j; group 0 reads stage j + 1 after E_{2j+1}.
//       WAR: fragment reads are retired (lgkmcnt(0)) before each LOAD's closing barrier, so the
//       stage j - 1 buffer is free after E_{2j-1}; the DMA of stage j + 3 goes into it in LOAD_j.
//   * Epilogue per tile: the groups realign (group 0's extra barrier), each wave writes its 128 x 64
//     accumulator slab through a private 4 KB region of the buffer of the tile's last stage (16 rows
//     at a time, no block barrier), adds the bias (DMA'd with the tile's first stage) and stores float4
//     rows with buffer stores, whose out-of-range rows the hardware drops (so every wave always
//     issues 32 stores and the vmcnt counts stay exact); one barrier, then the next tile's region.
// Arithmetic: per accumulator the same MFMAs in the same k order as gemm16_persist_kernel (16-deep
// stage j = k-step j & 1 of 32-deep tile j >> 1), so the outputs are bitwise equal.
// (round 5) the input projection's Gin rows (557 MB per layer at B = 256, each read once by the
// recurrence) go out with the non-temporal hint, so they do not displace what the caches hold for
// the recurrence and the next GEMM (three interleaved rounds, profiles/r05/gin_nt/: greedy batch
// 6.69-6.72 -> 6.59-6.60 ms, beam 10.65-10.75 -> 10.50-10.57 ms, the recurrence class the one that
// moves); 0 restores plain stores (diagnostic builds)
#ifndef CASR_GIN_NT
#define CASR_GIN_NT 1
#endif
constexpr int PP_ROWF = 16;                  // floats per staged row (64 B)
constexpr int PP_OP = G16_M * PP_ROWF;       // floats per operand and stage (16 KB)
constexpr int PP_STAGE = 2 * PP_OP;          // [A | W]
constexpr int PP_NBUF = 4;
constexpr int PP_LDS = PP_NBUF * PP_STAGE + 2 * G16_N;  // ring + two bias slots
constexpr int PP_EPI_STORES = 32;            // buffer stores per wave and tile
static_assert(PP_LDS * 4 <= 160 * 1024, "ring + bias slots fit the LDS");
static_assert(8 * 16 * 64 <= PP_STAGE, "eight private 16 x 64 epilogue slabs fit one stage buffer");

// s_waitcnt vmcnt(N) for the largest N of {40, 9, 8, 4, 0} not above `younger` (the VMEM operations
// this wave issued after the ones to retire): a smaller N only waits for more
CASR_DEV void pp_vm_wait(int younger) {
  if (younger >= 40) g16_vm_wait<40>();
  else if (younger >= 9) g16_vm_wait<9>();
  else if (younger >= 8) g16_vm_wait<8>();
  else if (younger >= 4) g16_vm_wait<4>();
  else g16_vm_wait<0>();
}

// DIAG (tools/probes/gemm16_pp_probe.hip only; results then wrong): 1 = no k-loop DMA, 2 = no MFMA,
// 4 = no epilogue stores, 8 = DMA from 1 KB contiguous sources (the same bytes in whole lines),
// 16 = s_memtime stamps of workgroup 0's second tile (g_pp_trace: results unchanged), 32 = no
// w_hi 2^11 multiply (the VALU of a pre-scaled W image).  PRIO: 0 no s_setprio, 1 prio 1 around each
// MFMA section, 2 prio 1 for the later group throughout
__device__ unsigned long long g_pp_trace[8][64][4];
CASR_DEV unsigned long long pp_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
// KM (tools/probes only so far): A and W images 16-k-block major, [Kp / 16][rows][16 hi | 16 lo]
// halves, so a stage of 16 rows is 1 KB contiguous (whole 128-B lines) instead of 16 half lines;
// Mimg = the A image's row count
template <int DIAG = 0, int PRIO = 1, int SG = 0, int AGPR = 0, bool KM = false>
__global__ __launch_bounds__(512, 2) void gemm16_pp_kernel(const float* __restrict__ A16, const float* __restrict__ W16,
                                                           const float* __restrict__ bias, float* __restrict__ Cout,
                                                           int M, int N, int Kp, Order16 order, int total, int nk,
                                                           int Mimg = 0) {
  __shared__ __attribute__((aligned(16))) float lds[PP_LDS];
  // AGPR: an AGPR clobber keeps the accumulation registers available, so hipcc picks the MFMA form
  // with the accumulators in AGPRs (C / D traffic off the VGPR file the partner's LDS returns use)
  if constexpr (AGPR != 0) asm volatile("; accumulators in AGPRs" ::: "a0");
  constexpr int NT = 2;  // 32-column MFMA tiles per wave (wave tile 128 x 64)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // the wave's 128-row half and 64-column quarter
  // stagger group (SG: diagnostic alternatives of which waves run one barrier behind)
  const int grp = SG == 0 ? wave >> 2 : SG == 1 ? wave & 1 : (wave >> 1) & 1;
  const int r32 = lane & 31, hsel = lane >> 5;
  const int G = gridDim.x;
  float* const bias_lds = lds + PP_NBUF * PP_STAGE;

  auto next_tile = [&](int L, int& n, int& m) {
    while (L < total && !order.tile(L, n, m)) L += G;
    return L;
  };
  // DMA of 16-deep stage s of tile (n, m) into ring buffer b: this wave's 32 A rows and 32 W rows
  // (two 16-row instructions each), plus, with the tile's first stage, the tile's bias (every wave
  // copies the same 1 KB into the slot, so every wave issues the same count).  Issued with a scalar
  // base (the operand's tile rows + the stage's k offset) and per-lane 32-bit row offsets computed
  // once per tile, so a stage's DMA costs no VALU work beside the partner's MFMAs
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  uint32_t vw[2];
  int coff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
    coff[i] = KM ? 4 * c : (c >> 1) * 16 + (c & 1) * 4;
    vw[i] = (uint32_t)(row * (KM ? 16 : Kp) + coff[i]) * 4u;  // N % 256 == 0 (host check): no clamp
  }
  auto a_offsets = [&](int m, uint32_t (&va)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wave * 32 + i * 16 + (lane >> 2);
      va[i] = (uint32_t)(min(row, M - 1 - m * G16_M) * (KM ? 16 : Kp) + coff[i]) * 4u;
    }
  };
  auto stage_dma = [&](int b, int n, int m, int s, int tpar, const uint32_t (&va)[2]) {
    const int kb = (s >> 1) * 32 + (s & 1) * 8;  // float offset of this stage's hi piece in the row image
    const float* sa = KM ? A16 + ((size_t)s * Mimg + (size_t)m * G16_M) * 16 : A16 + (size_t)m * G16_M * Kp + kb;
    const float* sw = KM ? W16 + ((size_t)s * N + (size_t)n * G16_N) * 16 : W16 + (size_t)n * G16_N * Kp + kb;
    const uint32_t l0 = lds_u32 + (uint32_t)(b * PP_STAGE + wave * 32 * PP_ROWF) * 4u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr ((DIAG & 8) != 0) {  // diagnostic: 1 KB contiguous sources (wrong data, same bytes)
        lds_dma16_s((uint32_t)(min(wave * 32 + i * 16, M - 16 - m * G16_M) * Kp * 4 + lane * 16), A16 + (size_t)m * G16_M * Kp + (s & 15) * 16,
                    l0 + i * 16 * PP_ROWF * 4u);
        lds_dma16_s((uint32_t)((wave * 32 + i * 16) * Kp * 4 + lane * 16), W16 + (size_t)n * G16_N * Kp + (s & 15) * 16,
                    l0 + (PP_OP + i * 16 * PP_ROWF) * 4u);
      } else {
        lds_dma16_s(va[i], sa, l0 + i * 16 * PP_ROWF * 4u);
        lds_dma16_s(vw[i], sw, l0 + (PP_OP + i * 16 * PP_ROWF) * 4u);
      }
    }
    if (s == 0)
      lds_dma16_s((uint32_t)min(lane * 16, (N - n * G16_N - 4) * 4), bias + n * G16_N,
                  lds_u32 + (uint32_t)(PP_NBUF * PP_STAGE + tpar * G16_N) * 4u);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  int n, m;
  int L = next_tile(blockIdx.x, n, m);
  if (L >= total) return;
  int n2 = n, m2 = m;
  int L2 = next_tile(L + G, n2, m2);
  int gb = 0, tpar = 0;  // ring buffer of the tile's stage 0; the tile's bias slot
  uint32_t va[2], va2[2];  // A row offsets of this tile and of the next
  a_offsets(m, va);
  a_offsets(m2, va2);
  if (PRIO == 2 && grp == 1) __builtin_amdgcn_s_setprio(1);  // static priority for the later group
  // prologue: stages 0..2 of the first tile
  for (int s = 0; s < 3 && s < nk; ++s) stage_dma(s, n, m, s, 0, va);
  pp_vm_wait(nk >= 3 ? 8 : 0);  // stage 0 (and its bias) landed: younger = stages 1 and 2
  barrier();
  bool after_epi = false;
  int tiles_done = 0;
  const _Float16 two11 = (_Float16)2048.0f;
  f32x16 acc[4][NT];
  while (true) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][t][e] = 0.f;
    // stage s of the current tile (s >= nk: of the next one) exists / carries a bias DMA
    auto ex = [&](int s) { return s < nk || L2 < total; };
    auto ops = [&](int s) { return ex(s) ? 4 + (s == nk ? 1 : 0) : 0; };
    if (grp == 1) barrier();  // the stagger: group 1 runs one barrier behind group 0
    const bool trace = (DIAG & 16) && blockIdx.x == 0 && tiles_done == 1 && lane == 0;
    for (int j = 0; j < nk; ++j) {
      const float* buf = lds + ((gb + j) & 3) * PP_STAGE;
      if (trace && j < 64) g_pp_trace[wave][j][0] = pp_stamp();
      // ---- LOAD_j: fragments of stage j, DMA of stage j + 3
      f16x8 wh[NT], wl[NT], ah[4], al[4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int row = wn * 64 + t * 32 + r32, sw = (row >> 2) & 3;
        wh[t] = *reinterpret_cast<const f16x8*>(buf + PP_OP + row * PP_ROWF + ((hsel ^ sw) << 2));
        wl[t] = *reinterpret_cast<const f16x8*>(buf + PP_OP + row * PP_ROWF + (((2 + hsel) ^ sw) << 2));
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 128 + tm * 32 + r32, sw = (row >> 2) & 3;
        ah[tm] = *reinterpret_cast<const f16x8*>(buf + row * PP_ROWF + ((hsel ^ sw) << 2));
        al[tm] = *reinterpret_cast<const f16x8*>(buf + row * PP_ROWF + (((2 + hsel) ^ sw) << 2));
      }
      const int s3 = j + 3;
      if (!(DIAG & 1)) {
        if (s3 < nk) stage_dma((gb + s3) & 3, n, m, s3, tpar, va);
        else if (L2 < total) stage_dma((gb + s3) & 3, n2, m2, s3 - nk, tpar ^ 1, va2);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      f16x8 w1[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) w1[t] = (DIAG & 32) ? wh[t] : wh[t] * two11;
      // VMEM operations issued after this wave's DMA of stage j + 1: stages j + 2, j + 3 and, while
      // stages 1 and 2 of a tile wait, the previous tile's 32 epilogue stores
      const int younger = (DIAG & 1) ? 0 : ops(j + 2) + ops(j + 3) + (after_epi && j < 2 ? PP_EPI_STORES : 0);
      if (grp == 1 && j + 1 < nk) pp_vm_wait(younger);
      barrier();
      if (trace && j < 64) g_pp_trace[wave][j][1] = pp_stamp();
      // ---- MFMA_j
      if (PRIO == 1) __builtin_amdgcn_s_setprio(1);
      if (!(DIAG & 2)) {
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], w1[t], acc[tm][t], 0, 0, 0);
            if constexpr (kS16Cross) {
              acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], wl[t], acc[tm][t], 0, 0, 0);
              acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], wh[t], acc[tm][t], 0, 0, 0);
            }
          }
      } else {
        if (ah[0][0] == (_Float16)1234.f && wh[0][0] == (_Float16)4321.f) acc[0][0][0] += 1.f;
      }
      if (PRIO == 1) __builtin_amdgcn_s_setprio(0);
      if (trace && j < 64) g_pp_trace[wave][j][2] = pp_stamp();
      if (grp == 0 && j + 1 < nk) pp_vm_wait(younger);
      barrier();
      if (trace && j < 64) g_pp_trace[wave][j][3] = pp_stamp();
    }
    if (grp == 0) barrier();  // realign the groups: every wave has passed every read of this tile
    // ---- epilogue: per wave, 8 rounds of 16 rows x 64 columns through a private 4 KB slab
    {
      float* slab = lds + ((gb + nk - 1) & 3) * PP_STAGE + wave * 16 * 64;
      const int c4 = lane & 15, rq = lane >> 4;
      const float4 b4 = *reinterpret_cast<const float4*>(bias_lds + tpar * G16_N + wn * 64 + c4 * 4);
      const int m0 = m * G16_M;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          Cout + (size_t)m0 * N, 0, (int)((size_t)min(G16_M, M - m0) * N * 4), 0x00020000);
      const int cbase = n * G16_N + wn * 64 + c4 * 4;
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int e = 8 * hh; e < 8 * hh + 8; ++e)
              slab[((e & 3) + 8 * ((e >> 2) & 1) + 4 * hsel) * 64 + t * 32 + r32] = acc[tm][t][e] * S16_LO_INV;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = rq + 4 * i;
            const float4 v = *reinterpret_cast<const float4*>(slab + row * 64 + c4 * 4);
            const int lr = wm * 128 + tm * 32 + 16 * hh + row;  // row within the tile
            const float4 o = make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
            if (!(DIAG & 4))
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, (lr * N + cbase) * 4, 0,
                                                     CASR_GIN_NT ? 2 : 0);
            else if (v.x == 12345.f)
              Cout[0] = o.x;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (L2 >= total) break;
    // the next tile's stage 0 (+ bias) landed: younger = its stages 1, 2 and the 32 stores
    pp_vm_wait((DIAG & 1) ? 0 : ops(nk + 1) + ops(nk + 2) + ((DIAG & 4) ? 0 : PP_EPI_STORES));
    barrier();  // ... visible to every wave; every wave is done with its epilogue slab
    gb = (gb + nk) & 3;
    L = L2;
    n = n2;
    m = m2;
    tpar ^= 1;
    after_epi = !(DIAG & 4);
    ++tiles_done;
    L2 = next_tile(L + G, n2, m2);
    va[0] = va2[0];
    va[1] = va2[1];
    a_offsets(m2, va2);
  }
}


// ---- lean ping-pong form (round 6, CASR_OPT_GEMM16_LEAN = 1, 16-k-block-major images, nk >= 8).
// gemm16_pp_kernel<…, KM = true> with the LOAD sections' scalar work cut; the same fragments, MFMAs,
// DMA bytes, ring slots and barriers in the same order, so the outputs are bitwise equal.  The round-6
// PMC passes (profiles/r06/gemm16_diag/) put the stage interval in the LOAD sections, not the LDS
// array (19 % busy, no bank conflicts, LDS-issue stalls 4 % of wave cycles): each wave issued ~65
// scalar instructions per 16-deep stage (SQ_INSTS_SALU, 3.2 per MFMA) -- 64-bit stage addresses
// rebuilt with s_mul, the runtime vmcnt ladder of pp_vm_wait (compares and branches, twice per stage)
// and the count it selects.  Here:
//   * the DMA sources are running pointers (stage j + 3 of the tile, then the next tile's stages),
//     advanced by one 32-bit byte stride per stage;
//   * the stages whose younger VMEM count is fixed (2 <= j < nk - 3: the 8 DMA instructions of
//     stages j + 2 and j + 3, no bias, no epilogue stores) wait with a constant vmcnt(8);
//   * the wave index goes through readfirstlane, so the group branches are scalar.
CASR_DEV void lds_dma16_u(uint32_t voff, const float* sbase, uint32_t lds_byte) {
  // lds_dma16_s with the base made visibly uniform: the running pointers are carried through a lambda,
  // where hipcc's divergence analysis loses them (they are uniform: tile indices and strides)
  const uint64_t u = (uint64_t)(uintptr_t)sbase;
  const float* sb = (const float*)(uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(u >> 32)) << 32) |
                                              (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)u));
  lds_dma16_s(voff, sb, lds_byte);
}

__global__ __launch_bounds__(512, 2) void gemm16_pp_lean_kernel(const float* __restrict__ A16, const float* __restrict__ W16,
                                                              const float* __restrict__ bias, float* __restrict__ Cout,
                                                              int M, int N, Order16 order, int total, int nk, int Mimg) {
  __shared__ __attribute__((aligned(16))) float lds[PP_LDS];
  constexpr int NT = 2;  // 32-column MFMA tiles per wave (wave tile 128 x 64)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3, grp = wave >> 2;
  const int r32 = lane & 31, hsel = lane >> 5;
  const int G = gridDim.x;
  float* const bias_lds = lds + PP_NBUF * PP_STAGE;
  auto next_tile = [&](int L, int& n, int& m) {
    while (L < total && !order.tile(L, n, m)) L += G;
    return L;
  };
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  uint32_t vw[2];
  int coff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
    coff[i] = 4 * c;
    vw[i] = (uint32_t)(row * 16 + coff[i]) * 4u;
  }
  auto a_offsets = [&](int m, uint32_t (&va)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wave * 32 + i * 16 + (lane >> 2);
      va[i] = (uint32_t)(min(row, M - 1 - m * G16_M) * 16 + coff[i]) * 4u;
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const uint32_t a_stb = (uint32_t)Mimg * 64u, w_stb = (uint32_t)N * 64u;  // bytes per 16-k block
  auto adv = [](const float*& p, uint32_t b) { p = (const float*)((const char*)p + b); };
  // one stage's DMA into ring buffer b from (pa, pw): this wave's 32 A rows and 32 W rows, plus the
  // tile's bias with its stage 0 (every wave copies the same 1 KB into the slot)
  auto dma = [&](int b, const float* sa, const float* sw, const uint32_t (&va)[2], bool with_bias, int nb, int tp) {
    const uint32_t l0 = lds_u32 + (uint32_t)(b * PP_STAGE + wave * 32 * PP_ROWF) * 4u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      lds_dma16_u(va[i], sa, l0 + i * 16 * PP_ROWF * 4u);
      lds_dma16_u(vw[i], sw, l0 + (PP_OP + i * 16 * PP_ROWF) * 4u);
    }
    if (with_bias)
      lds_dma16_u((uint32_t)min(lane * 16, (N - nb * G16_N - 4) * 4), bias + nb * G16_N,
                  lds_u32 + (uint32_t)(PP_NBUF * PP_STAGE + tp * G16_N) * 4u);
  };

  int n, m;
  int L = next_tile(blockIdx.x, n, m);
  if (L >= total) return;
  int n2 = n, m2 = m;
  int L2 = next_tile(L + G, n2, m2);
  int gb = 0, tpar = 0;
  uint32_t va[2], va2[2];
  a_offsets(m, va);
  a_offsets(m2, va2);
  const float* pa = A16 + (size_t)m * G16_M * 16;  // the next stage to DMA
  const float* pw = W16 + (size_t)n * G16_N * 16;
  for (int s = 0; s < 3; ++s) {  // prologue: stages 0..2 of the first tile (nk >= 8)
    dma(s, pa, pw, va, s == 0, n, 0);
    adv(pa, a_stb);
    adv(pw, w_stb);
  }
  pp_vm_wait(8);  // stage 0 (and its bias) landed: younger = stages 1 and 2
  barrier();
  bool after_epi = false;
  const _Float16 two11 = (_Float16)2048.0f;
  f32x16 acc[4][NT];
  while (true) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][t][e] = 0.f;
    auto ex = [&](int s) { return s < nk || L2 < total; };
    auto ops = [&](int s) { return ex(s) ? 4 + (s == nk ? 1 : 0) : 0; };
    if (grp == 1) barrier();  // the stagger: group 1 runs one barrier behind group 0
    auto stage = [&](int j, auto FIXED) {
      constexpr int fixed = decltype(FIXED)::value;
      const float* buf = lds + ((gb + j) & 3) * PP_STAGE;
      // ---- LOAD_j: fragments of stage j, DMA of stage j + 3
      f16x8 wh[NT], wl[NT], ah[4], al[4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int row = wn * 64 + t * 32 + r32, sw = (row >> 2) & 3;
        wh[t] = *reinterpret_cast<const f16x8*>(buf + PP_OP + row * PP_ROWF + ((hsel ^ sw) << 2));
        wl[t] = *reinterpret_cast<const f16x8*>(buf + PP_OP + row * PP_ROWF + (((2 + hsel) ^ sw) << 2));
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 128 + tm * 32 + r32, sw = (row >> 2) & 3;
        ah[tm] = *reinterpret_cast<const f16x8*>(buf + row * PP_ROWF + ((hsel ^ sw) << 2));
        al[tm] = *reinterpret_cast<const f16x8*>(buf + row * PP_ROWF + (((2 + hsel) ^ sw) << 2));
      }
      const int s3 = j + 3;
      if (fixed >= 0 || ex(s3)) {
        if (fixed < 0 && s3 == nk) {  // the next tile's stage 0 (and its bias)
          pa = A16 + (size_t)m2 * G16_M * 16;
          pw = W16 + (size_t)n2 * G16_N * 16;
        }
        const bool nxt = fixed < 0 && s3 >= nk;
        dma((gb + s3) & 3, pa, pw, nxt ? va2 : va, fixed < 0 && s3 == nk, n2, tpar ^ 1);
        adv(pa, a_stb);
        adv(pw, w_stb);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      f16x8 w1[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) w1[t] = wh[t] * two11;
      // VMEM operations issued after this wave's DMA of stage j + 1: stages j + 2, j + 3 and, while
      // stages 1 and 2 of a tile wait, the previous tile's 32 epilogue stores
      auto vwait = [&] {
        if constexpr (fixed >= 0) g16_vm_wait<fixed>();
        else pp_vm_wait(ops(j + 2) + ops(j + 3) + (after_epi && j < 2 ? PP_EPI_STORES : 0));
      };
      if (grp == 1 && j + 1 < nk) vwait();
      barrier();
      // ---- MFMA_j
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], w1[t], acc[tm][t], 0, 0, 0);
          if constexpr (kS16Cross) {
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], wl[t], acc[tm][t], 0, 0, 0);
            acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], wh[t], acc[tm][t], 0, 0, 0);
          }
        }
      __builtin_amdgcn_s_setprio(0);
      if (grp == 0 && j + 1 < nk) vwait();
      barrier();
    };
    using Dyn = std::integral_constant<int, -1>;
    for (int j = 0; j < 2; ++j) stage(j, Dyn{});
    for (int j = 2; j < nk - 3; ++j) stage(j, std::integral_constant<int, 8>{});
    for (int j = nk - 3; j < nk; ++j) stage(j, Dyn{});
    if (grp == 0) barrier();  // realign the groups: every wave has passed every read of this tile
    // ---- epilogue (gemm16_pp_kernel's): per wave, 8 rounds of 16 rows x 64 columns through a
    // private 4 KB slab
    {
      float* slab = lds + ((gb + nk - 1) & 3) * PP_STAGE + wave * 16 * 64;
      const int c4 = lane & 15, rq = lane >> 4;
      const float4 b4 = *reinterpret_cast<const float4*>(bias_lds + tpar * G16_N + wn * 64 + c4 * 4);
      const int m0 = m * G16_M;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          Cout + (size_t)m0 * N, 0, (int)((size_t)min(G16_M, M - m0) * N * 4), 0x00020000);
      const int cbase = n * G16_N + wn * 64 + c4 * 4;
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int e = 8 * hh; e < 8 * hh + 8; ++e)
              slab[((e & 3) + 8 * ((e >> 2) & 1) + 4 * hsel) * 64 + t * 32 + r32] = acc[tm][t][e] * S16_LO_INV;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = rq + 4 * i;
            const float4 v = *reinterpret_cast<const float4*>(slab + row * 64 + c4 * 4);
            const int lr = wm * 128 + tm * 32 + 16 * hh + row;  // row within the tile
            const float4 o = make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, (lr * N + cbase) * 4, 0,
                                                   CASR_GIN_NT ? 2 : 0);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (L2 >= total) break;
    // the next tile's stage 0 (+ bias) landed: younger = its stages 1, 2 and the 32 stores
    pp_vm_wait(ops(nk + 1) + ops(nk + 2) + PP_EPI_STORES);
    barrier();  // ... visible to every wave; every wave is done with its epilogue slab
    gb = (gb + nk) & 3;
    L = L2;
    n = n2;
    m = m2;
    tpar ^= 1;
    after_epi = true;
    L2 = next_tile(L + G, n2, m2);
    va[0] = va2[0];
    va[1] = va2[1];
    a_offsets(m2, va2);
  }
}


// ---- balanced tail (round 5, CASR_OPT_GEMM16_TAIL = 2, default): the rows after the persistent
// kernel's whole rounds as (32 RT)-row x 128-column tiles, RT picked so that they fill the CUs in one
// round (B = 256: 2,560 rows = 16 row blocks of 160 rows x 16 column blocks = 256 tiles; TAIL = 1 ran
// them as 160 half tiles of 128 x 256 on a two-buffer ring drained by __syncthreads, 36 us).  Four
// waves, wave w: columns 32 w .. 32 w + 31 of the tile over its RT row tiles of 32; a ring of four
// 32-deep stages [A 32 RT rows | W 128 rows] x 128 B (three in flight), LDS-DMA from inline asm with
// counted vmcnt waits and a raw s_barrier per stage.  The MFMAs per accumulator are compute() of
// gemm16_bias_kernel (same fragments, order and 2^11 scaling), and the epilogue its slab form: the
// same bits.
// KM: A (rows r0 .. r0 + M - 1 of an Mimg-row image) and W 16-k-block major, and a stage in LDS is
// [16-k block 0 | block 1] x [A rows | W rows] x 64 B (the ping-pong kernel's rows: chunk c of a row at
// c ^ ((row >> 2) & 3)), so each DMA instruction reads 16 rows of one block, 1 KB contiguous; else
// row images (A16 at row r0 already) and [rows] x 128 B stages
template <int RT, bool KM>
__global__ __launch_bounds__(256, 1) void gemm16_tail_kernel(const float* __restrict__ A16, const float* __restrict__ W16,
                                                             const float* __restrict__ bias, float* __restrict__ Cout,
                                                             int M, int N, int Kp, int r0, int Mimg) {
  constexpr int BM = 32 * RT, BN = 128, ROWS = BM + BN, STF = ROWS * G16_K;  // floats per stage
  constexpr int NBUF = 4, NI = ROWS / 8, PW = (NI + 3) / 4;  // DMA instructions per stage / per wave
  static_assert(NBUF * STF * 4 <= 160 * 1024 && (NBUF - 2) * PW < 64, "ring fits the LDS; vmcnt range");
  __shared__ __attribute__((aligned(16))) float ring[NBUF * STF];
  const int ncb = N / BN, mt = blockIdx.x / ncb, nt = blockIdx.x - mt * ncb;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, hsel = lane >> 5;
  const int cnt = (NI - wave + 3) / 4;  // DMA instructions this wave issues per stage (i = wave + 4 j < NI)
  f32x16 acc[RT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  // KM: instruction j's source walks two 16-k blocks per stage; its pointer is advanced after each
  // stage is issued (stages are issued in order), so a stage costs no address arithmetic
  const float* ksrc[PW];
  size_t kinc[PW];
  int kdst[PW];
  if constexpr (KM) {
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int i = min(wave + 4 * j, NI - 1);
      const int h = i / (NI / 2), q = i - h * (NI / 2), row = 16 * q + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      const bool isa = 16 * q < BM;
      ksrc[j] = isa ? A16 + ((size_t)h * Mimg + r0 + min(m0 + row, M - 1)) * 16 + 4 * c
                    : W16 + ((size_t)h * N + n0 + row - BM) * 16 + 4 * c;
      kinc[j] = (size_t)2 * (isa ? Mimg : N) * 16;
      kdst[j] = (h * ROWS + 16 * q) * 16;
    }
  }
  auto stage = [&](int kt) {
    float* dst = ring + (kt % NBUF) * STF;
    const int k0 = kt * G16_K;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int i = wave + 4 * j;
      if (i < NI) {
        if constexpr (KM) {  // instruction i: 16-k block h, 16 rows (A, then W) of it
          lds_dma16(ksrc[j], dst + kdst[j]);
          ksrc[j] += kinc[j];
        } else {
          const int row = 8 * i + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
          const int ar = min(m0 + row, M - 1), wr = n0 + row - BM;
          lds_dma16(row < BM ? A16 + (size_t)ar * Kp + k0 + 4 * c : W16 + (size_t)wr * Kp + k0 + 4 * c,
                    dst + 8 * i * G16_K);
        }
      }
    }
  };
  const _Float16 two11 = (_Float16)2048.0f;
  auto compute = [&](const float* src) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + hsel;  // 16-B chunk of this lane's 8 k (hi); lo is chunk 4 + ch
      // KM: block ks holds [hi 0-7 | hi 8-15 | lo 0-7 | lo 8-15] of each row: chunks hsel and 2 + hsel
      auto frag = [&](int row, bool lo) -> f16x8 {
        if constexpr (KM)
          return *reinterpret_cast<const f16x8*>(src + (ks * ROWS + row) * 16 + ((((lo ? 2 : 0) + hsel) ^ ((row >> 2) & 3)) << 2));
        else
          return *reinterpret_cast<const f16x8*>(src + row * G16_K + ((((lo ? 4 : 0) + ch) ^ ((row >> 1) & 7)) << 2));
      };
      const int wrow = BM + wave * 32 + r32;
      const f16x8 wh = frag(wrow, false);
      const f16x8 wl = frag(wrow, true);
      const f16x8 w1 = wh * two11;
#pragma unroll
      for (int tm = 0; tm < RT; ++tm) {
        const int row = tm * 32 + r32;
        const f16x8 ah = frag(row, false);
        const f16x8 al = frag(row, true);
        acc[tm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, w1, acc[tm], 0, 0, 0);
        if constexpr (kS16Cross) {
          acc[tm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, wl, acc[tm], 0, 0, 0);
          acc[tm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, wh, acc[tm], 0, 0, 0);
        }
      }
    }
  };
  const int nk = Kp / G16_K;
  for (int kt = 0; kt < NBUF - 1 && kt < nk; ++kt) stage(kt);
  for (int kt = 0; kt < nk; ++kt) {
    const int younger = min(NBUF - 2, nk - 1 - kt) * cnt;  // this wave's DMA issued after stage kt's
    if (younger >= 2 * PW) g16_vm_wait<2 * PW>();
    else if (younger >= 2 * PW - 2) g16_vm_wait<2 * PW - 2>();
    else if (younger >= PW) g16_vm_wait<PW>();
    else if (younger >= PW - 1) g16_vm_wait<PW - 1>();
    else g16_vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt landed for every wave; stage kt - 1's buffer is no longer read
    asm volatile("" ::: "memory");
    if (kt + NBUF - 1 < nk) stage(kt + NBUF - 1);
    compute(ring + (kt % NBUF) * STF);
  }
  // epilogue: RT 32-row slabs through the ring, stored as 512-B row segments (+ bias)
  constexpr int LDC = BN + 4;
  const int c4 = tid & 31, rp = tid >> 5;  // 32 float4 per row, 8 rows per pass
  const float4 b4 = *reinterpret_cast<const float4*>(bias + n0 + c4 * 4);
#pragma unroll
  for (int tm = 0; tm < RT; ++tm) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e)
      ring[((e & 3) + 8 * (e >> 2) + 4 * hsel) * LDC + wave * 32 + r32] = acc[tm][e] * S16_LO_INV;
    __syncthreads();
#pragma unroll
    for (int row = rp; row < 32; row += 8) {
      const int gr = m0 + tm * 32 + row;
      if (gr < M) {
        const float4 v = *reinterpret_cast<const float4*>(ring + row * LDC + c4 * 4);
        const float4 o4 = make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
        if (CASR_GIN_NT)
          __builtin_nontemporal_store(f32x4{o4.x, o4.y, o4.z, o4.w}, reinterpret_cast<f32x4*>(Cout + (size_t)gr * N + n0 + c4 * 4));
        else
          *reinterpret_cast<float4*>(Cout + (size_t)gr * N + n0 + c4 * 4) = o4;
      }
    }
  }
}

// tail rows [r0, M) of the input projection as gemm16_tail_kernel tiles (one round of ncu workgroups
// while the rows allow RT <= 5)
static bool launch_tail_balanced(const float* A16, const float* W16, const float* bias, float* Gin, int Mt, int N, int Kp,
                                 int ncu, hipStream_t s, int km, int r0, int Mimg) {
  if (Mt <= 0 || N % 128 != 0) return false;
  const int units = (Mt + 31) / 32 * (N / 128);
  const int RT = std::min(5, (units + ncu - 1) / ncu);  // (past 5 x ncu units: more than one round)
  const int blocks = (Mt + 32 * RT - 1) / (32 * RT) * (N / 128);
  switch (RT) {
    case 1: hipLaunchKernelGGL((km ? gemm16_tail_kernel<1, true> : gemm16_tail_kernel<1, false>), dim3(blocks), dim3(256), 0, s, A16, W16, bias, Gin, Mt, N, Kp, r0, Mimg); break;
    case 2: hipLaunchKernelGGL((km ? gemm16_tail_kernel<2, true> : gemm16_tail_kernel<2, false>), dim3(blocks), dim3(256), 0, s, A16, W16, bias, Gin, Mt, N, Kp, r0, Mimg); break;
    case 3: hipLaunchKernelGGL((km ? gemm16_tail_kernel<3, true> : gemm16_tail_kernel<3, false>), dim3(blocks), dim3(256), 0, s, A16, W16, bias, Gin, Mt, N, Kp, r0, Mimg); break;
    case 4: hipLaunchKernelGGL((km ? gemm16_tail_kernel<4, true> : gemm16_tail_kernel<4, false>), dim3(blocks), dim3(256), 0, s, A16, W16, bias, Gin, Mt, N, Kp, r0, Mimg); break;
    default: hipLaunchKernelGGL((km ? gemm16_tail_kernel<5, true> : gemm16_tail_kernel<5, false>), dim3(blocks), dim3(256), 0, s, A16, W16, bias, Gin, Mt, N, Kp, r0, Mimg); break;
  }
  return true;
}

}  // namespace

hipError_t launch_input_proj_s16_big(const float* X16, int M, int Kp, const float* W16, const float* bias,
                                     float* Gin, hipStream_t s, int K, int persist, int tail, int km, int lean) {
  const int N = 8 * H;
  if (km && (persist != 2 || tail == 1)) return hipErrorInvalidValue;  // the forms that read 16-k-major images
  if (Kp % (2 * G16_K) != 0 || M <= 0 || N % G16_N != 0) return hipErrorInvalidValue;
  const int NB = N / G16_N, NM = (M + G16_M - 1) / G16_M;
  // smallest group count whose W share (NB/NG slices of 256 rows x Kp words) fits 3/4 of an L2
  int NG = 1;
  while (NG < 8 && NB % (NG * 2) == 0 && (size_t)(NB / NG) * G16_N * Kp * 4 > (3u << 20)) NG *= 2;
  const Order16 order{NB, NM, NG};
  if (persist) {
    static int ncu = [] {
      int dev = 0, v = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
      return v > 0 ? v : 256;
    }();
    // the persistent kernel runs ceil(K / 32) stages of the Kp-wide images (both zero past K): layer
    // 0 (K = 720, Kp = 768) skips the all-zero last stage
    const int nk = (K > 0 && K <= Kp ? K + G16_K - 1 : Kp) / G16_K;
    // Balanced last round.  NB x NM tiles over ncu workgroups leave a partial last round (B = 256:
    // 2128 tiles = 8 rounds + 80 tiles, so 80 CUs run a ninth tile while 176 idle; B = 128: 4
    // rounds + 40).  The persistent kernel takes the first F = floor(NB NM / ncu) rounds (whole row
    // tiles: F ncu / NB of them, every workgroup exactly F tiles) and the rows after them go to
    // one launch of 128 x 256 half tiles (gemm16_bias_kernel<4, 1>, one per CU), which run at one
    // wave per SIMD.  Same per-element arithmetic as the persistent kernel: bitwise equal.
    int NMm = NM;
    const int F = NB * NM / ncu;
    if (tail && F >= 1 && (F * ncu) % NB == 0 && F * ncu / NB < NM) {
      const int nm = F * ncu / NB;
      const int tail_rows = M - nm * G16_M, NMt = (tail_rows + 127) / 128;
      if (NB * NMt <= ncu) NMm = nm;  // the half tiles fit one round
    }
    const Order16 om{NB, NMm, NG};
    const int total = om.blocks();
    const int Mm = std::min(M, NMm * G16_M);
    if (persist == 2) {  // ping-pong form: 16-deep stages
      const int nk16 = (K > 0 && K <= Kp ? K + 15 : Kp) / 16;
      if (km && lean && nk16 >= 8)
        hipLaunchKernelGGL(gemm16_pp_lean_kernel, dim3(std::min(total, ncu)), dim3(512), 0, s, X16, W16, bias, Gin, Mm, N,
                           om, total, nk16, M);
      else if (km)
        hipLaunchKernelGGL((gemm16_pp_kernel<0, 1, 0, 0, true>), dim3(std::min(total, ncu)), dim3(512), 0, s, X16, W16, bias,
                           Gin, Mm, N, Kp, om, total, nk16, M);
      else
        hipLaunchKernelGGL((gemm16_pp_kernel<0, 1>), dim3(std::min(total, ncu)), dim3(512), 0, s, X16, W16, bias, Gin, Mm,
                           N, Kp, om, total, nk16, M);
    } else {
      hipLaunchKernelGGL(gemm16_persist_kernel<0>, dim3(std::min(total, ncu)), dim3(512), 0, s, X16, W16, bias, Gin, Mm,
                         N, Kp, om, total, nk);
    }
    if (NMm < NM) {
      const size_t r0 = (size_t)NMm * G16_M;
      const int Mt = M - (int)r0, NMt = (Mt + 127) / 128;
      if (tail == 2 && launch_tail_balanced(km ? X16 : X16 + r0 * Kp, W16, bias, Gin + r0 * N, Mt, N, Kp, ncu, s, km,
                                            (int)r0, M))
        return hipGetLastError();
      // the row-image tail kernel below cannot read a 16-k-block-major image: a km image whose
      // balanced tail was not taken is refused, never read as rows
      if (km) return hipErrorInvalidValue;
      const Order16 ot{NB, NMt, NG};  // XCD grouping of the tail: the same column slices per XCD
      hipLaunchKernelGGL((gemm16_bias_kernel<4, 1>), dim3(ot.blocks()), dim3(256), 0, s, X16 + r0 * Kp, W16, bias,
                         Gin + r0 * N, Mt, N, Kp, ot);
    }
  } else {
    hipLaunchKernelGGL(gemm16_bias_kernel<4>, dim3(order.blocks()), dim3(512), 0, s, X16, W16, bias, Gin, M, N, Kp,
                       order);
  }
  return hipGetLastError();
}

// row image [R][Kp / 32][32 hi | 32 lo] halves -> 16-k-block major [Kp / 16][R][16 hi | 16 lo]: one
// thread per (row, 16-k block), 64 B read as two 32-B halves of the row's 128-B tile, 64 B written
__global__ void relayout_km16_kernel(const uint32_t* __restrict__ src, int R, int Kp, uint32_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = Kp / 16;
  if (i >= (size_t)R * nb) return;
  const int r = (int)(i / nb), kb = (int)(i - (size_t)r * nb);
  const uint32_t* t = src + (size_t)r * Kp + (kb >> 1) * 32 + (kb & 1) * 8;  // hi words of the block
  uint32_t* o = dst + ((size_t)kb * R + r) * 16;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] = t[e];           // hi halves
    o[8 + e] = t[16 + e];  // lo halves
  }
}

hipError_t launch_relayout_km16(const float* rowimg, int R, int Kp, float* km, hipStream_t s) {
  if (R <= 0 || Kp % 32 != 0) return hipErrorInvalidValue;
  const size_t n = (size_t)R * (Kp / 16);
  hipLaunchKernelGGL(relayout_km16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const uint32_t*>(rowimg), R, Kp, reinterpret_cast<uint32_t*>(km));
  return hipGetLastError();
}

}  // namespace casr
