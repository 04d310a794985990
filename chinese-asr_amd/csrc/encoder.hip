// BiLSTM encoder on gfx950 (RNNEncoder.forward encoder.py:36-81, RNN_RES.forward
// util.py:1223-1324) and the attention key projection (BauAttn.compute_key_value,
// attention.py:67-78).
//
// Layout in HBM: batch-major rows (b*Tp + t).
//   * input projection of a layer: one fp32 MFMA GEMM over all B*Tp rows for both
//     directions, Gin[b*Tp+t][d*4H + enc_gate_col(g,u)] = x . W_ih^T + (b_ih + b_hh)
//     (128x128 LDS-tiled, v_mfma_f32_16x16x4_f32, exact f32);
//   * recurrence: one launch per time step for both directions.  Each block owns
//     16 batch rows x 16 hidden units (x 4 gates) of one direction; its 4 waves split the
//     K = H contraction, read W_hh in MFMA-fragment-major order (one coalesced 1 KiB load
//     per wave instruction) and h_{t-1} straight into VGPRs, reduce through LDS and apply
//     the LSTM cell in the epilogue.  Packed-sequence semantics per row: forward step s
//     processes t = s, backward processes t = len_b - 1 - s, rows with s >= len_b are
//     untouched; the residual x + y (layers > 0) is fused into the output store.
#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

// ------------------------------------------------------------------ big NT GEMM
// C[M][N] = epilogue(A[M][K] . W[N][K]^T); 256 threads, 128x128 tile, BK = 32, 2x2 waves of
// 64x64 (4x4 MFMA tiles).  The k order inside a BK tile is permuted identically for A and
// W (lane group g takes k = 8g + 4*half + e) so each lane's A/W fragment is a contiguous
// float4 in LDS (ds_read_b128).  K must be a multiple of 4 (a partial last k tile is zero-filled).
constexpr int GB_M = 128, GB_N = 128, GB_K = 32;

struct StoreBiasEpi {  // C[row][col] = acc + bias[col]; N % 4 == 0, rows 16 B aligned
  static constexpr bool kRowTile = true;
  static constexpr bool kColTile = false;
  float* C;
  const float* bias;
  int ldc;
  __device__ __forceinline__ float4 bias4(int col) const { return *reinterpret_cast<const float4*>(bias + col); }
  __device__ __forceinline__ void store4(int row, int col, float4 v) const {
    *reinterpret_cast<float4*>(C + (size_t)row * ldc + col) = v;
  }
};

// keysT[b][a][t] = acc + b_attn[a], row = b*Tp + t, row stride Tq; and behind the B x A x Tq keys,
// ekT = exp(2 keys) for the attention's split exponential score form (attention.hip split_exp2x:
// v_exp_f32 of keys * 2 log2(e), NaN where |keys| >= 43, which sends a block to the direct form)
// The tile (128 rows m = b Tp + t x 128 columns a) goes out transposed (kColTile): staged through LDS
// as [a][m] in two 64-column passes, then written as float4 runs along t of keysT[b][a][.] (each
// (b, a) row is contiguous in t; Tq is a multiple of 4, so a quad t = 4q .. 4q + 3 is 16-B aligned;
// quads that cross the tile's first or last row or an utterance boundary are stored per element,
// each element by the tile that owns its row).  The scalar per-element form wrote 4-B pieces 1 KB
// apart (PMC: 129 MB written for 70 MB of keys and e^{2 keys}).
struct KeysEpi {
  static constexpr bool kRowTile = false;
  static constexpr bool kColTile = true;
  float* keysT;
  const float* bias;
  int Tp, Tq, B;
  __device__ __forceinline__ void operator()(int row, int col, float v) const {
    const int b = row / Tp, t = row - b * Tp;
    const float k = v + bias[col];
    const size_t i = ((size_t)b * A + col) * Tq + t;
    keysT[i] = k;
    keysT[(size_t)B * A * Tq + i] = split_exp2x(k);
  }
};

// XCD-aware tile order (speed only: MI355X_MICROARCH.md "Workgroup dispatch" — workgroups are
// dealt round-robin over the 8 XCDs, each with its own 4 MiB L2).  The NB column blocks are split
// into NG groups; XCD x works on group x % NG and on every (8/NG)-th row block, walking all the
// group's column blocks of one row block back to back.  Each XCD's L2 then holds 1/NG of W and
// each A row block is fetched by NG XCDs instead of all 8.
struct TileOrder {
  int NB, NM, NG;
  __host__ __device__ int blocks() const { return 8 * (NB / NG) * ((NM + 8 / NG - 1) / (8 / NG)); }
  __device__ bool tile(int L, int& n, int& m) const {
    const int x = L & 7, j = L >> 3, nbg = NB / NG;
    n = (x % NG) * nbg + (j % nbg);
    m = (j / nbg) * (8 / NG) + (x / NG);
    return m < NM;
  }
};

inline TileOrder tile_order(int NB, int NM, int K) {
  // smallest group count whose W share (NB/NG blocks of 128 rows x K) fits 3/4 of an L2
  // (input projection: NG = 2, 2.9 MB at K = 720)
  int NG = 1;
  while (NG < 8 && NB % (NG * 2) == 0 && (size_t)(NB / NG) * GB_N * K * 4 > (3u << 20)) NG *= 2;
  return TileOrder{NB, NM, NG};
}

// S16 = true: A and W are s16 row images (casr_common.h split16): row r holds K/32 k-tiles of
// 128 B = [32 hi halves | 32 lo halves], so one k-tile of a row is the same 128 B the f32 kernel
// stages (lda / ldw count 4-B words, K % 32 == 0) and the staging code is shared unchanged.
// Lane (r, g) reads chunk g (hi, k = 8g..8g+7) and chunk 4 + g (lo) of each row and issues the
// three f16 MFMAs of the s16x3 product per 16x16 tile.
template <class Epi, bool S16 = false>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const float* __restrict__ Amat, int lda,
                                                      const float* __restrict__ Wmat, int ldw,
                                                      int M, int N, int K, TileOrder order, Epi epi) {
  // Operand tiles are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4): no VGPR round
  // trip, so the next tile's loads stay in flight under all 128 MFMAs of the current one
  // (tools/probes/gemm_ablate.hip).  The two stage buffers are two distinct __shared__ arrays and
  // the k loop is unrolled by 2, so hipcc proves the in-flight DMA does not alias the ds_reads of
  // the other buffer (with one array and a runtime index it drained the DMA before every tile).
  // Rows are 128 B, lane-linear; the 16-B chunk c of row r sits at c ^ ((r >> 1) & 7) (XOR on the
  // per-lane SOURCE address, read back with the same XOR) so a ds_read_b128 over 16 rows hits 16
  // distinct bank slots.
  constexpr int TILE = GB_M * GB_K;  // floats per operand tile (16 KB)
  constexpr int LDC = GB_N + 4;      // epilogue row stride (32-row quarters)
  static_assert(32 * LDC <= 2 * TILE, "epilogue quarter fits one stage buffer");
  __shared__ __attribute__((aligned(16))) float buf0[2 * TILE];  // [A tile | W tile]
  __shared__ __attribute__((aligned(16))) float buf1[2 * TILE];

  int nt, mt;
  if (!order.tile(blockIdx.x, nt, mt)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = mt * GB_M, n0 = nt * GB_N;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // wave w stages rows [32w, 32w + 32) of the A and W tiles: 4 + 4 DMA instructions of 8 rows;
  // rows past M / N are clamped (their results are never stored)
  auto stage = [&](float* dst, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wave * 32 + i * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
      const int ar = min(m0 + row, M - 1), wr = min(n0 + row, N - 1);
      float* la = dst + (wave * 32 + i * 8) * GB_K;
      __builtin_amdgcn_global_load_lds(Amat + (size_t)ar * lda + k0 + c * 4,
                                       (__attribute__((address_space(3))) void*)la, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(Wmat + (size_t)wr * ldw + k0 + c * 4,
                                       (__attribute__((address_space(3))) void*)(la + TILE), 16, 0, 0);
    }
  };
  // partial last k tile (K = 720 = 22.5 tiles): register loads, zeros past K, same swizzle
  auto stage_partial = [&](float* dst, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, c = idx & 7, kk = k0 + c * 4;
      const int ar = min(m0 + row, M - 1), wr = min(n0 + row, N - 1);
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 va = kk < K ? *reinterpret_cast<const float4*>(Amat + (size_t)ar * lda + kk) : z;
      const float4 vw = kk < K ? *reinterpret_cast<const float4*>(Wmat + (size_t)wr * ldw + kk) : z;
      float* la = dst + row * GB_K + ((c ^ ((row >> 1) & 7)) << 2);
      *reinterpret_cast<float4*>(la) = va;
      *reinterpret_cast<float4*>(la + TILE) = vw;
    }
  };
  f32x4 accx[S16 ? 4 : 1][S16 ? 4 : 1];  // s16x3 cross-term accumulators
  if constexpr (S16) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accx[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto compute = [&](const float* src) {
    const float* as = src;
    const float* ws = src + TILE;
    if constexpr (S16) {
      f16x8 ah[4], al[4], wh[4], wl[4];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 64 + tm * 16 + r, sw = (row >> 1) & 7;
        ah[tm] = *reinterpret_cast<const f16x8*>(as + row * GB_K + ((g ^ sw) << 2));
        al[tm] = *reinterpret_cast<const f16x8*>(as + row * GB_K + (((4 + g) ^ sw) << 2));
      }
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const int row = wn * 64 + tn * 16 + r, sw = (row >> 1) & 7;
        wh[tn] = *reinterpret_cast<const f16x8*>(ws + row * GB_K + ((g ^ sw) << 2));
        wl[tn] = *reinterpret_cast<const f16x8*>(ws + row * GB_K + (((4 + g) ^ sw) << 2));
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) mfma_s16(ah[tm], al[tm], wh[tn], wl[tn], acc[tm][tn], accx[tm][tn]);
      return;
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int c = g * 2 + half;  // logical chunk of k = 8g + 4 half (same k order as the MFMA)
      float4 a[4], w[4];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int row = wm * 64 + tm * 16 + r;
        a[tm] = *reinterpret_cast<const float4*>(as + row * GB_K + ((c ^ ((row >> 1) & 7)) << 2));
      }
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const int row = wn * 64 + tn * 16 + r;
        w[tn] = *reinterpret_cast<const float4*>(ws + row * GB_K + ((c ^ ((row >> 1) & 7)) << 2));
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) {
          acc[tm][tn] = mfma16x16x4(a[tm].x, w[tn].x, acc[tm][tn]);
          acc[tm][tn] = mfma16x16x4(a[tm].y, w[tn].y, acc[tm][tn]);
          acc[tm][tn] = mfma16x16x4(a[tm].z, w[tn].z, acc[tm][tn]);
          acc[tm][tn] = mfma16x16x4(a[tm].w, w[tn].w, acc[tm][tn]);
        }
    }
  };

  const int nk = K / GB_K;  // full tiles, staged by DMA
  if (nk > 0) {
    stage(buf0, 0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; kt += 2) {
    if (kt + 1 < nk) stage(buf1, (kt + 1) * GB_K);
    compute(buf0);
    __syncthreads();  // retires this wave's DMA into buf1 and everyone's reads of buf0
    if (kt + 1 >= nk) break;
    if (kt + 2 < nk) stage(buf0, (kt + 2) * GB_K);
    compute(buf1);
    __syncthreads();
  }
  if (nk * GB_K < K) {  // both buffers are free here
    stage_partial(buf0, nk * GB_K);
    __syncthreads();
    compute(buf0);
    __syncthreads();
  }
  if constexpr (S16) {
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[tm][tn][e] = s16_combine(acc[tm][tn][e], accx[tm][tn][e]);
  }

  if constexpr (Epi::kRowTile) {
    // stage the tile through LDS in four 32-row quarters and store whole rows: 16 B per lane
    const int c4 = tid & 31, r0 = tid >> 5;  // 32 float4 per row, 8 rows per pass
    const int col = n0 + c4 * 4;
    const float4 bias4 = col < N ? epi.bias4(col) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // quarter p = rows [32p, 32p + 32): tiles tm in {2(p&1), 2(p&1)+1} of the waves with wm = p >> 1
      if (wm == (p >> 1)) {
#pragma unroll
        for (int th = 0; th < 2; ++th) {
          const int tm = 2 * (p & 1) + th;
#pragma unroll
          for (int tn = 0; tn < 4; ++tn)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              buf0[(th * 16 + g * 4 + e) * LDC + wn * 64 + tn * 16 + r] = acc[tm][tn][e];
        }
      }
      __syncthreads();
      if (col < N) {
#pragma unroll
        for (int row = r0; row < 32; row += 8) {
          if (m0 + p * 32 + row >= M) break;
          const float4 v = *reinterpret_cast<const float4*>(buf0 + row * LDC + c4 * 4);
          epi.store4(m0 + p * 32 + row, col, make_float4(v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w));
        }
      }
      __syncthreads();
    }
  } else if constexpr (Epi::kColTile) {
    // [a][m] staging, 64 columns per pass (the waves with wn == pass), rows XOR-swizzled by the
    // column (phys row = m ^ 4 (a & 15)): the 16 columns of a store hit 16 bank groups; a 4-aligned
    // run of rows stays contiguous
    static_assert(GB_N == 128 && GB_M == 128 && 64 * GB_M <= 2 * TILE, "a 64-column pass fits one stage buffer");
    const int Mt = min(GB_M, M - m0);  // rows of this tile
    const int b0 = m0 / epi.Tp, b1 = (m0 + Mt - 1) / epi.Tp;  // the utterances the tile spans
    const size_t eoff = (size_t)epi.B * A * epi.Tq;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      __syncthreads();  // the ring (or the previous pass) is no longer read
      if (wn == pass) {
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int tn = 0; tn < 4; ++tn)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int a = tn * 16 + r, m = wm * 64 + tm * 16 + g * 4 + e;  // a within the pass
              buf0[a * GB_M + (m ^ ((a & 15) << 2))] = acc[tm][tn][e];
            }
      }
      __syncthreads();
      // per utterance segment b: t in [ta, tb], quads qa .. qa + nq - 1, thread = (column, quad)
      for (int b = b0; b <= b1; ++b) {
        const int ta = max(0, m0 - b * epi.Tp), tb = min(epi.Tp - 1, m0 + Mt - 1 - b * epi.Tp);
        const int qa = ta >> 2, nq = (tb >> 2) - qa + 1;
        for (int it = tid; it < 64 * nq; it += 256) {
          const int a = it & 63, t4 = (qa + (it >> 6)) * 4;
          const int col = n0 + pass * 64 + a;
          const float bv = epi.bias[col];
          float v[4];
          bool ok[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int t = t4 + j, m = b * epi.Tp + t - m0;  // row within the tile
            ok[j] = t >= ta && t <= tb;
            v[j] = ok[j] ? buf0[a * GB_M + (m ^ ((a & 15) << 2))] + bv : 0.f;
          }
          float* kp = epi.keysT + ((size_t)b * A + col) * epi.Tq + t4;
          if (ok[0] && ok[1] && ok[2] && ok[3]) {
            *reinterpret_cast<float4*>(kp) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4*>(kp + eoff) =
                make_float4(split_exp2x(v[0]), split_exp2x(v[1]), split_exp2x(v[2]), split_exp2x(v[3]));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (ok[j]) {
                kp[j] = v[j];
                kp[eoff + j] = split_exp2x(v[j]);
              }
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const int col = n0 + wn * 64 + tn * 16 + r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * 64 + tm * 16 + g * 4 + e;
          if (row < M && col < N) epi(row, col, acc[tm][tn][e]);
        }
      }
  }
}

hipError_t launch_input_proj(const float* X, int M, int Din, const float* W, const float* bias,
                             float* Gin, hipStream_t s) {
  const int N = 8 * H;
  if (Din % 4 != 0 || M <= 0) return hipErrorInvalidValue;  // 16-B rows chunks (K tail: gemm_nt_kernel)
  StoreBiasEpi epi{Gin, bias, N};
  const TileOrder order = tile_order(N / GB_N, (M + GB_M - 1) / GB_M, Din);
  hipLaunchKernelGGL(gemm_nt_kernel<StoreBiasEpi>, dim3(order.blocks()), dim3(256), 0, s, X, Din, W,
                     Din, M, N, Din, order, epi);
  return hipGetLastError();
}

// f32 rows [M][K] (stride ldx) -> s16 row images [M][Kp/32][32 hi | 32 lo] (zeros past K).
// One thread per 8 consecutive k: two 16-B stores.  Raises CASR_DEV_F16_RANGE for a finite
// element beyond the f16 range (its hi would be infinite).
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ X, int ldx, int M, int K,
                                                         int Kp, uint16_t* __restrict__ out,
                                                         int32_t* __restrict__ err, int km) {
  const int ng = Kp / 8;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * ng) return;
  const int row = (int)(i / ng), q = (int)(i - (size_t)row * ng), k0 = q * 8;
  float v[8];
  const float* xp = X + (size_t)row * ldx + k0;
  if (k0 + 8 <= K && (ldx & 3) == 0) {
    const float4 a = *reinterpret_cast<const float4*>(xp), b = *reinterpret_cast<const float4*>(xp + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = k0 + e < K ? xp[e] : 0.f;
  }
  u32x4 hv, lv;
  bool range_ok = true;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const uint32_t w0 = split16_word(v[e]), w1 = split16_word(v[e + 1]);
    const float m = fmaxf(fabsf(v[e]), fabsf(v[e + 1]));  // f16_rn overflows from 65520 on
    range_ok &= !(m >= 65520.f && m < INFINITY);
    hv[e / 2] = __builtin_amdgcn_perm(w1, w0, 0x05040100u);
    lv[e / 2] = __builtin_amdgcn_perm(w1, w0, 0x07060302u);
  }
  if (!range_ok) __hip_atomic_fetch_or(err, CASR_DEV_F16_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // row image [M][Kp / 32][32 hi | 32 lo], or (km) 16-k-block major [Kp / 16][M][16 hi | 16 lo]
  uint16_t* op = km ? out + ((size_t)(k0 / 16) * M + row) * 32 + (k0 % 16) : out + (size_t)row * Kp * 2 + (k0 / 32) * 64 + (k0 % 32);
  *reinterpret_cast<u32x4*>(op) = hv;
  *reinterpret_cast<u32x4*>(op + (km ? 16 : 32)) = lv;
}

hipError_t launch_split_rows(const float* X, int ldx, int M, int K, int Kp, uint16_t* out, int32_t* err,
                             hipStream_t s, int km) {
  if (M <= 0 || Kp % 32 != 0 || K > Kp) return hipErrorInvalidValue;
  const size_t n = (size_t)M * (Kp / 8);
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, X, ldx, M, K, Kp, out,
                     err, km);
  return hipGetLastError();
}

hipError_t launch_keys(const float* enc, int B, int Tp, const float* wencT, const float* b_attn,
                       float* keysT, hipStream_t s) {
  const int M = B * Tp;
  if (M <= 0) return hipErrorInvalidValue;
  KeysEpi epi{keysT, b_attn, Tp, (Tp + 3) & ~3, B};
  const TileOrder order = tile_order(A / GB_N, (M + GB_M - 1) / GB_M, C);
  hipLaunchKernelGGL(gemm_nt_kernel<KeysEpi>, dim3(order.blocks()), dim3(256), 0, s, enc, C, wencT,
                     C, M, A, C, order, epi);
  return hipGetLastError();
}

// ------------------------------------------------------------------ keys, row-streaming form
// keys16_kernel (round 5, default; CASR_OPT_KEYS_ROWS = 0 keeps gemm_nt_kernel<KeysEpi, true>).  The
// keys GEMM is N = A = 128 columns by K = C = 512 over B Tp rows: gemm_nt_kernel's 128 x 128 tiles
// give 532 blocks at B = 256 for 512 slots (two per CU), so 20 blocks ran a second round and the
// launch took two block times (94 us).  Here one workgroup per CU keeps W_enc's s16 image in
// registers (wave w: columns 16 w .. 16 w + 15 over all 16 k-tiles, 128 VGPRs) and streams items of
// 16 A rows (16 consecutive t of one utterance, 32 KB) through an LDS ring of four (three in
// flight): [k-tile][16 rows][128 B], chunk c of a row's k-tile at slot c ^ ((row >> 1) & 7), filled
// by LDS-DMA.  Each wave multiplies every item by its columns with the s16x3 MFMAs of
// gemm_nt_kernel<KeysEpi, true> in the same k order, and the lane's four rows of one column are
// four consecutive t: one float4 of keysT and one of e^{2 keys} (KeysEpi's arithmetic) per lane and
// item, written by buffer stores whose lanes past the utterance's Tq slots are dropped by the
// hardware, so every wave issues exactly two stores per item and the counted vmcnt waits stay exact.
// Rows past Tp (the last item of an utterance) read row Tp - 1 and land in the pad slots
// t in [Tp, Tq), which the attention never reads (masked past len), or are dropped.
template <int VM>
CASR_DEV void g16_vm_wait_k() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
}
// (diagnostic builds only, tools/probes/keys_probe.hip: bit 0 drops the item DMA, bit 1 the MFMAs,
// bit 2 the stores; the results are then wrong)
#ifndef CASR_KR_DIAG
#define CASR_KR_DIAG 0
#endif
constexpr int KR_G = 16;                   // A rows per item
constexpr int KR_KT = C / 32;              // 32-deep k-tiles
constexpr int KR_IF = KR_KT * KR_G * 32;   // floats per item (32 KB)
constexpr int KR_NBUF = 4;                 // ring slots (three items in flight)
// 16-k-major items (km): a row's 64-B piece of a block in LDS, sub-chunk s at slot s ^ kr_swz(row):
// the swizzle {0, 2, 3, 1} by row / 4 keeps every ds_read_b128 lane group of the (row r, chunk g)
// fragment reads on 16 distinct bank groups, for the hi (s = g & 1) and the lo (s = 2 + (g & 1)) reads
CASR_DEV int kr_swz(int row) { return (120 >> (2 * ((row >> 2) & 3))) & 3; }

__global__ __launch_bounds__(512, 1) void keys16_kernel(const float* __restrict__ enc16, const float* __restrict__ w16,
                                                        const float* __restrict__ bias, float* __restrict__ keysT,
                                                        int B, int Tp, int Tq, int km) {
  __shared__ __attribute__((aligned(16))) float ring[KR_NBUF * KR_IF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, g = lane >> 4;
  const int ng = (Tp + KR_G - 1) / KR_G, NI = B * ng, G = gridDim.x;
  const int nitems = blockIdx.x < NI ? (NI - 1 - blockIdx.x) / G + 1 : 0;
  // W fragments of columns 16 w + r: lane (r, g) holds hi / lo chunk g of every k-tile
  f16x8 wh[KR_KT], wl[KR_KT];
  {
    const float* wr = w16 + (size_t)(16 * w + r) * C + 4 * g;
#pragma unroll
    for (int kt = 0; kt < KR_KT; ++kt) {
      wh[kt] = *reinterpret_cast<const f16x8*>(wr + kt * 32);
      wl[kt] = *reinterpret_cast<const f16x8*>(wr + kt * 32 + 16);
    }
  }
  const float bv = bias[16 * w + r];
  // item q of this block: utterance b, rows t = 16 j .. 16 j + 15
  auto item = [&](int q, int& b, int& j) {
    const int x = blockIdx.x + q * G;
    b = x / ng;
    j = x - b * ng;
  };
  // 32 DMA instructions of 1 KB per item (k-tile kt, rows 8 h .. 8 h + 7), four per wave.  km:
  // chunk c of a row's 32-k tile kt is sub-chunk (c & 1) + 2 (c >> 2) of 16-k block 2 kt + ((c >> 1) & 1)
  const size_t Mimg = (size_t)B * Tp;
  auto stage = [&](int q) {
    int b, j;
    item(q, b, j);
    float* dst = ring + (q % KR_NBUF) * KR_IF;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = w + 8 * u;
      if (km) {  // instruction i: 16-k block i of the 16 rows, 1 KB contiguous; slot s of a row holds
                 // sub-chunk s ^ kr_swz(row)
        const int row = lane >> 2, c = (lane & 3) ^ kr_swz(row);
        const size_t gr = (size_t)b * Tp + min(KR_G * j + row, Tp - 1);
        if (!(CASR_KR_DIAG & 1)) lds_dma16(enc16 + ((size_t)i * Mimg + gr) * 16 + 4 * c, dst + i * KR_G * 16);
      } else {
        const int kt = i >> 1, h = i & 1;
        const int row = 8 * h + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
        const size_t gr = (size_t)b * Tp + min(KR_G * j + row, Tp - 1);
        if (!(CASR_KR_DIAG & 1)) lds_dma16(enc16 + gr * C + kt * 32 + 4 * c, dst + (kt * KR_G + 8 * h) * 32);
      }
    }
  };
  // VMEM operations this wave issued after the DMA of item q, at the top of iteration q: each
  // iteration i issues the DMA of item i + 3 (when it exists, 4 operations) and then the item's two
  // stores; the prologue issues the DMAs of items 0 .. 2
  auto younger = [&](int q) {
    auto dma = [&](int i) { return i + KR_NBUF - 1 < nitems ? 4 : 0; };
    int n = 0;
    if (q < KR_NBUF - 1) {
      n += 4 * (min(KR_NBUF - 1, nitems) - 1 - q);
      for (int i = 0; i < q; ++i) n += dma(i) + 2;
    } else {
      n += 2;
      for (int i = q - KR_NBUF + 2; i < q; ++i) n += dma(i) + 2;
    }
    return n;
  };
  const size_t eoff = (size_t)B * A * Tq;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(keysT, 0, (int)(2 * eoff * 4), 0x00020000);
  for (int q = 0; q < KR_NBUF - 1 && q < nitems; ++q) stage(q);
  for (int q = 0; q < nitems; ++q) {
    const int y = younger(q);
    if (y >= 14) g16_vm_wait_k<14>();
    else if (y >= 12) g16_vm_wait_k<12>();
    else if (y >= 10) g16_vm_wait_k<10>();
    else if (y >= 8) g16_vm_wait_k<8>();
    else if (y >= 6) g16_vm_wait_k<6>();
    else if (y >= 4) g16_vm_wait_k<4>();
    else if (y >= 2) g16_vm_wait_k<2>();
    else g16_vm_wait_k<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's part of item q landed; item q - 1's slot is free
    asm volatile("" ::: "memory");
    if (q + KR_NBUF - 1 < nitems) stage(q + KR_NBUF - 1);
    const float* as = ring + (q % KR_NBUF) * KR_IF;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accx = {0.f, 0.f, 0.f, 0.f};
    const int sw = (r >> 1) & 7, swk = kr_swz(r);
#pragma unroll
    for (int kt = 0; kt < KR_KT; ++kt) {
      f16x8 ah, al;
      if (km) {  // hi chunk g of the 32-k tile = sub-chunk g & 1 of block 2 kt + (g >> 1); lo = 2 + (g & 1)
        const float* ar = as + ((2 * kt + (g >> 1)) * KR_G + r) * 16;
        ah = *reinterpret_cast<const f16x8*>(ar + (((g & 1) ^ swk) << 2));
        al = *reinterpret_cast<const f16x8*>(ar + (((2 + (g & 1)) ^ swk) << 2));
      } else {
        const float* ar = as + (kt * KR_G + r) * 32;
        ah = *reinterpret_cast<const f16x8*>(ar + ((g ^ sw) << 2));
        al = *reinterpret_cast<const f16x8*>(ar + (((4 + g) ^ sw) << 2));
      }
      if (!(CASR_KR_DIAG & 2)) mfma_s16(ah, al, wh[kt], wl[kt], acc, accx);
      else acc[0] += (float)ah[0] + (float)al[1];
    }
    int b, j;
    item(q, b, j);
    const int t0 = KR_G * j + 4 * g;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = s16_combine(acc[e], accx[e]) + bv;
    // lanes whose quad lies past the utterance's Tq slots store out of range (dropped)
    const uint32_t off = t0 < Tq ? (uint32_t)((((size_t)b * A + 16 * w + r) * Tq + t0) * 4) : 0xFFFFFFF0u;
    const float4 kq = make_float4(v[0], v[1], v[2], v[3]);
    const float4 eq = make_float4(split_exp2x(v[0]), split_exp2x(v[1]), split_exp2x(v[2]), split_exp2x(v[3]));
    const uint32_t off2 = (CASR_KR_DIAG & 4) ? 0xFFFFFFF0u : off;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, kq), rs, off2, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, eq), rs,
                                           t0 < Tq && !(CASR_KR_DIAG & 4) ? off + (uint32_t)(eoff * 4) : 0xFFFFFFF0u, 0, 0);
  }
}

// keys from the s16 row image of the encoder output (written by the last persistent layer) and
// of wencT: s16x3 products, same KeysEpi store (rows = 1: keys16_kernel, the default)
hipError_t launch_keys_s16(const float* enc16, int B, int Tp, const float* wenc16, const float* b_attn,
                           float* keysT, hipStream_t s, int rows, int km) {
  const int M = B * Tp;
  if (M <= 0 || C % GB_K != 0 || (km && !rows)) return hipErrorInvalidValue;
  if (rows) {
    static int ncu = [] {
      int dev = 0, v = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
      return v > 0 ? v : 256;
    }();
    const int Tq = (Tp + 3) & ~3, NI = B * ((Tp + KR_G - 1) / KR_G);
    if ((size_t)2 * B * A * Tq * 4 >= 0xFFFFFFF0u) return hipErrorInvalidValue;  // 32-bit buffer offsets
    hipLaunchKernelGGL(keys16_kernel, dim3(std::min(NI, ncu)), dim3(512), 0, s, enc16, wenc16, b_attn, keysT, B, Tp,
                       Tq, km);
    return hipGetLastError();
  }
  KeysEpi epi{keysT, b_attn, Tp, (Tp + 3) & ~3, B};
  const TileOrder order = tile_order(A / GB_N, (M + GB_M - 1) / GB_M, C);
  hipLaunchKernelGGL((gemm_nt_kernel<KeysEpi, true>), dim3(order.blocks()), dim3(256), 0, s, enc16, C, wenc16,
                     C, M, A, C, order, epi);
  return hipGetLastError();
}

// ------------------------------------------------------------------ recurrence step
// grid (H/16 unit blocks, ceil(B/16) row blocks, 2 directions), block 256.
// S16: s16 W_hh image and s16x3 MFMAs, the h operand split in registers by the same
// split16_word the persistent kernel's producers apply (so both paths give the same bits).
template <bool S16>
__global__ __launch_bounds__(256) void rec_step_kernel(
    const float* __restrict__ Whh_f, const float* __restrict__ Gin, const float* __restrict__ xin,
    float* __restrict__ out, const float* __restrict__ hprev, float* __restrict__ hnext,
    float* __restrict__ cst, float* __restrict__ hfin, const int32_t* __restrict__ lens, int B,
    int Tp, int step, int residual, int row0, int row1) {
  constexpr int NKC = H / 64;  // k chunks of 64
  __shared__ f32x4 red[4][4][64];
  const int jb = blockIdx.x, rb = blockIdx.y, d = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const float* Wd = Whh_f + (size_t)d * (H / 16) * 4 * NKC * FRAG;

  // epilogue cell of this thread: (row rl, unit u).  Its operands (4 gate pre-activations
  // from Gin, c, the residual input) do not depend on this step's GEMM, so they are loaded
  // first and their latency hides behind the W_hh / h loads and the MFMAs.
  const int rl = threadIdx.x >> 4, u = threadIdx.x & 15;
  const int b = row0 + rb * 16 + rl;  // rows [row0, row1) of the batch
  const int len = b < row1 ? min(lens[b], Tp) : 0;
  const bool act = step < len;
  const int t = (d == 0) ? step : (len - 1 - step);
  const int U = jb * 16 + u;
  const size_t si = ((size_t)d * B + b) * H + U;
  const size_t oi = ((size_t)b * Tp + t) * C + d * H + U;
  float gin_v[4] = {0.f, 0.f, 0.f, 0.f}, c_old = 0.f, x_res = 0.f;
  if (act) {
    const float4 q = *reinterpret_cast<const float4*>(Gin + ((size_t)b * Tp + t) * (8 * H) + d * 4 * H + U * 4);
    gin_v[0] = q.x, gin_v[1] = q.y, gin_v[2] = q.z, gin_v[3] = q.w;  // enc_gate_col: adjacent gates
    c_old = cst[si];
    if (residual) x_res = xin[oi];
  }

  f32x4 acc[4];
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) acc[tn] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int row = row0 + rb * 16 + r;
  for (int kc = w; kc < NKC; kc += 4) {
    float4 a[4], bw[4][4];
    const float* ap = hprev + ((size_t)d * B + row) * H + kc * 64 + g * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      a[q] = row < row1 ? *reinterpret_cast<const float4*>(ap + q * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const float* wb = Wd + ((size_t)(jb * 4 + tn) * NKC + kc) * FRAG + lane * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) bw[tn][q] = *reinterpret_cast<const float4*>(wb + q * 256);
    }
    if constexpr (S16) {
      // unit 16g + 8j + e of the chunk: a[2j] / a[2j + 1] hold e = 0..3 / 4..7
      f32x4 accx[4];
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) accx[tn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float4 p = a[2 * j], q = a[2 * j + 1];
        const u32x4 w0 = {split16_word(p.x), split16_word(p.y), split16_word(p.z), split16_word(p.w)};
        const u32x4 w1 = {split16_word(q.x), split16_word(q.y), split16_word(q.z), split16_word(q.w)};
        f16x8 ah, al;
        unpack16(w0, w1, ah, al);
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
          mfma_s16(ah, al, __builtin_bit_cast(f16x8, bw[tn][2 * j]), __builtin_bit_cast(f16x8, bw[tn][2 * j + 1]),
                   acc[tn], accx[tn]);
      }
#pragma unroll
      for (int tn = 0; tn < 4; ++tn)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[tn][e] = s16_combine(acc[tn][e], accx[tn][e]);
      continue;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        acc[tn] = mfma16x16x4(a[q].x, bw[tn][q].x, acc[tn]);
        acc[tn] = mfma16x16x4(a[q].y, bw[tn][q].y, acc[tn]);
        acc[tn] = mfma16x16x4(a[q].z, bw[tn][q].z, acc[tn]);
        acc[tn] = mfma16x16x4(a[q].w, bw[tn][q].w, acc[tn]);
      }
  }
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) red[w][tn][lane] = acc[tn];
  __syncthreads();

  if (!act) return;
  const int src_lane = u + 16 * (rl >> 2), reg = rl & 3;
  float gate[4];
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    float sum = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) sum += red[ww][tn][src_lane][reg];
    gate[tn] = sum + gin_v[tn];
  }
  float h2, c2;
  if constexpr (S16)  // the persistent kernel's cell, bit for bit
    lstm_cell_hw(gate[0], gate[1], gate[2], gate[3], c_old, h2, c2);
  else
    lstm_cell(gate[0], gate[1], gate[2], gate[3], c_old, h2, c2);
  cst[si] = c2;
  hnext[si] = h2;
  if (step == len - 1) hfin[si] = h2;
  out[oi] = residual ? residual_add(h2, x_res) : h2;
}

hipError_t launch_rec_step(const float* Whh_f, const float* Gin, const float* xin, float* out,
                           const float* hprev, float* hnext, float* cst, float* hfin,
                           const int32_t* lens, int B, int Tp, int step, int residual, int row0, int row1,
                           int s16, hipStream_t s) {
  dim3 grid(H / 16, (row1 - row0 + 15) / 16, 2);
  if (s16)
    hipLaunchKernelGGL(rec_step_kernel<true>, grid, dim3(256), 0, s, Whh_f, Gin, xin, out, hprev, hnext,
                       cst, hfin, lens, B, Tp, step, residual, row0, row1);
  else
    hipLaunchKernelGGL(rec_step_kernel<false>, grid, dim3(256), 0, s, Whh_f, Gin, xin, out, hprev, hnext,
                       cst, hfin, lens, B, Tp, step, residual, row0, row1);
  return hipGetLastError();
}

}  // namespace casr
