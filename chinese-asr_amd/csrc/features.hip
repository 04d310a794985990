// Feature post-processing on gfx950: fbank [B][T][80] -> encoder input [B][Tp][720].
//
// Reference: add_delta_deltas (data.py:129-164: zero-pad 4 frames each side, cross-
// correlate with [identity, delta, delta-delta] 9-tap filters normalised to unit L2 norm),
// 3-frame stacking (data.py:242-249: out[j, c*240 + r*80 + m] = F[c, 3j + r, m]) and the
// per-utterance CMVN of main.py:37 ((x - mean_t) / (std_t,unbiased + eps)).
//
// HBM-bound byte work, no MFMA.  Pass 1 (stack kernel) writes the stacked, un-normalised
// rows with coalesced 720-float stores; pass 2 (cmvn kernel) owns a 64-dimension column
// slab of one utterance, reduces mean and the centred second moment over time in two
// sweeps, then normalises in place (the slab is L2-resident between the sweeps).
#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

// Filter taps as float32, normalised exactly like data.py:146-148 (float32 division by the
// float32 L2 norm).  c = 0 is the identity tap.
struct DeltaTaps {
  float d1[9];
  float d2[9];
};

__device__ __forceinline__ DeltaTaps make_taps() {
  DeltaTaps t;
  const float n1 = sqrtf(10.0f);    // 2^2 + 1 + 1 + 2^2
  const float n2 = sqrtf(198.0f);   // 16+16+1+16+100+16+1+16+16
  const float r1[9] = {0.f, 0.f, 2.f, 1.f, 0.f, -1.f, -2.f, 0.f, 0.f};
  const float r2[9] = {4.f, 4.f, 1.f, -4.f, -10.f, -4.f, 1.f, 4.f, 4.f};
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    t.d1[i] = r1[i] / n1;
    t.d2[i] = r2[i] / n2;
  }
  return t;
}

// grid (Tp, B), block 256: one stacked output row per block.
__global__ __launch_bounds__(256) void stack_kernel(const float* __restrict__ fbank,
                                                    const int32_t* __restrict__ frames, int T,
                                                    int Tp, float* __restrict__ feat,
                                                    int32_t* __restrict__ feat_len) {
  const int j = blockIdx.x, b = blockIdx.y;
  const int nf = min(frames[b], T);
  const int lp = nf / 3;
  if (j == 0 && threadIdx.x == 0) feat_len[b] = lp;
  float* out = feat + ((size_t)b * Tp + j) * D;
  if (j >= lp) {
    for (int o = threadIdx.x; o < D; o += 256) out[o] = 0.f;
    return;
  }
  const float* x = fbank + (size_t)b * T * F;
  const DeltaTaps taps = make_taps();
  for (int o = threadIdx.x; o < D; o += 256) {
    const int c = o / (3 * F);
    const int r = (o % (3 * F)) / F;
    const int m = o % F;
    const int t = 3 * j + r;
    float v;
    if (c == 0) {
      v = x[(size_t)t * F + m];
    } else {
      const float* w = (c == 1) ? taps.d1 : taps.d2;
      v = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int tt = t + k - 4;
        const float xv = (tt >= 0 && tt < nf) ? x[(size_t)tt * F + m] : 0.f;
        v = fmaf(w[k], xv, v);  // fused, as oneDNN's conv2d (torch's tap order)
      }
    }
    out[o] = v;
  }
}

// grid (ceil(D/64), B), block 256 = 64 dims x 4 time phases.
__global__ __launch_bounds__(256) void cmvn_kernel(float* __restrict__ feat,
                                                   const int32_t* __restrict__ feat_len, int Tp,
                                                   float eps) {
  __shared__ float part[4][64];
  __shared__ float stat[2][64];
  const int b = blockIdx.y;
  const int dcol = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const int n = feat_len[b];
  const bool valid = dcol < D;
  float* base = feat + (size_t)b * Tp * D + dcol;

  float s = 0.f;
  if (valid)
    for (int t = ph; t < n; t += 4) s += base[(size_t)t * D];
  part[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0) {
    const int i = threadIdx.x;
    stat[0][i] = ((part[0][i] + part[1][i]) + (part[2][i] + part[3][i])) / (float)n;
  }
  __syncthreads();
  const float mean = stat[0][threadIdx.x & 63];
  float q = 0.f;
  if (valid)
    for (int t = ph; t < n; t += 4) {
      const float dv = base[(size_t)t * D] - mean;
      q += dv * dv;
    }
  part[ph][threadIdx.x & 63] = q;
  __syncthreads();
  if (ph == 0) {
    const int i = threadIdx.x;
    const float var = ((part[0][i] + part[1][i]) + (part[2][i] + part[3][i])) / (float)(n - 1);
    stat[1][i] = sqrtf(var) + eps;
  }
  __syncthreads();
  const float den = stat[1][threadIdx.x & 63];
  if (valid)
    for (int t = ph; t < n; t += 4) {
      float* p = base + (size_t)t * D;
      *p = (*p - mean) / den;
    }
}

// Two kernels for T <= FS_MAX_T (the common case; longer utterances take the two-pass kernels
// above):
//   features_stats_kernel: grid (F / SM mel slabs, B), block 576 threads = 24 (stacked frame,
//     mel) pairs (3 x SM = 8 mels) x 24 time chunks.  The block's fbank columns (nf x 8 floats) are
//     staged in LDS once; each thread sweeps its chunk of output rows twice (sum, then centred
//     second moment) with a 9-frame register window that slides by 3 frames per row, computing
//     the three channels of its pair from the same window, and the statistics (mean, std + eps) of
//     the utterance's 720 dimensions go to a [B][2][D] buffer.
//   features_rows_kernel: grid (ceil(Tp / RJ), B), block 384 = one thread per column PAIR of an
//     output row (768 columns: the 720 features and the zero pad of the s16 image), RJ rows per
//     block from an LDS window of 3 RJ + 8 frames x 80 mels, so every row is written whole by one
//     block: coalesced 512-B segments per wave (X16: one hi word and one lo word per lane pair of
//     columns), instead of the 32-B pieces a mel-slab block left to the L2 to merge.
// The round-1/2 single-kernel form (one mel slab per block, the values of all rows of a thread in
// 68 registers: 152 VGPRs, one block per CU; stores of 32-B pieces) took 0.25 ms at B = 256, T =
// 800 (0.14 of it compute, the rest stores).
// Arithmetic: every feature value is fmaf over the 9 taps in tap order with zero frames outside
// [0, nf) (stack_kernel's); mean = the 24 chunk sums (each in row order) added in a fixed tree,
// / lp; var likewise over (v - mean)^2 / (lp - 1); std = sqrt(var) + eps (main.py:37).
constexpr int SM = 8, SRM = 3 * SM, SPH = 24, SQ = 9 * SM;  // mels, (frame, mel) pairs, chunks, dims
constexpr int FS_MAX_T = 1024;  // stats kernel's LDS: (nf + 14) x SM floats (33 KB) + 7 KB
// zero frames staged before / after the nf frames: windows reach t = -4 and, with the refill after
// a chunk's last row, t = 3 lp + 6 <= nf + 6; FS_PAD2 = 10 covers it (the refill's values are unused)
constexpr int FS_PAD = 4, FS_PAD2 = 10;
constexpr int RJ = 16, RNF = 3 * RJ + 8, RTH = 384;
static_assert(F % SM == 0 && 2 * RTH >= D, "mel slabs tile the 80 mels; a block's pairs cover a row");

// one thread per (stacked frame r, mel) pair and time chunk: the three channels (identity, delta,
// delta-delta) of a pair read the same 9-frame window, so they are computed together
__global__ __launch_bounds__(SRM * SPH) void features_stats_kernel(const float* __restrict__ fbank,
                                                                   const int32_t* __restrict__ frames, int B, int T,
                                                                   float eps, float* __restrict__ stats,
                                                                   int32_t* __restrict__ feat_len) {
  extern __shared__ float xs[];  // [FS_PAD + nf + FS_PAD2][SM]: frames -4 .. nf + 9, zero outside [0, nf)
  __shared__ float part[SPH][SQ];
  __shared__ float mean_s[SQ];
  // 1-D grid, XCD-aware: the F / SM slab blocks of one utterance take ids with equal id % 8, so
  // they run on one XCD and its L2 fetches each 320-B fbank row once for all of them (each block
  // reads a 32-B piece of every row; spread over the XCDs every piece cost a line fetch of its own)
  constexpr int NS = F / SM;
  const int L = blockIdx.x, xq = L & 7, jq = L >> 3;
  const int b = (jq / NS) * 8 + xq, m0 = (jq % NS) * SM;
  if (b >= B) return;
  const int tid = threadIdx.x, rm = tid % SRM, ph = tid / SRM;
  const int nf = min(max(frames[b], 0), T);
  const int lp = nf / 3;
  if (m0 == 0 && tid == 0) feat_len[b] = lp;
  const float* x = fbank + (size_t)b * T * F + m0;
  // every staging load of a thread in flight before its first LDS store
  constexpr int NLD = (FS_MAX_T * (SM / 4) + SRM * SPH - 1) / (SRM * SPH);
  float4 ld[NLD];
#pragma unroll
  for (int u = 0; u < NLD; ++u) {
    const int i = tid + u * SRM * SPH;
    ld[u] = make_float4(0.f, 0.f, 0.f, 0.f);  // (left undefined, hipcc kept the array in scratch)
    if (i < nf * (SM / 4)) ld[u] = *reinterpret_cast<const float4*>(x + (size_t)(i / (SM / 4)) * F + 4 * (i % (SM / 4)));
  }
#pragma unroll
  for (int u = 0; u < NLD; ++u) {
    const int i = tid + u * SRM * SPH;
    if (i < nf * (SM / 4)) *reinterpret_cast<float4*>(xs + (FS_PAD + i / (SM / 4)) * SM + 4 * (i % (SM / 4))) = ld[u];
  }
  // the zero frames either side, so the windows below read LDS with no bounds test (a test per
  // read made every window load a branch: half the kernel's instructions were exec-mask handling)
  if (tid < (FS_PAD + FS_PAD2) * (SM / 4)) {
    const int fz = tid / (SM / 4), f = fz < FS_PAD ? fz : nf + fz;
    *reinterpret_cast<float4*>(xs + f * SM + 4 * (tid % (SM / 4))) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  // pair rm = r * SM + mm; its dims q = c * SRM + rm  ->  output column c*240 + r*80 + m0 + mm
  const int r = rm / SM, mm = rm % SM;
  const DeltaTaps taps = make_taps();
  const int ch = (lp + SPH - 1) / SPH, ja = min(ph * ch, lp), jb = min(ja + ch, lp);
  auto frame = [&](int t) { return xs[(t + FS_PAD) * SM + mm]; };  // t in [-4, nf + 9]
  auto sweep = [&](auto&& use) {
    float win[9];  // frames t-4 .. t+4 of t = 3 j + r
#pragma unroll
    for (int k = 0; k < 9; ++k) win[k] = frame(3 * ja + r + k - 4);
    for (int j = ja; j < jb; ++j) {
      float v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {  // as oneDNN's conv2d (torch's tap order)
        v1 = fmaf(taps.d1[k], win[k], v1);
        v2 = fmaf(taps.d2[k], win[k], v2);
      }
      use(win[4], v1, v2);
#pragma unroll
      for (int k = 0; k < 6; ++k) win[k] = win[k + 3];
#pragma unroll
      for (int k = 6; k < 9; ++k) win[k] = frame(3 * (j + 1) + r + k - 4);
    }
  };
  // fixed-order sum of the SPH = 24 chunk partials of dim q: three groups of eight
  auto chunks = [&](int q) {
    auto g8 = [&](int g) {
      const float* p = &part[8 * g][q];
      return ((p[0] + p[SQ]) + (p[2 * SQ] + p[3 * SQ])) + ((p[4 * SQ] + p[5 * SQ]) + (p[6 * SQ] + p[7 * SQ]));
    };
    return (g8(0) + g8(1)) + g8(2);
  };
  static_assert(SPH == 24, "chunks() sums 24 partials");
#ifdef CASR_FEAT_DIAG  // diagnostic build: staging only
  if (xs[tid] == 1234.5f) stats[0] = 1.f;
  return;
#endif
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  sweep([&](float v0, float v1, float v2) {
    s0 += v0;
    s1 += v1;
    s2 += v2;
  });
  part[ph][rm] = s0;
  part[ph][SRM + rm] = s1;
  part[ph][2 * SRM + rm] = s2;
  __syncthreads();
  if (tid < SQ) mean_s[tid] = chunks(tid) / (float)lp;
  __syncthreads();
  const float mu0 = mean_s[rm], mu1 = mean_s[SRM + rm], mu2 = mean_s[2 * SRM + rm];
  s0 = s1 = s2 = 0.f;
  sweep([&](float v0, float v1, float v2) {
    const float d0 = v0 - mu0, d1 = v1 - mu1, d2 = v2 - mu2;
    s0 += d0 * d0;
    s1 += d1 * d1;
    s2 += d2 * d2;
  });
  __syncthreads();  // everyone has read part before it is reused
  part[ph][rm] = s0;
  part[ph][SRM + rm] = s1;
  part[ph][2 * SRM + rm] = s2;
  __syncthreads();
  if (tid < SQ) {
    const int c = tid / SRM, rr = (tid % SRM) / SM, m = tid % SM;
    const int o = c * 3 * F + rr * F + m0 + m;
    const float var = chunks(tid) / (float)(lp - 1);
    float* st = stats + (size_t)b * 2 * D;
    st[o] = mean_s[tid];
    st[D + o] = sqrtf(var) + eps;
  }
}

// X16: the layer-0 s16 row image of the encoder's input projection ([B Tp][Kp/32][32 hi | 32 lo]
// halves, split16_word of the same f32 value, zero columns 720..Kp-1) instead of the f32 rows, so
// the f32 features never reach HBM and split_rows_kernel does not run (casr_encode_fbank); a
// finite value beyond the f16 range raises CASR_DEV_F16_RANGE as there.  stats == nullptr: no
// CMVN (eps < 0).  Rows past a length (j >= lp) are zero.
template <bool X16>
__global__ __launch_bounds__(RTH) void features_rows_kernel(const float* __restrict__ fbank,
                                                            const int32_t* __restrict__ frames, int T, int Tp,
                                                            const float* __restrict__ stats, float* __restrict__ feat,
                                                            uint32_t* __restrict__ x16, int Kp,
                                                            int32_t* __restrict__ err, int km) {
  __shared__ __attribute__((aligned(16))) float xs[RNF * F];  // frames 3 j0 - 4 .. 3 (j0 + RJ) + 3
  // km: per-wave transpose of a row pair, so a lane stores 16 B and 8 lanes one whole 128-B line (two
  // adjacent rows' 64-B pieces of a 16-k block); 40-word pieces put the 8 blocks on distinct banks
  __shared__ __attribute__((aligned(16))) uint32_t kx[X16 ? (RTH / 64) * 8 * 40 : 1];
  const int b = blockIdx.y, j0 = blockIdx.x * RJ, p = threadIdx.x;
  const int nf = min(max(frames[b], 0), T), lp = nf / 3;
  const int t_lo = 3 * j0 - 4;
  const float* x = fbank + (size_t)b * T * F;
  constexpr int NLD = (RNF * (F / 4) + RTH - 1) / RTH;  // staging loads per thread, all in flight
  float4 ld[NLD];
#pragma unroll
  for (int u = 0; u < NLD; ++u) {
    const int i = p + u * RTH, fr = i / (F / 4), c4 = i % (F / 4), t = t_lo + fr;
    ld[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < RNF * (F / 4) && t >= 0 && t < nf) ld[u] = *reinterpret_cast<const float4*>(x + (size_t)t * F + 4 * c4);
  }
#pragma unroll
  for (int u = 0; u < NLD; ++u) {
    const int i = p + u * RTH;
    if (i < RNF * (F / 4)) *reinterpret_cast<float4*>(xs + (i / (F / 4)) * F + 4 * (i % (F / 4))) = ld[u];
  }
  __syncthreads();
  const int o0 = 2 * p;  // columns o0, o0 + 1: same channel and stacked frame, mels m, m + 1
  const bool live = o0 < D;
  const int c = live ? o0 / (3 * F) : 0, r = live ? (o0 % (3 * F)) / F : 0, m = live ? o0 % F : 0;
  float2 mean = make_float2(0.f, 0.f), den = make_float2(1.f, 1.f);
  const bool cmvn = stats != nullptr;
  if (live && cmvn) {
    const float* st = stats + (size_t)b * 2 * D + o0;
    mean = *reinterpret_cast<const float2*>(st);
    den = *reinterpret_cast<const float2*>(st + D);
  }
  const DeltaTaps taps = make_taps();
  const float* w = (c == 1) ? taps.d1 : taps.d2;
  // window of row jj: LDS frames r + 3 jj + k (k = 0..8) = t - 4 + k of t = 3 (j0 + jj) + r
  float2 win[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) win[k] = *reinterpret_cast<const float2*>(xs + (r + k) * F + m);
  bool range_ok = true;
  uint32_t ph = 0, pl = 0;  // km: the even row's hi / lo words, stored with the odd row
  const int jn = min(RJ, Tp - j0);
  for (int jj = 0; jj < jn; ++jj) {
    const int j = j0 + jj;
    float2 v = make_float2(0.f, 0.f);
    if (live && j < lp) {
      if (c == 0) {
        v = win[4];
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          v.x = fmaf(w[k], win[k].x, v.x);
          v.y = fmaf(w[k], win[k].y, v.y);
        }
      }
      if (cmvn) {
        v.x = (v.x - mean.x) / den.x;
        v.y = (v.y - mean.y) / den.y;
      }
    }
    if constexpr (X16) {
      const uint32_t w0 = split16_word(v.x), w1 = split16_word(v.y);
      // row image: 32-k tiles [32 hi | 32 lo] halves; km: 16-k-block major [Kp / 16][B Tp][16 hi | 16 lo]
      const uint32_t hw = (w0 & 0xFFFFu) | (w1 << 16), lw = (w0 >> 16) | (w1 & 0xFFFF0000u);  // hi / lo halves
      if (km && (jj & 1)) {  // rows j - 1, j (j0 is even): one 128-B line per 16-k block
        uint32_t* sc = kx + (p >> 6) * 320 + ((p & 63) >> 3) * 40;
        const int wl = p & 7;
        sc[wl] = ph;
        sc[8 + wl] = pl;
        sc[16 + wl] = hw;
        sc[24 + wl] = lw;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint4 q = *reinterpret_cast<const uint4*>(sc + 4 * wl);
        *reinterpret_cast<uint4*>(x16 + ((size_t)(o0 >> 4) * gridDim.y * Tp + (size_t)b * Tp + j - 1) * 16 + 4 * wl) = q;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else if (km && jj + 1 < jn) {
        ph = hw;
        pl = lw;
      } else {
        uint32_t* row = km ? x16 + ((size_t)(o0 >> 4) * gridDim.y * Tp + (size_t)b * Tp + j) * 16 + ((o0 & 15) >> 1)
                           : x16 + ((size_t)b * Tp + j) * Kp + (o0 >> 5) * 32 + ((o0 & 31) >> 1);
        row[0] = hw;
        row[km ? 8 : 16] = lw;
      }
      const float ax = fabsf(v.x), ay = fabsf(v.y);
      range_ok &= !(ax >= 65520.f && ax < INFINITY) && !(ay >= 65520.f && ay < INFINITY);
    } else {
      if (live) *reinterpret_cast<float2*>(feat + ((size_t)b * Tp + j) * D + o0) = v;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) win[k] = win[k + 3];
    if (jj + 1 < jn) {
#pragma unroll
      for (int k = 6; k < 9; ++k) win[k] = *reinterpret_cast<const float2*>(xs + (r + 3 * (jj + 1) + k) * F + m);
    }
  }
  if (X16 && !range_ok) __hip_atomic_fetch_or(err, CASR_DEV_F16_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_features(const float* fbank, const int32_t* frames, int B, int T, float eps,
                           float* feat, int32_t* feat_len, float* stats, hipStream_t s) {
  const int Tp = T / 3;
  if (Tp <= 0 || B <= 0) return hipErrorInvalidValue;
  // eps < 0: no CMVN (the stacked features get_log_mel returns, data.py:226-249)
  if (T <= FS_MAX_T) {
    const size_t shm = (size_t)(T + FS_PAD + FS_PAD2) * SM * sizeof(float);
    hipLaunchKernelGGL(features_stats_kernel, dim3((F / SM) * ((B + 7) / 8 * 8)), dim3(SRM * SPH), shm, s, fbank, frames, B, T, eps, stats,
                       feat_len);
    hipLaunchKernelGGL(features_rows_kernel<false>, dim3((Tp + RJ - 1) / RJ, B), dim3(RTH), 0, s, fbank, frames, T, Tp,
                       eps >= 0.f ? stats : nullptr, feat, nullptr, 0, nullptr, 0);
    return hipGetLastError();
  }
  // longer utterances: the two-pass kernels
  hipLaunchKernelGGL(stack_kernel, dim3(Tp, B), dim3(256), 0, s, fbank, frames, T, Tp, feat,
                     feat_len);
  if (eps >= 0.f)
    hipLaunchKernelGGL(cmvn_kernel, dim3((D + 63) / 64, B), dim3(256), 0, s, feat, feat_len, Tp, eps);
  return hipGetLastError();
}

bool features_x16_supported(int T) { return T / 3 > 0 && T <= FS_MAX_T; }

hipError_t launch_features_x16(const float* fbank, const int32_t* frames, int B, int T, float eps,
                               int32_t* feat_len, float* stats, uint16_t* x16, int Kp, int32_t* err, hipStream_t s,
                               int km) {
  const int Tp = T / 3;
  if (B <= 0 || !features_x16_supported(T) || Kp != 2 * RTH) return hipErrorInvalidValue;
  const size_t shm = (size_t)(T + FS_PAD + FS_PAD2) * SM * sizeof(float);
  hipLaunchKernelGGL(features_stats_kernel, dim3((F / SM) * ((B + 7) / 8 * 8)), dim3(SRM * SPH), shm, s, fbank, frames, B, T, eps, stats,
                     feat_len);
  hipLaunchKernelGGL(features_rows_kernel<true>, dim3((Tp + RJ - 1) / RJ, B), dim3(RTH), 0, s, fbank, frames, T, Tp,
                     eps >= 0.f ? stats : nullptr, nullptr, reinterpret_cast<uint32_t*>(x16), Kp, err, km);
  return hipGetLastError();
}

// grid (Tp, B): copy row j of utterance b (or zeros past its length), 16 B per lane.
__global__ __launch_bounds__(192) void gather_kernel(const float* const* __restrict__ ptrs,
                                                     const int32_t* __restrict__ lens, int Tp,
                                                     float* __restrict__ feat) {
  const int j = blockIdx.x, b = blockIdx.y;
  float4* out = reinterpret_cast<float4*>(feat + ((size_t)b * Tp + j) * D);
  const int i = threadIdx.x;  // D / 4 = 180 float4 per row
  if (i >= D / 4) return;
  if (j < lens[b]) {
    const float4* in = reinterpret_cast<const float4*>(ptrs[b] + (size_t)j * D);
    out[i] = in[i];
  } else {
    out[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

hipError_t launch_gather_utts(const float* const* ptrs, const int32_t* lens, int B, int Tp,
                              float* feat, hipStream_t s) {
  if (Tp <= 0 || B <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_kernel, dim3(Tp, B), dim3(192), 0, s, ptrs, lens, Tp, feat);
  return hipGetLastError();
}

}  // namespace casr
