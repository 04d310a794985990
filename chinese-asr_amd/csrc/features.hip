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
//   features_stats_kernel: grid (F / SM mel slabs, B), block SQ x SPH threads = 144 output
//     dimensions (3 channels x 3 stacked frames x SM = 16 mels) x 4 time chunks.  The block's
//     fbank columns (nf x 16 floats) are staged in LDS once; each thread sweeps its chunk of output
//     rows twice (sum, then centred second moment) with a 9-frame register window that slides by
//     3 frames per row (3 LDS reads per value), and the statistics (mean, std + eps) of the
//     utterance's 720 dimensions go to a [B][2][D] buffer.
//   features_rows_kernel: grid (ceil(Tp / RJ), B), block 384 = one thread per column PAIR of an
//     output row (768 columns: the 720 features and the zero pad of the s16 image), RJ rows per
//     block from an LDS window of 3 RJ + 8 frames x 80 mels, so every row is written whole by one
//     block: coalesced 512-B segments per wave (X16: one hi word and one lo word per lane pair of
//     columns), instead of the 32-B pieces a mel-slab block left to the L2 to merge.
// The round-1/2 single-kernel form (one mel slab per block, the values of all rows of a thread in
// 68 registers: 152 VGPRs, one block per CU; stores of 32-B pieces) took 0.25 ms at B = 256, T =
// 800 (0.14 of it compute, the rest stores).
// Arithmetic: every feature value is fmaf over the 9 taps in tap order with zero frames outside
// [0, nf) (stack_kernel's); mean = ((s0 + s1) + (s2 + s3)) / lp over the four chunk sums (each in
// row order), var likewise over (v - mean)^2 / (lp - 1), std = sqrt(var) + eps (main.py:37).
constexpr int SM = 16, SQ = 9 * SM, SPH = 4;
constexpr int FS_MAX_T = 900;  // stats kernel's LDS: nf x SM floats (56 KB) + 3 KB, under 64 KB
constexpr int RJ = 16, RNF = 3 * RJ + 8, RTH = 384;
static_assert(F % SM == 0 && 2 * RTH >= D, "mel slabs tile the 80 mels; a block's pairs cover a row");

__global__ __launch_bounds__(SQ * SPH) void features_stats_kernel(const float* __restrict__ fbank,
                                                                  const int32_t* __restrict__ frames, int T,
                                                                  float eps, float* __restrict__ stats,
                                                                  int32_t* __restrict__ feat_len) {
  extern __shared__ float xs[];  // [nf][SM]
  __shared__ float part[SPH][SQ];
  __shared__ float mean_s[SQ];
  const int m0 = blockIdx.x * SM, b = blockIdx.y;
  const int tid = threadIdx.x, q = tid % SQ, ph = tid / SQ;
  const int nf = min(max(frames[b], 0), T);
  const int lp = nf / 3;
  if (blockIdx.x == 0 && tid == 0) feat_len[b] = lp;
  const float* x = fbank + (size_t)b * T * F + m0;
  for (int i = tid; i < nf * (SM / 4); i += SQ * SPH) {
    const int t = i / (SM / 4), c4 = i % (SM / 4);
    *reinterpret_cast<float4*>(xs + t * SM + 4 * c4) = *reinterpret_cast<const float4*>(x + (size_t)t * F + 4 * c4);
  }
  __syncthreads();
  // dimension q = (c * 3 + r) * SM + mm  ->  output column c*240 + r*80 + m0 + mm
  const int cr = q / SM, mm = q % SM, c = cr / 3, r = cr % 3;
  const int o = c * 3 * F + r * F + m0 + mm;
  const DeltaTaps taps = make_taps();
  const float* w = (c == 1) ? taps.d1 : taps.d2;
  const int ch = (lp + SPH - 1) / SPH, ja = min(ph * ch, lp), jb = min(ja + ch, lp);
  auto frame = [&](int t) { return (t >= 0 && t < nf) ? xs[t * SM + mm] : 0.f; };
  auto sweep = [&](auto&& use) {
    float win[9];  // frames t-4 .. t+4 of t = 3 j + r
#pragma unroll
    for (int k = 0; k < 9; ++k) win[k] = frame(3 * ja + r + k - 4);
    for (int j = ja; j < jb; ++j) {
      float v = 0.f;
      if (c == 0) {
        v = win[4];
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) v = fmaf(w[k], win[k], v);  // as oneDNN's conv2d (torch's tap order)
      }
      use(v);
#pragma unroll
      for (int k = 0; k < 6; ++k) win[k] = win[k + 3];
#pragma unroll
      for (int k = 6; k < 9; ++k) win[k] = frame(3 * (j + 1) + r + k - 4);
    }
  };
  float s = 0.f;
  sweep([&](float v) { s += v; });
  part[ph][q] = s;
  __syncthreads();
  if (ph == 0) mean_s[q] = ((part[0][q] + part[1][q]) + (part[2][q] + part[3][q])) / (float)lp;
  __syncthreads();
  const float mean = mean_s[q];
  float s2 = 0.f;
  sweep([&](float v) {
    const float dv = v - mean;
    s2 += dv * dv;
  });
  __syncthreads();  // everyone has read part before it is reused
  part[ph][q] = s2;
  __syncthreads();
  if (ph == 0) {
    const float var = ((part[0][q] + part[1][q]) + (part[2][q] + part[3][q])) / (float)(lp - 1);
    float* st = stats + (size_t)b * 2 * D;
    st[o] = mean;
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
                                                            int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) float xs[RNF * F];  // frames 3 j0 - 4 .. 3 (j0 + RJ) + 3
  const int b = blockIdx.y, j0 = blockIdx.x * RJ, p = threadIdx.x;
  const int nf = min(max(frames[b], 0), T), lp = nf / 3;
  const int t_lo = 3 * j0 - 4;
  const float* x = fbank + (size_t)b * T * F;
  for (int i = p; i < RNF * (F / 4); i += RTH) {
    const int fr = i / (F / 4), c4 = i % (F / 4), t = t_lo + fr;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t >= 0 && t < nf) v = *reinterpret_cast<const float4*>(x + (size_t)t * F + 4 * c4);
    *reinterpret_cast<float4*>(xs + fr * F + 4 * c4) = v;
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
      uint32_t* row = x16 + ((size_t)b * Tp + j) * Kp + (o0 >> 5) * 32 + ((o0 & 31) >> 1);
      row[0] = (w0 & 0xFFFFu) | (w1 << 16);            // hi halves of columns o0, o0 + 1
      row[16] = (w0 >> 16) | (w1 & 0xFFFF0000u);      // lo halves
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
    const size_t shm = (size_t)T * SM * sizeof(float);
    hipLaunchKernelGGL(features_stats_kernel, dim3(F / SM, B), dim3(SQ * SPH), shm, s, fbank, frames, T, eps, stats,
                       feat_len);
    hipLaunchKernelGGL(features_rows_kernel<false>, dim3((Tp + RJ - 1) / RJ, B), dim3(RTH), 0, s, fbank, frames, T, Tp,
                       eps >= 0.f ? stats : nullptr, feat, nullptr, 0, nullptr);
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
                               int32_t* feat_len, float* stats, uint16_t* x16, int Kp, int32_t* err, hipStream_t s) {
  const int Tp = T / 3;
  if (B <= 0 || !features_x16_supported(T) || Kp != 2 * RTH) return hipErrorInvalidValue;
  const size_t shm = (size_t)T * SM * sizeof(float);
  hipLaunchKernelGGL(features_stats_kernel, dim3(F / SM, B), dim3(SQ * SPH), shm, s, fbank, frames, T, eps, stats,
                     feat_len);
  hipLaunchKernelGGL(features_rows_kernel<true>, dim3((Tp + RJ - 1) / RJ, B), dim3(RTH), 0, s, fbank, frames, T, Tp,
                     eps >= 0.f ? stats : nullptr, nullptr, reinterpret_cast<uint32_t*>(x16), Kp, err);
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
