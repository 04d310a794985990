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

// One pass for the whole chain (stack + deltas + CMVN): grid (F / FM mel slabs, B), block
// 4 x 144 threads = 144 output dimensions (3 channels x 3 stacked frames x FM = 16 mels) x 4
// time phases.  The block's fbank columns (nf x 16 floats) are staged in LDS once; each thread
// computes its dimension's delta features for its time phase once, into registers (NJ per
// thread), and the three sweeps (mean, centred second moment, normalise + store) run from
// there, instead of round-tripping the un-normalised rows through HBM (the two kernels above:
// 654 MB of traffic at B = 256, T = 800; here 65 MB read + 196 MB written).  Every feature value
// is computed with stack_kernel's arithmetic (same taps and tap order); the statistics use
// cmvn_kernel's 4-phase fixed-order reduction.
constexpr int FM = 16, FQ = 9 * FM, FPH = 4, FNJ = 68;  // FNJ x FPH >= Tp (T <= 816 frames)
static_assert(F % FM == 0, "mel slabs tile the 80 mels");

// X16: instead of the f32 rows, the layer-0 s16 row image of the encoder's input projection
// ([B Tp][Kp/32][32 hi | 32 lo] halves, split16_word of the same f32 value, zero columns
// 720..Kp-1), so the f32 features never reach HBM and split_rows_kernel does not run
// (casr_encode_fbank); a finite value beyond the f16 range raises CASR_DEV_F16_RANGE as there.
template <bool X16>
__global__ __launch_bounds__(FQ * FPH) void features_fused_kernel(const float* __restrict__ fbank,
                                                                  const int32_t* __restrict__ frames, int T,
                                                                  int Tp, float eps, float* __restrict__ feat,
                                                                  int32_t* __restrict__ feat_len,
                                                                  uint16_t* __restrict__ x16, int Kp,
                                                                  int32_t* __restrict__ err) {
  extern __shared__ float xs[];  // [nf][FM]
  __shared__ float part[FPH][FQ];
  __shared__ float stat[2][FQ];
  const int m0 = blockIdx.x * FM, b = blockIdx.y;
  const int tid = threadIdx.x, q = tid % FQ, ph = tid / FQ;
  const int nf = min(frames[b], T);
  const int lp = nf / 3;
  if (blockIdx.x == 0 && tid == 0) feat_len[b] = lp;
  const float* x = fbank + (size_t)b * T * F + m0;
  for (int i = tid; i < nf * (FM / 4); i += FQ * FPH) {
    const int t = i / (FM / 4), c4 = i % (FM / 4);
    *reinterpret_cast<float4*>(xs + t * FM + 4 * c4) = *reinterpret_cast<const float4*>(x + (size_t)t * F + 4 * c4);
  }
  __syncthreads();
  // dimension q = (c * 3 + r) * FM + mm  ->  output column c*240 + r*80 + m0 + mm
  const int cr = q / FM, mm = q % FM, c = cr / 3, r = cr % 3;
  const int o = c * 3 * F + r * F + m0 + mm;
  const DeltaTaps taps = make_taps();
  const float* w = (c == 1) ? taps.d1 : taps.d2;
  float vals[FNJ];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FNJ; ++i) {
    const int j = ph + FPH * i;
    float v = 0.f;
    if (j < lp) {
      const int t = 3 * j + r;
      if (c == 0) {
        v = xs[t * FM + mm];
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int tt = t + k - 4;
          const float xv = (tt >= 0 && tt < nf) ? xs[tt * FM + mm] : 0.f;
          v = fmaf(w[k], xv, v);  // fused, as oneDNN's conv2d (torch's tap order)
        }
      }
      s += v;
    }
    vals[i] = v;
  }
  float mean = 0.f, den = 1.f;
  if (eps >= 0.f) {
    part[ph][q] = s;
    __syncthreads();
    if (ph == 0) stat[0][q] = ((part[0][q] + part[1][q]) + (part[2][q] + part[3][q])) / (float)lp;
    __syncthreads();
    mean = stat[0][q];
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FNJ; ++i)
      if (ph + FPH * i < lp) {
        const float dv = vals[i] - mean;
        s2 += dv * dv;
      }
    __syncthreads();  // everyone has read part before it is reused
    part[ph][q] = s2;
    __syncthreads();
    if (ph == 0) {
      const float var = ((part[0][q] + part[1][q]) + (part[2][q] + part[3][q])) / (float)(lp - 1);
      stat[1][q] = sqrtf(var) + eps;
    }
    __syncthreads();
    den = stat[1][q];
  }
  if constexpr (X16) {
    // lanes q and q ^ 1 hold adjacent columns o, o + 1 (o even: FQ, the mel slab and FM are
    // even): the even lane stores both hi halves as one word, the odd lane both lo halves
    const bool odd = q & 1;
    uint32_t* xo = reinterpret_cast<uint32_t*>(x16 + (size_t)b * Tp * Kp * 2 + ((o & ~1) / 32) * 64 +
                                               ((o & ~1) % 32) + (odd ? 32 : 0));
    bool range_ok = true;
#pragma unroll
    for (int i = 0; i < FNJ; ++i) {
      const int j = ph + FPH * i;
      if (j < Tp) {  // uniform over the lane pair (same time phase)
        const float y = (j < lp && eps >= 0.f) ? (vals[i] - mean) / den : vals[i];
        const uint32_t wv = split16_word(y);
        const uint32_t pw = (uint32_t)dpp_i<DPP_XOR1>((int)wv);
        xo[(size_t)j * Kp] = odd ? ((pw >> 16) | (wv & 0xFFFF0000u)) : ((wv & 0xFFFFu) | (pw << 16));
        const float m = fabsf(y);
        range_ok &= !(m >= 65520.f && m < INFINITY);
      }
    }
    if (!range_ok) __hip_atomic_fetch_or(err, CASR_DEV_F16_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) {  // the zero columns D..Kp-1 of every row of this utterance
      const int npad = Kp - D;
      for (int i = tid; i < Tp * npad; i += FQ * FPH) {
        const int j = i / npad, col = D + i % npad;
        uint16_t* zp = x16 + ((size_t)b * Tp + j) * Kp * 2 + (col / 32) * 64 + (col % 32);
        zp[0] = 0;
        zp[32] = 0;
      }
    }
  } else {
    float* out = feat + (size_t)b * Tp * D + o;
#pragma unroll
    for (int i = 0; i < FNJ; ++i) {
      const int j = ph + FPH * i;
      if (j < Tp) out[(size_t)j * D] = (j < lp && eps >= 0.f) ? (vals[i] - mean) / den : vals[i];
    }
  }
}

hipError_t launch_features(const float* fbank, const int32_t* frames, int B, int T, float eps,
                           float* feat, int32_t* feat_len, hipStream_t s) {
  const int Tp = T / 3;
  if (Tp <= 0 || B <= 0) return hipErrorInvalidValue;
  // eps < 0: no CMVN (the stacked features get_log_mel returns, data.py:226-249)
  if (Tp <= FNJ * FPH) {
    const size_t shm = (size_t)T * FM * sizeof(float);
    hipLaunchKernelGGL(features_fused_kernel<false>, dim3(F / FM, B), dim3(FQ * FPH), shm, s, fbank, frames, T, Tp,
                       eps, feat, feat_len, nullptr, 0, nullptr);
    return hipGetLastError();
  }
  // longer utterances: the two-pass kernels
  hipLaunchKernelGGL(stack_kernel, dim3(Tp, B), dim3(256), 0, s, fbank, frames, T, Tp, feat,
                     feat_len);
  if (eps >= 0.f)
    hipLaunchKernelGGL(cmvn_kernel, dim3((D + 63) / 64, B), dim3(256), 0, s, feat, feat_len, Tp, eps);
  return hipGetLastError();
}

bool features_x16_supported(int T) { return T / 3 > 0 && T / 3 <= FNJ * FPH; }

hipError_t launch_features_x16(const float* fbank, const int32_t* frames, int B, int T, float eps,
                               int32_t* feat_len, uint16_t* x16, int Kp, int32_t* err, hipStream_t s) {
  const int Tp = T / 3;
  if (B <= 0 || !features_x16_supported(T) || Kp < D || Kp % 32 != 0) return hipErrorInvalidValue;
  const size_t shm = (size_t)T * FM * sizeof(float);
  hipLaunchKernelGGL(features_fused_kernel<true>, dim3(F / FM, B), dim3(FQ * FPH), shm, s, fbank, frames, T, Tp, eps,
                     nullptr, feat_len, x16, Kp, err);
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
