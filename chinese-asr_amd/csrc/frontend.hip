// wav -> log-mel front-end on gfx950 (get_log_mel data.py:167-224, inference: no dither, no
// augmentation; MelScale / create_fb_matrix data.py:21-106; AudioBase data.py:371-382).
//
//   y[m]   = x[m+1] - 0.97 x[m]                            (float32, data.py:201-202)
//   frame f: y[160 f + j] * w[j], j < 512, w = periodic hann(400) zero-padded to 512 and centred
//            (torch.stft n_fft 512, hop 160, win_length 400, center=False, data.py:205-208)
//   P[k]   = |rfft_512(frame)[k]|^2, k <= 256                (data.py:220-221)
//   mel    = P . fb  (fb [257][80], linspace(80, 7600, 257) bin-frequency quirk, data.py:43)
//   out    = log(mel == 0 ? FLT_EPSILON : mel)               (data.py:223-224)
//
// One wave per frame, 4 frames in flight per 256-thread block.  The 512-point real transform is a
// 256-point complex radix-2 FFT of z[m] = y[2m] + i y[2m+1] in LDS followed by the even/odd
// split; it runs in fp64 so its rounding is far below the reference's own fp32 FFT error (the
// oracle does the same, numpy float64 rfft).  Power and the mel projection are float32 like the
// reference.  Frames past an utterance's length are written as zeros.  The constant tables
// (fb with per-filter nonzero ranges, window, twiddles) are built on the host in this file.
#include <math.h>

#include <vector>

#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

namespace {
constexpr int NFFT = 512, HOP = 160, WIN = 400, LPAD = (NFFT - WIN) / 2, NBIN = NFFT / 2 + 1;
constexpr int NC = NFFT / 2;  // complex FFT size
constexpr int FPB = 4;        // frames per block (one per wave)

// torch's elementwise steps, each rounded (no FMA contraction: hipcc's default would fuse them):
// pre-emphasis x[t+1] - 0.97 x[t] (data.py:201-202), the window product, |X|^2 = re^2 + im^2
// (data.py:220-221)
CASR_DEV float preemph_win(float w, float x1, float x0, float pre) {
#pragma clang fp contract(off)
  return w * (x1 - pre * x0);
}
CASR_DEV float power2(float re, float im) {
#pragma clang fp contract(off)
  return re * re + im * im;
}

__device__ __forceinline__ int bitrev8(int x) { return (int)(__brev((unsigned)x) >> 24); }

__global__ __launch_bounds__(256) void log_mel_kernel(const float* __restrict__ wav,
                                                      const int32_t* __restrict__ nsamp, int Nmax,
                                                      int Tmax, float pre, const FrontendConst* __restrict__ k,
                                                      float* __restrict__ out, int32_t* __restrict__ frames,
                                                      int32_t* __restrict__ err) {
  __shared__ double zr[FPB][NC], zi[FPB][NC];
  __shared__ float pw[FPB][NBIN + 3];
  const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * FPB + w;
  int n = nsamp[b];
  if (n < NFFT + 1 || n > Nmax) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, CASR_DEV_BAD_AUDIO);
    n = n > Nmax ? Nmax : n;
  }
  const int L = n - 1 >= NFFT ? 1 + (n - 1 - NFFT) / HOP : 0;  // frames of the pre-emphasised signal
  if (blockIdx.x == 0 && threadIdx.x == 0) frames[b] = L < Tmax ? L : Tmax;
  // every wave runs through every barrier; only frames f < min(L, Tmax) read samples
  const bool live = f < L && f < Tmax;
  const float* x = wav + (size_t)b * Nmax + (size_t)(live ? f : 0) * HOP;
  // windowed frame, complex-packed and bit-reversed: z[m] = (y[2m] w[2m], y[2m+1] w[2m+1])
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = lane + 64 * i, j0 = 2 * m, j1 = j0 + 1;
    float v0 = 0.f, v1 = 0.f;
    if (live && j0 >= LPAD && j0 < LPAD + WIN)
      v0 = preemph_win(k->win[j0 - LPAD], x[j0 + 1], x[j0], pre);
    if (live && j1 >= LPAD && j1 < LPAD + WIN)
      v1 = preemph_win(k->win[j1 - LPAD], x[j1 + 1], x[j1], pre);
    const int r = bitrev8(m);
    zr[w][r] = v0;
    zi[w][r] = v1;
  }
  __syncthreads();
  // 8 radix-2 DIT stages, 128 butterflies each: 2 per lane
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int half = 1 << s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = lane + 64 * i, pos = t & (half - 1);
      const int i0 = ((t >> s) << (s + 1)) + pos, i1 = i0 + half;
      const double wr = k->tw256r[pos << (7 - s)], wi = k->tw256i[pos << (7 - s)];
      const double br = zr[w][i1] * wr - zi[w][i1] * wi, bi = zr[w][i1] * wi + zi[w][i1] * wr;
      const double ar = zr[w][i0], ai = zi[w][i0];
      zr[w][i0] = ar + br;
      zi[w][i0] = ai + bi;
      zr[w][i1] = ar - br;
      zi[w][i1] = ai - bi;
    }
    __syncthreads();
  }
  // real-input split: X[q] = E + W512^q O, E = (Z[q] + conj Z[-q]) / 2, O = (Z[q] - conj Z[-q]) / 2i
  for (int q = lane; q < NBIN; q += 64) {
    const int qa = q & (NC - 1), qb = (NC - q) & (NC - 1);
    const double zr1 = zr[w][qa], zi1 = zi[w][qa], zr2 = zr[w][qb], zi2 = -zi[w][qb];
    const double er = 0.5 * (zr1 + zr2), ei = 0.5 * (zi1 + zi2);
    const double orr = 0.5 * (zi1 - zi2), oi = -0.5 * (zr1 - zr2);
    const double c = k->tw512r[q], sn = k->tw512i[q];
    const float xr = (float)(er + (orr * c - oi * sn)), xi = (float)(ei + (orr * sn + oi * c));
    pw[w][q] = power2(xr, xi);
  }
  __syncthreads();
  if (f >= Tmax) return;
  float* o = out + ((size_t)b * Tmax + f) * F;
  for (int m = lane; m < F; m += 64) {
    if (!live) {  // padding rows past the utterance
      o[m] = 0.f;
      continue;
    }
    float acc = 0.f;
    for (int q = k->lo[m]; q < k->hi[m]; ++q) acc = fmaf(pw[w][q], k->fb[q * F + m], acc);  // matmul: fused
    o[m] = logf(acc == 0.f ? 1.1920928955078125e-07f : acc);
  }
}
}  // namespace

// create_fb_matrix (data.py:21-57) in float32 like the reference's torch ops, including the
// quirk stft_freqs = linspace(f_min, f_max, n_stft) (data.py:43).  fb is [n_stft][n_mels].
void mel_filterbank(int n_stft, float f_min, float f_max, int n_mels, float* fb) {
  auto linspace = [](float a, float e, int n, int i) -> float {  // torch CPU linspace (symmetric)
    if (n == 1) return a;
    const float step = (e - a) / (float)(n - 1);
    return i < n / 2 ? a + step * (float)i : e - step * (float)(n - 1 - i);
  };
  auto hz2mel = [](float f) { return 2595.f * log10f(1.f + f / 700.f); };
  auto mel2hz = [](float m) { return 700.f * (powf(10.f, m / 2595.f) - 1.f); };
  const float m_min = f_min == 0.f ? 0.f : hz2mel(f_min), m_max = hz2mel(f_max);
  std::vector<float> f_pts(n_mels + 2), f_diff(n_mels + 1);
  for (int i = 0; i < n_mels + 2; ++i) f_pts[i] = mel2hz(linspace(m_min, m_max, n_mels + 2, i));
  for (int i = 0; i < n_mels + 1; ++i) f_diff[i] = f_pts[i + 1] - f_pts[i];
  for (int q = 0; q < n_stft; ++q) {
    const float fq = linspace(f_min, f_max, n_stft, q);
    for (int m = 0; m < n_mels; ++m) {
      const float down = (-1.f * (f_pts[m] - fq)) / f_diff[m];
      const float up = (f_pts[m + 2] - fq) / f_diff[m + 1];
      const float v = down < up ? down : up;
      fb[q * n_mels + m] = v > 0.f ? v : 0.f;
    }
  }
}

void build_frontend_const(FrontendConst* c) {
  float fb[NBIN * F];
  mel_filterbank(NBIN, 80.f, 7600.f, F, fb);
  for (int i = 0; i < NBIN * F; ++i) c->fb[i] = fb[i];
  for (int m = 0; m < F; ++m) {
    int lo = NBIN, hi = 0;
    for (int q = 0; q < NBIN; ++q)
      if (fb[q * F + m] != 0.f) {
        lo = q < lo ? q : lo;
        hi = q + 1;
      }
    c->lo[m] = lo < hi ? lo : 0;
    c->hi[m] = lo < hi ? hi : 0;
  }
  // torch.hann_window(400) (periodic): 0.5 - 0.5 cos(2 pi j / 400), evaluated in float32
  for (int j = 0; j < WIN; ++j) c->win[j] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * j / WIN));
  for (int i = 0; i < NC / 2; ++i) {
    c->tw256r[i] = cos(-2.0 * M_PI * i / NC);
    c->tw256i[i] = sin(-2.0 * M_PI * i / NC);
  }
  for (int q = 0; q < NBIN; ++q) {
    c->tw512r[q] = cos(-2.0 * M_PI * q / NFFT);
    c->tw512i[q] = sin(-2.0 * M_PI * q / NFFT);
  }
}

int frontend_frames(int n_samples) {
  return n_samples - 1 >= NFFT ? 1 + (n_samples - 1 - NFFT) / HOP : 0;
}

hipError_t launch_log_mel(const float* wav, const int32_t* nsamp, int B, int Nmax, int Tmax, float pre,
                          const FrontendConst* k, float* out, int32_t* frames, int32_t* err, hipStream_t s) {
  dim3 grid((Tmax + FPB - 1) / FPB > 0 ? (Tmax + FPB - 1) / FPB : 1, B);
  hipLaunchKernelGGL(log_mel_kernel, grid, dim3(256), 0, s, wav, nsamp, Nmax, Tmax, pre, k, out, frames, err);
  return hipGetLastError();
}

}  // namespace casr
