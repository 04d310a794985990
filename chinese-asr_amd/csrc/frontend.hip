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
// One wave per frame; a 256-thread block runs 4 waves, each over FE_FPW consecutive frames.  The
// 512-point real transform is a 256-point complex FFT of z[m] = y[2m] + i y[2m+1] followed by the
// even/odd split, all in float32 like the reference's torch.stft (data.py:205-221): four radix-4
// decimation-in-frequency stages, each lane one butterfly of 4 points held in registers, the wave
// exchanging points between stages through its own 2 KiB LDS buffer (no block barrier: a wave's LDS
// operations complete in order).  The exchange address p ^ ((p >> 2) & 31) keeps every stage's
// ds_write_b64 / ds_read_b64 free of bank conflicts.  A lane's window values and twiddles are the
// same for every frame and stay in registers.  Power and the mel projection are float32 like the
// reference.  Frames past an utterance's length are written as zeros.  The constant tables
// (per-filter nonzero weights, window, twiddles rounded once from double) are built on the host.
#include <assert.h>
#include <math.h>

#include <type_traits>
#include <vector>

#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

namespace {
constexpr int NFFT = 512, HOP = 160, WIN = 400, LPAD = (NFFT - WIN) / 2, NBIN = NFFT / 2 + 1;
constexpr int NC = NFFT / 2;  // complex FFT size
constexpr int FE_WAVES = 4;   // waves (frames in flight) per block
constexpr int FE_FPW = 8;     // consecutive frames per wave
constexpr int FE_W0 = 10, FE_W1 = 17;  // widest of mel filters 0..63 / 64..79 (build_frontend_const checks)
#ifndef FQ_FPQ
#define FQ_FPQ 4  // frames per quad (log_mel_q16_kernel)
#endif

// torch's elementwise steps, each rounded (no FMA contraction: hipcc's default would fuse them):
// pre-emphasis x[t+1] - 0.97 x[t] (data.py:201-202), the window product (|X|^2: split_power)
CASR_DEV float preemph_win(float w, float x1, float x0, float pre) {
#pragma clang fp contract(off)
  return w * (x1 - pre * x0);
}

// exchange slot of FFT position p (conflict-free for the four stage patterns)
CASR_DEV int fe_slot(int p) { return p ^ ((p >> 2) & 31); }
// base-4 digit reversal of an 8-bit index: after the four DIF stages X[k] sits at position rev4(k)
CASR_DEV int rev4(int k) {
  return ((k & 3) << 6) | (((k >> 2) & 3) << 4) | (((k >> 4) & 3) << 2) | ((k >> 6) & 3);
}
// complex product with its contraction written out (both log-mel kernels: the same bits whatever
// code surrounds it; hipcc's default contraction of a.x w.x - a.y w.y depends on the context)
CASR_DEV float2 cmul(float2 a, float2 w) {
#pragma clang fp contract(off)
  const float p = a.y * w.y, q = a.y * w.x;
  return make_float2(fmaf(a.x, w.x, -p), fmaf(a.x, w.y, q));
}

// the real-input split of bin q and its power: X[q] = E + W512^q O, E = (Z[q] + conj Z[-q]) / 2,
// O = (Z[q] - conj Z[-q]) / 2i, P = |X[q]|^2 (data.py:220-221), contraction written out
CASR_DEV float split_power(float2 z1, float2 z2, float2 tq) {
#pragma clang fp contract(off)
  const float er = 0.5f * (z1.x + z2.x), ei = 0.5f * (z1.y - z2.y);
  const float orr = 0.5f * (z1.y + z2.y), oi = -0.5f * (z1.x - z2.x);
  const float xr = er + fmaf(orr, tq.x, -(oi * tq.y));
  const float xi = ei + fmaf(orr, tq.y, oi * tq.x);
  return xr * xr + xi * xi;
}

// one radix-4 DIF butterfly: y_q = sum_r a_r (-i)^(rq), then y_q *= w_q (q = 1..3)
CASR_DEV void bfly4(float2 (&a)[4], const float2 (&w)[3], bool twiddle) {
  const float2 t0 = make_float2(a[0].x + a[2].x, a[0].y + a[2].y), t1 = make_float2(a[0].x - a[2].x, a[0].y - a[2].y);
  const float2 t2 = make_float2(a[1].x + a[3].x, a[1].y + a[3].y), t3 = make_float2(a[1].x - a[3].x, a[1].y - a[3].y);
  a[0] = make_float2(t0.x + t2.x, t0.y + t2.y);
  const float2 y2 = make_float2(t0.x - t2.x, t0.y - t2.y);
  const float2 y1 = make_float2(t1.x + t3.y, t1.y - t3.x);  // t1 - i t3
  const float2 y3 = make_float2(t1.x - t3.y, t1.y + t3.x);  // t1 + i t3
  a[1] = twiddle ? cmul(y1, w[0]) : y1;
  a[2] = twiddle ? cmul(y2, w[1]) : y2;
  a[3] = twiddle ? cmul(y3, w[2]) : y3;
}

CASR_DEV void lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// FPW frames per wave.  A lane's mel-filter weights (filters lane and lane + 64) are read from LDS
// once into registers for all its frames: 7 % faster than an LDS read per weight and frame at the
// same bits (tools/probes/logmel_variants.hip, profiles/r04/logmel/variants_r04g.txt)
template <int FPW = FE_FPW>
__global__ __launch_bounds__(256) void log_mel_kernel(const float* __restrict__ wav,
                                                      const int32_t* __restrict__ nsamp, int Nmax,
                                                      int Tmax, float pre, const FrontendConst* __restrict__ k,
                                                      float* __restrict__ out, int32_t* __restrict__ frames,
                                                      int32_t* __restrict__ err) {
  __shared__ float2 zs[FE_WAVES][NC];
  __shared__ float pw[FE_WAVES][NBIN + 3];
  __shared__ float fbs[F][FE_FBW + 1];  // the filters' nonzero weights (+1: lanes m read conflict-free)
  __shared__ int lohi[2][F];
  __shared__ float2 t256[NC], t512s[NBIN];  // twiddles (read per frame with the stage's data: registers
                                           // for a fourth wave per SIMD)
  const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < F * FE_FBW; i += blockDim.x) fbs[i / FE_FBW][i % FE_FBW] = (&k->fb[0][0])[i];
  for (int i = threadIdx.x; i < NC; i += blockDim.x) t256[i] = make_float2(k->tw256r[i], k->tw256i[i]);
  for (int i = threadIdx.x; i < NBIN; i += blockDim.x) t512s[i] = make_float2(k->tw512r[i], k->tw512i[i]);
  for (int i = threadIdx.x; i < F; i += blockDim.x) {
    lohi[0][i] = k->lo[i];
    lohi[1][i] = k->hi[i];
  }
  __syncthreads();  // the only block barrier: the waves run their frames independently after it
  int n = nsamp[b];
  if (n < NFFT + 1 || n > Nmax) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, CASR_DEV_BAD_AUDIO);
    n = n > Nmax ? Nmax : n;
  }
  const int L = n - 1 >= NFFT ? 1 + (n - 1 - NFFT) / HOP : 0;  // frames of the pre-emphasised signal
  if (blockIdx.x == 0 && threadIdx.x == 0) frames[b] = L < Tmax ? L : Tmax;
  const int f0 = (blockIdx.x * FE_WAVES + w) * FPW;
  if (f0 >= Tmax) return;  // no block barrier below: the waves are independent
  // per-lane constants of every frame: window values of the lane's 8 samples, the twiddles of the
  // three twiddled stages (group offset j of the lane: lane, lane & 15, lane & 3), the split twiddles
  float wn[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * (lane + 64 * r) + e;
      wn[r][e] = (j >= LPAD && j < LPAD + WIN) ? k->win[j - LPAD] : 0.f;
    }
  // stage s's twiddles of this lane: W_{256 / step}^{j q} = W_256^{step j q}, j = lane & (63 >> 2s)
  auto twiddles = [&](int s, float2 (&tw)[3]) {
    const int j = lane & (63 >> (2 * s)), step = 1 << (2 * s);
#pragma unroll
    for (int q = 1; q <= 3; ++q) tw[q - 1] = t256[(step * j * q) & (NC - 1)];
  };
  // the samples of a frame: point m = lane + 64 r needs x[2m .. 2m + 2] (pre-emphasis reads the next
  // sample); loaded one frame ahead, so a frame's loads fly while the previous frame computes
  float xs[4][3];
  auto load_frame = [&](int f) {
    const bool live = f < L && f < Tmax;
    const float* x = wav + (size_t)b * Nmax + (size_t)(live ? f : 0) * HOP;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 2 * (lane + 64 * r);
      const bool in = live && j + 1 >= LPAD && j < LPAD + WIN;  // a window value of the pair is nonzero
#pragma unroll
      for (int e = 0; e < 3; ++e) xs[r][e] = in ? x[j + e] : 0.f;
    }
  };
  load_frame(f0);
  // this lane's weights of filters lane (pass 0) and lane + 64 (pass 1)
  float fw0[FE_W0], fw1[FE_W1];
#pragma unroll
  for (int i = 0; i < FE_W0; ++i) fw0[i] = fbs[lane][i];
#pragma unroll
  for (int i = 0; i < FE_W1; ++i) fw1[i] = lane + 64 < F ? fbs[lane + 64][i] : 0.f;
  for (int fi = 0; fi < FPW; ++fi) {
    const int f = f0 + fi;
    if (f >= Tmax) break;
    float* o = out + ((size_t)b * Tmax + f) * F;
    if (f >= L) {  // padding rows past the utterance (wave-uniform)
      for (int m = lane; m < F; m += 64) o[m] = 0.f;
      continue;
    }
    float2 a[4];
    // windowed, pre-emphasised frame: point m = lane + 64 r is (y[2m] w, y[2m+1] w)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      a[r] = make_float2(preemph_win(wn[r][0], xs[r][1], xs[r][0], pre), preemph_win(wn[r][1], xs[r][2], xs[r][1], pre));
    if (fi + 1 < FPW) load_frame(f + 1);
    // stage 0 (S = 64): the lane's points are its butterfly
    float2 tw[3];
    twiddles(0, tw);
    bfly4(a, tw, true);
#pragma unroll
    for (int q = 0; q < 4; ++q) zs[w][fe_slot(lane + 64 * q)] = a[q];
    lds_fence();
    // stage 1 (S = 16): group lane >> 4, offset lane & 15
    {
      const int base = 64 * (lane >> 4) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = zs[w][fe_slot(base + 16 * r)];
      twiddles(1, tw);
      bfly4(a, tw, true);
#pragma unroll
      for (int q = 0; q < 4; ++q) zs[w][fe_slot(base + 16 * q)] = a[q];
    }
    lds_fence();
    {  // stage 2 (S = 4): group lane >> 2, offset lane & 3
      const int base = 16 * (lane >> 2) + (lane & 3);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = zs[w][fe_slot(base + 4 * r)];
      twiddles(2, tw);
      bfly4(a, tw, true);
#pragma unroll
      for (int q = 0; q < 4; ++q) zs[w][fe_slot(base + 4 * q)] = a[q];
    }
    lds_fence();
    {  // stage 3 (S = 1): group lane, no twiddle
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = zs[w][fe_slot(4 * lane + r)];
      bfly4(a, tw, false);
#pragma unroll
      for (int q = 0; q < 4; ++q) zs[w][fe_slot(4 * lane + q)] = a[q];
    }
    lds_fence();
    // real-input split: X[q] = E + W512^q O, E = (Z[q] + conj Z[-q]) / 2, O = (Z[q] - conj Z[-q]) / 2i
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int q = lane + 64 * r;
      if (q < NBIN) {
        const float2 z1 = zs[w][fe_slot(rev4(q & (NC - 1)))], z2 = zs[w][fe_slot(rev4((NC - q) & (NC - 1)))];
        pw[w][q] = split_power(z1, z2, t512s[q]);
      }
    }
    lds_fence();
    // mel projection (a float32 fma chain over the filter's nonzero bins, in bin order) and log.
    // Fixed trip counts, every LDS read of a pass issued before its fma chain: pass 0 = filters
    // 0..63 (at most FE_W0 bins), pass 1 = filters 64..79 on lanes 0..15 (at most FE_W1 bins).  The
    // weights past a filter's last bin are zero (fma(x, 0, acc) = acc for the finite powers; a
    // non-finite power makes the sum NaN, as the reference's full-length matmul does)
    auto mel = [&](auto NW, int m, const float* wreg) {  // (the weights from registers, in bin order)
      constexpr int W = decltype(NW)::value;
      const int lo = lohi[0][m];
      float pv[W], wv[W];
#pragma unroll
      for (int i = 0; i < W; ++i) {
        pv[i] = pw[w][min(lo + i, NBIN - 1)];
        wv[i] = wreg[i];
      }
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < W; ++i) acc = fmaf(pv[i], wv[i], acc);  // matmul: fused
      o[m] = logf(acc == 0.f ? 1.1920928955078125e-07f : acc);
    };
    mel(std::integral_constant<int, FE_W0>{}, lane, fw0);
    if (lane + 64 < F) mel(std::integral_constant<int, FE_W1>{}, lane + 64, fw1);
    lds_fence();  // this frame's pw / zs reads are done before the next frame's writes
  }
}

// ---- the 16-lane form (round 5, the default): 16 lanes per frame, 16 points per lane, 4 frames per
// wave in flight.  With lane l holding the points m = l + 16 r (r = 0..15), the butterflies of
// radix-4 DIF stages 0 (stride 64) and 1 (stride 16) are all within the lane; one transpose through
// LDS gives lane l the points 16 l + i, and stages 2 (stride 4) and 3 (stride 1) are again within the
// lane.  So a frame is one stage exchange instead of three (log_mel_kernel: six dependent LDS round
// trips per frame), with the same butterflies, twiddles and operation order: the same bits as
// log_mel_kernel (tests/test_gpu_frontend.py).  Exchange slot p ^ ((p >> 4) & 15): the transpose's
// writes (p = l + 16 r) and reads (p = 16 l + i) of a quad are conflict-free; quads are 128 B apart.
// Lane l's constants for every frame: the stage-0 and stage-1 twiddles and the weights of its mel
// filters l + 16 i (i < 4: filters 0..63, at most FE_W0 bins; i = 4: 64..79, at most FE_W1).
constexpr int FQ_Q = 8;   // frames in flight per block: 2 waves x 4 quads of 16 lanes
constexpr int FQ_ZS = NC + 16;  // float2 per quad's exchange buffer (+128 B: quads apart in the banks)
CASR_DEV int fq_slot(int p) { return p ^ ((p >> 4) & 15); }

template <int FPQ>
__global__ __launch_bounds__(64 * FQ_Q / 4) void log_mel_q16_kernel(const float* __restrict__ wav,
                                                                    const int32_t* __restrict__ nsamp, int Nmax,
                                                                    int Tmax, float pre,
                                                                    const FrontendConst* __restrict__ k,
                                                                    float* __restrict__ out,
                                                                    int32_t* __restrict__ frames,
                                                                    int32_t* __restrict__ err) {
  __shared__ float2 zs[FQ_Q][FQ_ZS];
  __shared__ float pw[FQ_Q][NBIN + 3];
  __shared__ float2 wins[NC];  // (w[2m], w[2m + 1]) of point m
  __shared__ float2 t256[NC], t512s[NBIN];
  __shared__ float fbs[F][FE_W1 + 1];  // the filters' weights (+1: the 16 lanes' rows in distinct banks)
  __shared__ int lohi[F];
  const int b = blockIdx.y, tid = threadIdx.x, qd = tid >> 4, l = tid & 15;
  for (int i = tid; i < NC; i += blockDim.x) {
    t256[i] = make_float2(k->tw256r[i], k->tw256i[i]);
    const int j0 = 2 * i - LPAD, j1 = j0 + 1;
    wins[i] = make_float2(j0 >= 0 && j0 < WIN ? k->win[j0] : 0.f, j1 >= 0 && j1 < WIN ? k->win[j1] : 0.f);
  }
  for (int i = tid; i < NBIN; i += blockDim.x) t512s[i] = make_float2(k->tw512r[i], k->tw512i[i]);
  for (int i = tid; i < F * FE_W1; i += blockDim.x) fbs[i / FE_W1][i % FE_W1] = k->fb[i / FE_W1][i % FE_W1];
  for (int i = tid; i < F; i += blockDim.x) lohi[i] = k->lo[i];
  __syncthreads();  // the only block barrier: the quads run their frames independently after it
  int n = nsamp[b];
  if (n < NFFT + 1 || n > Nmax) {
    if (blockIdx.x == 0 && tid == 0) atomicOr(err, CASR_DEV_BAD_AUDIO);
    n = n > Nmax ? Nmax : n;
  }
  const int L = n - 1 >= NFFT ? 1 + (n - 1 - NFFT) / HOP : 0;  // frames of the pre-emphasised signal
  if (blockIdx.x == 0 && tid == 0) frames[b] = L < Tmax ? L : Tmax;
  const int f0 = (blockIdx.x * FQ_Q + qd) * FPQ;
  float2* z = zs[qd];
  float* p = pw[qd];
  // the samples of a frame: point m = l + 16 r needs x[2m .. 2m + 2] (x[512] at most: inside the
  // signal for every frame f < L); loaded one frame ahead, so a frame's loads fly while the previous
  // frame computes.  All points are loaded, from one lane pointer with immediate offsets: the window
  // zeroes the ones outside it, as the reference's full-frame product does
  float xs[16][3];
  auto load_frame = [&](int f) {
    const bool live = f < L && f < Tmax;
    const float* x = wav + (size_t)b * Nmax + (size_t)(live ? f : 0) * HOP + 2 * l;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int e = 0; e < 3; ++e) xs[r][e] = x[32 * r + e];
  };
  load_frame(f0);
  for (int fi = 0; fi < FPQ; ++fi) {
    const int f = f0 + fi;
    if (f >= Tmax) break;
    float* o = out + ((size_t)b * Tmax + f) * F;
    if (f >= L) {  // padding rows past the utterance (quad-uniform)
#pragma unroll
      for (int i = 0; i < 5; ++i) o[l + 16 * i] = 0.f;
      continue;
    }
    float2 a[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {  // point m = l + 16 r: (y[2m] w[2m], y[2m+1] w[2m+1])
      const float2 wv = wins[l + 16 * r];
      a[r] = make_float2(preemph_win(wv.x, xs[r][1], xs[r][0], pre), preemph_win(wv.y, xs[r][2], xs[r][1], pre));
    }
    if (fi + 1 < FPQ) load_frame(f + 1);
    // stage 0 (stride 64): group r' = points l + 16 r' + 64 q = a[r' + 4 q], twiddle j = l + 16 r'
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float2 tw[3];
#pragma unroll
      for (int q = 1; q <= 3; ++q) tw[q - 1] = t256[((l + 16 * r) * q) & (NC - 1)];
      float2 g[4] = {a[r], a[r + 4], a[r + 8], a[r + 12]};
      bfly4(g, tw, true);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[r + 4 * q] = g[q];
    }
    // stage 1 (stride 16): group g = points 64 g + l + 16 q = a[4 g + q], twiddle j = l
    {
      float2 tw[3];
#pragma unroll
      for (int q = 1; q <= 3; ++q) tw[q - 1] = t256[(4 * l * q) & (NC - 1)];
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        float2 g[4] = {a[4 * gi], a[4 * gi + 1], a[4 * gi + 2], a[4 * gi + 3]};
        bfly4(g, tw, true);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[4 * gi + q] = g[q];
      }
    }
    // the transpose: lane l takes the points 16 l + i
#pragma unroll
    for (int r = 0; r < 16; ++r) z[fq_slot(l + 16 * r)] = a[r];
    lds_fence();
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = z[fq_slot(16 * l + i)];
    // stage 2 (stride 4): group o = points 16 l + o + 4 q = a[o + 4 q], twiddle j = o
#pragma unroll
    for (int oo = 0; oo < 4; ++oo) {
      float2 tw[3];
#pragma unroll
      for (int q = 1; q <= 3; ++q) tw[q - 1] = t256[(16 * oo * q) & (NC - 1)];
      float2 g[4] = {a[oo], a[oo + 4], a[oo + 8], a[oo + 12]};
      bfly4(g, tw, true);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[oo + 4 * q] = g[q];
    }
    // stage 3 (stride 1): group = points 16 l + 4 gi + q = a[4 gi + q], no twiddle
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      float2 g[4] = {a[4 * gi], a[4 * gi + 1], a[4 * gi + 2], a[4 * gi + 3]};
      const float2 tw[3] = {};
      bfly4(g, tw, false);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[4 * gi + q] = g[q];
    }
    lds_fence();  // the transpose's reads are done before the spectrum overwrites the buffer
    // Z[k] sits at position rev4(k) = 16 l + i
#pragma unroll
    for (int i = 0; i < 16; ++i) z[fq_slot(16 * l + i)] = a[i];
    lds_fence();
#pragma unroll
    for (int i = 0; i < 17; ++i) {  // bins q = l + 16 i (and 256 on lane 0)
      const int q = l + 16 * i;
      if (q < NBIN) p[q] = split_power(z[fq_slot(rev4(q & (NC - 1)))], z[fq_slot(rev4((NC - q) & (NC - 1)))], t512s[q]);
    }
    lds_fence();
    // mel projection: a float32 fma chain over the filter's bins in bin order (fixed trip counts,
    // zero weights past its last bin), then log with the FLT_EPSILON floor (data.py:222-224)
    auto mel = [&](auto NW, int m) {
      constexpr int W = decltype(NW)::value;
      const int lo = lohi[m];
      float pv[W], wv[W];
#pragma unroll
      for (int i = 0; i < W; ++i) {
        pv[i] = p[min(lo + i, NBIN - 1)];
        wv[i] = fbs[m][i];
      }
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < W; ++i) acc = fmaf(pv[i], wv[i], acc);  // matmul: fused
      o[m] = logf(acc == 0.f ? 1.1920928955078125e-07f : acc);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) mel(std::integral_constant<int, FE_W0>{}, l + 16 * i);
    mel(std::integral_constant<int, FE_W1>{}, 64 + l);
    lds_fence();  // this frame's pw / z reads are done before the next frame's writes
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
  std::vector<float> fb(NBIN * F);
  mel_filterbank(NBIN, 80.f, 7600.f, F, fb.data());
  *c = FrontendConst{};
  for (int m = 0; m < F; ++m) {
    int lo = NBIN, hi = 0;
    for (int q = 0; q < NBIN; ++q)
      if (fb[q * F + m] != 0.f) {
        lo = q < lo ? q : lo;
        hi = q + 1;
      }
    if (lo >= hi) lo = hi = 0;
    // the kernel's fixed trip counts (FE_W0 / FE_W1 bins): not exceeded by this filterbank (widest 10 /
    // 17); a wider filter would be truncated, so fail loudly in a debug build
    const int wmax = m < 64 ? FE_W0 : FE_W1;
    assert(hi - lo <= wmax);
    if (hi - lo > wmax) hi = lo + wmax;
    c->lo[m] = lo;
    c->hi[m] = hi;
    for (int q = lo; q < hi; ++q) c->fb[m][q - lo] = fb[q * F + m];
  }
  // torch.hann_window(400) (periodic): 0.5 - 0.5 cos(2 pi j / 400), evaluated in float32
  for (int j = 0; j < WIN; ++j) c->win[j] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * j / WIN));
  for (int i = 0; i < NC; ++i) {
    c->tw256r[i] = (float)cos(-2.0 * M_PI * i / NC);
    c->tw256i[i] = (float)sin(-2.0 * M_PI * i / NC);
  }
  for (int q = 0; q < NBIN; ++q) {
    c->tw512r[q] = (float)cos(-2.0 * M_PI * q / NFFT);
    c->tw512i[q] = (float)sin(-2.0 * M_PI * q / NFFT);
  }
}

int frontend_frames(int n_samples) {
  return n_samples - 1 >= NFFT ? 1 + (n_samples - 1 - NFFT) / HOP : 0;
}

hipError_t launch_log_mel(const float* wav, const int32_t* nsamp, int B, int Nmax, int Tmax, float pre,
                          const FrontendConst* k, float* out, int32_t* frames, int32_t* err, hipStream_t s,
                          int form) {
  if (form == 0) {  // the one-wave-per-frame form (round 4), kept for comparison: the same bits
    constexpr int FPB = FE_WAVES * FE_FPW;  // frames per block
    dim3 grid((Tmax + FPB - 1) / FPB > 0 ? (Tmax + FPB - 1) / FPB : 1, B);
    hipLaunchKernelGGL(log_mel_kernel<>, grid, dim3(256), 0, s, wav, nsamp, Nmax, Tmax, pre, k, out, frames, err);
  } else {
    constexpr int FPB = FQ_Q * FQ_FPQ;
    dim3 grid((Tmax + FPB - 1) / FPB > 0 ? (Tmax + FPB - 1) / FPB : 1, B);
    hipLaunchKernelGGL(log_mel_q16_kernel<FQ_FPQ>, grid, dim3(16 * FQ_Q), 0, s, wav, nsamp, Nmax, Tmax, pre, k, out,
                       frames, err);
  }
  return hipGetLastError();
}

}  // namespace casr
