// Shared device helpers for the gfx950 kernels of casr (CDNA4: wave64, MFMA f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CASR_DEV __device__ __forceinline__

// v_mfma_f32_16x16x4_f32: exact f32 (k-ordered fmaf chain).  Lane l supplies
// A[l&15][k=l>>4] and B[k=l>>4][l&15]; C/D: col = l&15, row = 4*(l>>4) + reg.
CASR_DEV f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- split-f16 ("s16x3") fp32 contraction on the f16 MFMA pipes (2.5 PF dense vs 157 TF f32).
// x = hi + 2^-11 lo with hi = f16_rn(x) and lo = f16_rn((x - hi) * 2^11): x - hi is exact in
// f32 and the 2^11 scale keeps lo a normal f16, so hi:lo carries 22 significant bits.
//   a.b = hi_a.hi_b + 2^-11 (hi_a.lo_b + lo_a.hi_b)   (+ the dropped 2^-22 lo.lo term)
// with every f16 x f16 product exact and accumulated in f32 by v_mfma_f32_16x16x32_f16.
// Measured on MI355X (tools/probes/split16_probe.hip, error / sum|a_k b_k| vs fp64): 8.8e-8 max,
// against 2.6e-7 for the exact-f32 MFMA k-ordered chain on the same operands.  Operands must
// stay below 65504 in magnitude (f16 range); the host rejects weights beyond 2^14.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr float S16_LO_SCALE = 2048.0f;
constexpr float S16_LO_INV = 1.0f / 2048.0f;

// v_mfma_f32_16x16x32_f16: lane l supplies A[l&15][k = 8(l>>4) + e] and B[k][l&15] for e = 0..7;
// C/D as mfma16x16x4.
CASR_DEV f32x4 mfma16x16x32h(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// hi / lo halves of one f32 packed as (hi | lo << 16); a non-finite x keeps hi = f16(x) and
// lo = 0 so bit 30 (lo's exponent MSB, 0 whenever |lo| < 2) stays free for hand-off tags
CASR_DEV uint32_t split16_word(float x) {
  const _Float16 hi = (_Float16)x;
  const float r = (x - (float)hi) * S16_LO_SCALE;
  const _Float16 lo = (r == r && fabsf(r) < 65504.f) ? (_Float16)r : (_Float16)0.f;
  return (uint32_t)__builtin_bit_cast(uint16_t, hi) | ((uint32_t)__builtin_bit_cast(uint16_t, lo) << 16);
}

// 8 split words (two u32x4) -> the 8-wide hi and lo MFMA operands
CASR_DEV void unpack16(u32x4 w0, u32x4 w1, f16x8& hi, f16x8& lo) {
  u32x4 h, l;
  h.x = __builtin_amdgcn_perm(w0.y, w0.x, 0x05040100u);
  h.y = __builtin_amdgcn_perm(w0.w, w0.z, 0x05040100u);
  h.z = __builtin_amdgcn_perm(w1.y, w1.x, 0x05040100u);
  h.w = __builtin_amdgcn_perm(w1.w, w1.z, 0x05040100u);
  l.x = __builtin_amdgcn_perm(w0.y, w0.x, 0x07060302u);
  l.y = __builtin_amdgcn_perm(w0.w, w0.z, 0x07060302u);
  l.z = __builtin_amdgcn_perm(w1.y, w1.x, 0x07060302u);
  l.w = __builtin_amdgcn_perm(w1.w, w1.z, 0x07060302u);
  hi = __builtin_bit_cast(f16x8, h);
  lo = __builtin_bit_cast(f16x8, l);
}

// unpack16 of hand-off words whose bit 30 (lo's exponent MSB) carries a tag: cleared here
CASR_DEV void unpack16_tagged(u32x4 w0, u32x4 w1, f16x8& hi, f16x8& lo) {
  unpack16(w0, w1, hi, lo);
  u32x4 l = __builtin_bit_cast(u32x4, lo);
  l &= 0xBFFFBFFFu;
  lo = __builtin_bit_cast(f16x8, l);
}

// CASR_S16_ONE = 1 is the s16x1 build (libcasr_hip_s16x1.so, casr/build.py; round 6, BASELINE
// config 2's opt-in perf arithmetic, CASR_PREC_S16X1): every split product keeps its hi.hi MFMA
// only, the two cross-term MFMAs of each site are compiled out (11 significant operand bits
// instead of 22; the same images, bytes and code otherwise).  The shipped library is built
// without it.
#ifndef CASR_S16_ONE
#define CASR_S16_ONE 0
#endif
constexpr bool kS16Cross = !CASR_S16_ONE;

// three MFMAs of one s16x3 product into the (hi.hi, cross) accumulator pair (s16x1: the first)
CASR_DEV void mfma_s16(f16x8 ah, f16x8 al, f16x8 bh, f16x8 bl, f32x4& hh, f32x4& x) {
  hh = mfma16x16x32h(ah, bh, hh);
  if constexpr (kS16Cross) {
    x = mfma16x16x32h(ah, bl, x);
    x = mfma16x16x32h(al, bh, x);
  }
}

CASR_DEV float s16_combine(float hh, float x) { return hh + x * S16_LO_INV; }

// global_load_lds_dwordx4 in inline asm: hipcc does not see these DMAs, so it inserts no wait of
// its own for them (seen, every ds_read of the ring waited vmcnt(0): the DMAs carry no alias
// scope); the kernel orders them itself with counted vmcnt waits + s_barrier.  M0 = the wave's
// LDS destination base (lane l writes base + 16 l), saved and restored around the load.
CASR_DEV void lds_dma16(const float* src, float* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds_wave_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

// the same DMA from a scalar base + per-lane 32-bit byte offset (global_load_lds_dwordx4 v, s[]),
// M0 = the wave's LDS destination byte address (a 32-bit LDS offset computed by the caller)
CASR_DEV void lds_dma16_s(uint32_t voff, const float* sbase, uint32_t lds_byte) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory");
}

CASR_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Accurate variants used on every parity-relevant path (torch CPU uses libm-accurate
// expf/tanhf; the fast __expf differs by a few ulp, so it is not used for gates).
CASR_DEV float sigmoid_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---- wave reductions on DPP lane moves (no LDS round trip; __shfl_xor lowers to ds_bpermute /
// ds_swizzle, ~100+ cycles per dependent step).  Within each 16-lane row: quad_perm xor 1, xor 2,
// then row_ror 4 and 8; across the 4 rows: v_readlane of lanes 0, 16, 32, 48 combined in a fixed
// order, so every lane gets the same value (sums: row sums are read from each row's lane 0, so
// the result does not depend on which lane computes it).  All 64 lanes must be active.
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;
template <int CTRL>
CASR_DEV int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
CASR_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
}
CASR_DEV float readlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// every lane of each 16-lane row: that row's maximum / minimum / sum (sum: as computed in the
// row's first quad)
CASR_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  v = fmaxf(v, dpp_f<DPP_XOR2>(v));
  v = fmaxf(v, dpp_f<DPP_ROR4>(v));
  return fmaxf(v, dpp_f<DPP_ROR8>(v));
}
CASR_DEV int row16_min(int v) {
  v = min(v, dpp_i<DPP_XOR1>(v));
  v = min(v, dpp_i<DPP_XOR2>(v));
  v = min(v, dpp_i<DPP_ROR4>(v));
  return min(v, dpp_i<DPP_ROR8>(v));
}
CASR_DEV float row16_sum(float v) {
  v += dpp_f<DPP_XOR1>(v);
  v += dpp_f<DPP_XOR2>(v);
  v += dpp_f<DPP_ROR4>(v);
  return v + dpp_f<DPP_ROR8>(v);
}
CASR_DEV int row16_isum(int v) {
  v += dpp_i<DPP_XOR1>(v);
  v += dpp_i<DPP_XOR2>(v);
  v += dpp_i<DPP_ROR4>(v);
  return v + dpp_i<DPP_ROR8>(v);
}

// exp(2x) for the attention's split exponential score form (attention.hip): v_exp_f32 of
// x * 2 log2(e) while |x| < 43 (a finite normal float), NaN beyond (the block then falls back to
// the direct tanh(k + q) form)
CASR_DEV float split_exp2x(float x) {
  return fabsf(x) < 43.f ? __builtin_amdgcn_exp2f(x * 2.8853900817779268f) : __builtin_nanf("");
}

CASR_DEV float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

CASR_DEV float wave_sum(float v) {
  v = row16_sum(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}

CASR_DEV int wave_min_i(int v) {
  v = row16_min(v);
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// (largest value, lowest index among lanes holding it) in every lane: the `better` order of
// the selects (greater value; on equal values the lower index)
CASR_DEV void wave_best(float& v, int& i) {
  const float m = wave_max(v);
  i = wave_min_i(v == m ? i : 0x7fffffff);
  v = m;
}

// Decode early exit (model.py:578, :897-901): newdone[s] counts rows / utterances that
// finished at step s; step l runs only while fewer than `total` finished before it.
// rows finished before decode step l (the per-step counters of steps 0..l-1): one wave-wide
// load per 64 steps and a DPP reduction, not l dependent loads
CASR_DEV int done_before(const int32_t* __restrict__ newdone, int l) {
  const int lane = threadIdx.x & 63;
  int s = 0;
  for (int i0 = 0; i0 < l; i0 += 64) s += (i0 + lane < l) ? newdone[i0 + lane] : 0;
  s = row16_isum(s);
  return (__builtin_amdgcn_readlane(s, 0) + __builtin_amdgcn_readlane(s, 16)) +
         (__builtin_amdgcn_readlane(s, 32) + __builtin_amdgcn_readlane(s, 48));
}

// done_before2 for at most 64 steps in two halves: the counters' load (lane i: step i) and its
// reduction, so a caller can issue other loads in between without its wait for the counters waiting
// for them too (a wave's loads retire in issue order)
CASR_DEV int done_load(const int32_t* __restrict__ newdone, int lm) {
  const int lane = threadIdx.x & 63;
  return lane < lm ? newdone[lane] : 0;
}
CASR_DEV void done_reduce(int v, int l1, int l2, int& d1, int& d2) {
  const int lane = threadIdx.x & 63;
  int s1 = lane < l1 ? v : 0, s2 = lane < l2 ? v : 0;
  s1 = row16_isum(s1);
  s2 = row16_isum(s2);
  d1 = (__builtin_amdgcn_readlane(s1, 0) + __builtin_amdgcn_readlane(s1, 16)) +
       (__builtin_amdgcn_readlane(s1, 32) + __builtin_amdgcn_readlane(s1, 48));
  d2 = (__builtin_amdgcn_readlane(s2, 0) + __builtin_amdgcn_readlane(s2, 16)) +
       (__builtin_amdgcn_readlane(s2, 32) + __builtin_amdgcn_readlane(s2, 48));
}

// rows finished before steps l1 and l2 from one pass of loads over the counters
CASR_DEV void done_before2(const int32_t* __restrict__ newdone, int l1, int l2, int& d1, int& d2) {
  const int lane = threadIdx.x & 63, lm = max(l1, l2);
  int s1 = 0, s2 = 0;
  for (int i0 = 0; i0 < lm; i0 += 64) {
    const int i = i0 + lane;
    const int v = i < lm ? newdone[i] : 0;
    s1 += i < l1 ? v : 0;
    s2 += i < l2 ? v : 0;
  }
  s1 = row16_isum(s1);
  s2 = row16_isum(s2);
  d1 = (__builtin_amdgcn_readlane(s1, 0) + __builtin_amdgcn_readlane(s1, 16)) +
       (__builtin_amdgcn_readlane(s1, 32) + __builtin_amdgcn_readlane(s1, 48));
  d2 = (__builtin_amdgcn_readlane(s2, 0) + __builtin_amdgcn_readlane(s2, 16)) +
       (__builtin_amdgcn_readlane(s2, 32) + __builtin_amdgcn_readlane(s2, 48));
}

// Hardware-exp forms (v_exp_f32 / v_rcp_f32, no IEEE division: __frcp_rn / __fdividef / 1.f / x
// compile to a div_scale / div_fmas / div_fixup sequence of ~10 dependent instructions, and this
// cell sits on the recurrence's critical path).  exp(y) = exp2(y log2 e) with the product rounded
// once: relative error ~|y| 6e-8, which the sigmoid's slope damps (absolute error <~1e-8); v_rcp_f32
// is within 1 ulp.  tanh = sign(x) (1 - e) / (1 + e), e = exp(-2|x|): absolute error ~2e-7.  Used by
// the encoder cell in s16x3 arithmetic (the f32 arithmetic keeps the libm cell below).
CASR_DEV float sigmoid_hw(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
CASR_DEV float tanh_hw(float x) {
  const float e = __builtin_amdgcn_exp2f(fabsf(x) * -2.8853900817779268f);
  return copysignf((1.f - e) * __builtin_amdgcn_rcpf(1.f + e), x);
}
CASR_DEV void lstm_cell_hw(float gi, float gf, float gg, float go, float c, float& h2, float& c2) {
#pragma clang fp contract(off)  // lexical: __fmul_rn / __fadd_rn are plain * / + in their own (contracting) bodies
  const float i = sigmoid_hw(gi), f = sigmoid_hw(gf), g = tanh_hw(gg), o = sigmoid_hw(go);
  c2 = f * c + i * g;  // two rounded products and a rounded add (contract off above)
  h2 = o * tanh_hw(c2);
}

// residual add x + y of RNN_RES (util.py:1289), never fused with the cell's o * tanh(c') product
CASR_DEV float residual_add(float y, float x) {
#pragma clang fp contract(off)
  return y + x;
}

// LSTM cell with PyTorch gate order (i, f, g, o): c' = f*c + i*g, h' = o*tanh(c').
CASR_DEV void lstm_cell(float gi, float gf, float gg, float go, float c, float& h2, float& c2) {
#pragma clang fp contract(off)  // lexical: __fmul_rn / __fadd_rn are plain * / + in their own (contracting) bodies
  const float i = sigmoid_acc(gi);
  const float f = sigmoid_acc(gf);
  const float g = tanhf(gg);
  const float o = sigmoid_acc(go);
  // no FMA contraction: torch evaluates (f * c) + (i * g) and o * tanh(c') as separate ops
  c2 = f * c + i * g;
  h2 = o * tanhf(c2);
}
