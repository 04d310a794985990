// Shared device helpers for the gfx950 kernels of casr (CDNA4: wave64, MFMA f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CASR_DEV __device__ __forceinline__

// v_mfma_f32_16x16x4_f32: exact f32 (k-ordered fmaf chain).  Lane l supplies
// A[l&15][k=l>>4] and B[k=l>>4][l&15]; C/D: col = l&15, row = 4*(l>>4) + reg.
CASR_DEV f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

CASR_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Accurate variants used on every parity-relevant path (torch CPU uses libm-accurate
// expf/tanhf; the fast __expf differs by a few ulp, so it is not used for gates).
CASR_DEV float sigmoid_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

// Decode early exit (model.py:578, :897-901): newdone[s] counts rows / utterances that
// finished at step s; step l runs only while fewer than `total` finished before it.
CASR_DEV int done_before(const int32_t* __restrict__ newdone, int l) {
  int s = 0;
  for (int i = 0; i < l; ++i) s += newdone[i];
  return s;
}

CASR_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

CASR_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LSTM cell with PyTorch gate order (i, f, g, o): c' = f*c + i*g, h' = o*tanh(c').
CASR_DEV void lstm_cell(float gi, float gf, float gg, float go, float c, float& h2, float& c2) {
  const float i = sigmoid_acc(gi);
  const float f = sigmoid_acc(gf);
  const float g = tanhf(gg);
  const float o = sigmoid_acc(go);
  // no FMA contraction: torch evaluates (f * c) + (i * g) and o * tanh(c') as separate ops
  c2 = __fadd_rn(__fmul_rn(f, c), __fmul_rn(i, g));
  h2 = __fmul_rn(o, tanhf(c2));
}
