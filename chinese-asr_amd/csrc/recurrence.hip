// Persistent bidirectional-LSTM recurrence: one launch per encoder layer runs all Tp steps.
//
// Reference: RNN_RES.forward util.py:1223-1324 (one nn.LSTM(bidirectional) per layer over a
// packed batch, encoder.py:36-81), i.e. per direction d and step the gate pre-activations
//   g[b] = Gin[b, t] + W_hh[d] . h_{t-1}[b]        (Gin = x W_ih^T + b_ih + b_hh, encoder.hip)
// followed by the (i, f, g, o) cell.  The per-step launch (encoder.hip rec_step_kernel) pays a
// kernel boundary, a W_hh re-read and a c round trip every step; here each workgroup keeps its
// W_hh slice and its cells' c in registers for the whole layer and hands h to the other
// workgroups of its row group through tagged granules (MI355X_MICROARCH.md price list,
// handoff-1to1 / cdna_hip_programming.md Guideline 16 R2: the data is its own flag):
//
//   granule = ONE 4-byte word: the h bits with bit 30 replaced by the step-parity tag.  h =
//   o * tanh(c) has |h| <= 1, so bit 30 (the exponent MSB, set only for |x| >= 2) is always
//   0 in a finite h and is free to carry the tag; a non-finite h is sent as 0x3FFFFFFF (a
//   value in [1, 2) no LSTM output takes) and decoded back to NaN.  Producers store each word
//   write-through (sc1), or plain when its whole group shares its XCD (see the placement table
//   below); a consumer wave re-reads (sc1 loads, L1 bypassed) its 16 rows x 64
//   units until every tag matches: no counter, no fence, no barrier, 4 B per value.
//
// Geometry (gfx950, 256 CUs): workgroup (ub, rg, d) = 16 hidden units (64 gate rows, all four
// gates) x 32 batch rows of direction d; 512 threads = 8 waves, wave w owns k-chunk (w & 3) of
// the contraction for batch-row half (w >> 2).  16 x ceil(B/32) x 2 <= 256 workgroups at
// B <= 256, one per CU, all resident (checked by the host against the occupancy query).
// Every arithmetic step (per-wave MFMA order, 4-way k-chunk reduction order, cell) equals
// rec_step_kernel's, so both paths give bitwise identical results.
//
// Triple-buffered granules: a workgroup writing step s's h into buffer (s+1)%3 has, during step
// s-1, seen every group member's step s-2 output, hence every member finished reading buffer
// (s-2)%3 == (s+1)%3.  Successive writes of one buffer are 3 steps apart, so their parity tags
// differ and a 1-bit tag separates new from old; the initial fill gives each buffer the parity
// its first reader does NOT expect (reset_rec_layer).  Every cell writes its word every step
// (0 for inactive and padding rows) so no wait depends on lengths.  Spins are bounded (~2 s of
// s_memrealtime and a pass count); a timeout sets CASR_DEV_REC_TIMEOUT and the workgroup leaves
// the loop.
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

namespace {

constexpr int NKC = H / 64;            // 4 k-chunks of 64 hidden units
constexpr uint64_t SPIN_TICKS = 200000000ull;  // s_memrealtime runs at 100 MHz: 2 s

constexpr uint32_t TAG_BIT = 0x40000000u;
constexpr uint32_t NONFINITE = 0x3FFFFFFFu;

// S16: the granule is the s16 split word of h (casr_common.h split16_word: hi | lo << 16).  |h| <=
// 1 keeps |lo| < 2, so bit 30 (lo's exponent MSB) is free for the tag here too; a non-finite h
// travels as hi = f16(h) (NaN) with lo = 0.  The consumer masks the tag and feeds the halves to
// the f16 MFMAs directly.
template <bool S16>
CASR_DEV void store_granule(uint32_t* p, int step_tagged, float v, int plain) {
  uint32_t x;
  if constexpr (S16) {
    x = split16_word(v);
  } else {
    x = __float_as_uint(v);
    if (!(fabsf(v) < 2.0f)) x = NONFINITE;
  }
  x |= (step_tagged & 1) ? TAG_BIT : 0u;
  if (plain)
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // global_store_dword
  else
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store_dword sc1
}

CASR_DEV float decode_granule(uint32_t x) {
  x &= ~TAG_BIT;
  return (x & 0x7FFFFFFFu) == NONFINITE ? __uint_as_float(0x7FC00000u) : __uint_as_float(x);
}

// Workgroup = RG batch rows x UW hidden units (x 4 gates) of one direction; NW = 4 k-chunks x
// RG/16 row halves x UW/16 unit halves waves.  32 x 16 (default): 16 producers per row group;
// 16 x 32: 8 producers per row group (a consumer waits on fewer workgroups; the two unit-half
// waves of a k-chunk sweep the same words); 16 x 16: 4 waves, two workgroups per CU.
// S16: W_hh is the s16 fragment image (casr_capi.hip pack_frag16) and the contraction runs as
// s16x3 on v_mfma_f32_16x16x32_f16 (2 k-steps of 32 per 64-unit chunk, 24 MFMAs per wave and
// step instead of 64 f32 ones at twice the cycles each).  Lane (r, g) of k-step j covers units
// 16g + 8j + e of its chunk: exactly the granule words its sweep already loaded.
template <int RG, int UW, bool S16>
__global__ __launch_bounds__(RG * UW, 2) void rec_layer_kernel(
    const float* __restrict__ Whh_f, const float* __restrict__ Gin, const float* __restrict__ xin,
    float* __restrict__ out, uint16_t* __restrict__ x16, uint32_t* __restrict__ hx, float* __restrict__ hfin,
    float* __restrict__ cst, const int32_t* __restrict__ lens, int B, int Bp, int Tp, int residual,
    int32_t* __restrict__ err, uint32_t* __restrict__ trace, int nrg, int pre_sleep, int poll_gap,
    int store_plain, int km) {
  constexpr int NW = RG * UW / 64;      // waves: 4 k-chunks x RG/16 row halves x UW/16 unit halves
  __shared__ f32x4 red[2][NW][4][64];  // double-buffered k-chunk partials
  __shared__ int s_tmax, s_quit[2];  // quit flag per step parity (read after the step's barrier)
  // ---- placement (speed only, never correctness).  Workgroups are dealt round-robin over the 8
  // XCDs (MI355X_MICROARCH.md "Workgroup dispatch"), so ids L and L + 8 share one: the P members
  // of a hand-off group (the unit blocks of one row group and direction) take ids with equal L % 8
  // and exchange h inside one XCD.  Measured: 3.49 -> 3.07 us per step.
  constexpr int P = H / UW;  // producers per group
  const int G = 2 * nrg, L = blockIdx.x;
  int grp, mem;
  if (G % 8 == 0) {
    const int x = L & 7, j = L >> 3;
    grp = x * (G / 8) + j / P;
    mem = j % P;
  } else {
    grp = L / P;
    mem = L % P;
  }
  const int ub = mem, rg = grp % nrg, d = grp / nrg;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // waves w and w + 4 share a SIMD (a workgroup's waves are dealt to the 4 SIMDs cyclically): give
  // them different k-chunks, so their sweeps wait for different producers and their MFMA bursts
  // do not meet on one pipe (with kc = w & 3 both completed together, behind the same producers).
  // Measured: rec 2.62-2.72 -> 2.59-2.63 ms per greedy batch (three interleaved rounds), beam equal
  const int kc = (w + (w >> 2)) & 3, half = (w >> 2) % (RG / 16), uh = (w >> 2) / (RG / 16);
  const size_t plane = (size_t)Bp * H;  // granules per direction per buffer

  // ---- epilogue cell of this thread: batch row rl (of RG), unit u (of UW)
  const int rl = tid / UW, u = tid % UW;
  const int b = rg * RG + rl;
  const int len = b < B ? min(max(lens[b], 0), Tp) : 0;
  const int U = ub * UW + u;
  const size_t si = ((size_t)d * B + b) * H + U;       // hfin / cst index (valid when b < B)
  const size_t gi = ((size_t)d * Bp + b) * H + U;      // granule index within a buffer
  // s16 image position of (d, U) in halves: row image rows of 2 C halves, column (d H + U) in 32-k tiles
  // [32 hi | 32 lo]; km: 16-k-block major [C / 16][B Tp][16 hi | 16 lo] (lo 16 halves after hi)
  const int xcol = d * H + U;
  const size_t x16_base = km ? (size_t)(xcol >> 4) * B * Tp * 32 + (xcol & 15) : (size_t)((xcol >> 5) * 64 + (xcol & 31));
  const size_t x16_rs = km ? 32 : 2 * C;  // halves per image row
  const int x16_lo = km ? 16 : 32;
  __shared__ int s_plain;
  if (tid == 0) {
    s_tmax = 0;
    s_quit[0] = s_quit[1] = 0;
  }
  // ---- hand-off store flavour (speed only, never correctness).  A plain (sc0) store keeps the
  // word's line in this XCD's L2, where a same-XCD member's sc1 poll (L1 bypassed, L2-served)
  // finds it without the memory-side round trip an sc1 store (line dropped from L2) costs; a
  // member on another XCD would never see it (MI355X_MICROARCH.md, stores of each flavour).  So
  // each workgroup publishes its XCC id (sc1) in a per-launch table (zeroed by reset_rec_layer)
  // and stores plain only when it has read all P ids of its group equal to its own: every
  // consumer of its words is then on its XCD.  Any other outcome (another XCD, a poll bound)
  // keeps sc1 stores, which every consumer sees wherever it runs.
  if (w == 0) {
    int plain = 0;
    if (store_plain) {
      uint32_t* xt = hx + (size_t)3 * 2 * plane;
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
      const uint32_t me = 0x100u | (xcc & 0xFu);
      if (lane == 0) __hip_atomic_store(xt + grp * P + mem, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t got = me;
      if (lane < P) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          got = __hip_atomic_load(xt + grp * P + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((got & 0x100u) || __builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS / 1000) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      plain = __all(got == me) ? 1 : 0;
    }
    if (lane == 0) s_plain = plain;
  }
  __syncthreads();
  const int plain_st = s_plain;
  if (u == 0 && len > 0) atomicMax(&s_tmax, len);

  // ---- this wave's W_hh fragments, resident for the whole layer (64 VGPRs)
  const float* Wd = Whh_f + (size_t)d * (H / 16) * 4 * NKC * FRAG;
  float4 bw[4][4];
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    const float* wb = Wd + ((size_t)((ub * (UW / 16) + uh) * 4 + tn) * NKC + kc) * FRAG + lane * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bw[tn][q] = *reinterpret_cast<const float4*>(wb + q * 256);
  }
  // S16 view of the same registers: bw[tn][2j + hl] = the 8 halves of k-step j (hl 0 hi, 1 lo)
  // granule sweep of this wave: rows (lane & 15) of its half, units kc*64 + (lane>>4)*16 + 0..15;
  // the buffer descriptor takes the wave-uniform part, the lane part is the byte voffset
  const int wbase = __builtin_amdgcn_readfirstlane(((d * Bp + rg * RG + half * 16) * H + kc * 64));
  const int voff = ((lane & 15) * H + (lane >> 4) * 16) * (int)sizeof(uint32_t);
  __syncthreads();
  const int tmax = s_tmax;

  float c = 0.f;
  // epilogue operands that do not depend on h (Gin gates, residual input) are software-pipelined
  // one step ahead: step s+1's are issued after step s's MFMAs (round 2; right after the sweep
  // before: rec 2.82-2.88 -> 2.62-2.63 ms per greedy batch), so they land
  // during the MFMAs / cell instead of in front of the next sweep's vmcnt(0) wait
  auto load_operands = [&](int s, float (&g)[4], float& xr) {
    if (s < len) {
      const int t = (d == 0) ? s : (len - 1 - s);
      // the cell's four gates are adjacent (casr_internal.h enc_gate_col): one 16-B load
      const float4 q = *reinterpret_cast<const float4*>(Gin + ((size_t)b * Tp + t) * (8 * H) + d * 4 * H + U * 4);
      g[0] = q.x, g[1] = q.y, g[2] = q.z, g[3] = q.w;
      if (residual) xr = xin[((size_t)b * Tp + t) * C + d * H + U];
    }
  };
  uint32_t* tr = trace ? trace + ((size_t)(grp * P + mem) * NW + w) * Tp * 5 : nullptr;
  // The loop runs two steps per iteration over two statically named operand sets (A, B): step s
  // uses the set loaded after sweep s-1 (retired by sweep s's vmcnt(0)) and loads the other one
  // for s+1 right after its own sweep, so no operand register is copied and nothing waits at the
  // loop latch (a one-set loop copied the fresh loads there behind a vmcnt(0) that also waited
  // for the step's stores).
  // FIRST (step 0, peeled): no sweep, no MFMA.  The later steps have both unconditionally, so every
  // operand load is provably retired by the sweep's vmcnt(0) before its use.
  auto step =[&](auto first_c, const int s, const float (&gin_v)[4], const float x_res, float (&gin_n)[4],
                  float& x_n) -> bool {
    constexpr bool FIRST = decltype(first_c)::value;
    const bool act = s < len;
    uint32_t npass = 0;
    if (tr && lane == 0) tr[s * 5 + 0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    f32x4 acc[4];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) acc[tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 v[4];
    if constexpr (!FIRST) {
      // h_{s-1}: words tagged with the parity of s in buffer s % 3
      uint32_t* src = hx + (size_t)(s % 3) * 2 * plane + wbase;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(src, 0, 16 * H * (int)sizeof(uint32_t), 0x00020000);
      const uint32_t want = (s & 1) ? TAG_BIT : 0u;
      // pacing of the first poll (CASR_OPT_REC_SLEEP): sleep pre_sleep x 64 clocks.  A poll issued
      // before the group's stores have landed fails and costs a whole extra round trip.
      // Measured (round 1, ms per greedy batch, one poll per pass after a wait for the wave's own
      // stores): no wait 5.95, wait + sleep 0 / 2 / 4 / 5 / 6 / 8 / 10 = 3.05 / 3.24 / 2.91 / 2.80 /
      // 2.82-2.85 / 2.87 / 2.89.  With the plain hand-off stores and two polls per pass (below) the
      // own-store wait measured slower (2.67 -> 2.76-2.79 ms) and was removed (round 3).
      for (int i = 0; i < pre_sleep; ++i) __builtin_amdgcn_s_sleep(1);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      {
        // two polls in flight per pass, the second poll_gap x 64 clocks after the first: a first
        // poll that arrives before the group's last store costs the gap instead of a round trip.
        // Measured on one box, rec ms per greedy batch (3 rounds, interleaved): one poll after
        // sleep 6 3.13-3.19; sleep 2 + gap 4 3.07-3.11; sleep 1 + gap 3 3.07-3.11; sleep 0 +
        // gap 3-5 3.11-3.16; no own-store wait + sleep 4 + gap 3 3.08-3.14.  With plain (L2-kept)
        // hand-off stores (below): wait 2 + sleep 0 + gap 2 2.83-2.88, no wait + sleep 0 / 1 / 2 +
        // gap 2 2.78-2.87 / 2.80-2.82 / 2.80-2.86, gap 1 2.82-2.87.  Default: no wait, sleep 1, gap 2.
        for (uint32_t pass = 0;; ++pass) {
          asm volatile("" ::: "memory");
          u32x4 v2[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + i * 16, 0, 16 /* sc1 */);
          __builtin_amdgcn_sched_barrier(0);
          for (int i = 0; i < poll_gap; ++i) __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int i = 0; i < 4; ++i) v2[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + i * 16, 0, 16 /* sc1 */);
          __builtin_amdgcn_sched_barrier(0);
          uint32_t bad = 0, bad2 = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) bad |= (v[i].x ^ want) | (v[i].y ^ want) | (v[i].z ^ want) | (v[i].w ^ want);
          npass = 2 * pass + 1;
          if (__all((bad & TAG_BIT) == 0)) break;
#pragma unroll
          for (int i = 0; i < 4; ++i) bad2 |= (v2[i].x ^ want) | (v2[i].y ^ want) | (v2[i].z ^ want) | (v2[i].w ^ want);
          npass = 2 * pass + 2;
          if (__all((bad2 & TAG_BIT) == 0)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = v2[i];
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || pass > (1u << 21)) {
            if (lane == 0) {
              s_quit[s & 1] = 1;
              __hip_atomic_fetch_or(err, CASR_DEV_REC_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
          }
        }
      }
      if (tr && lane == 0) tr[s * 5 + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
    if constexpr (!FIRST) {
      if constexpr (S16) {
        f32x4 accx[4];
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) accx[tn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f16x8 ah, al;
          unpack16_tagged(v[2 * j], v[2 * j + 1], ah, al);
#pragma unroll
          for (int tn = 0; tn < 4; ++tn)
            mfma_s16(ah, al, __builtin_bit_cast(f16x8, bw[tn][2 * j]), __builtin_bit_cast(f16x8, bw[tn][2 * j + 1]),
                     acc[tn], accx[tn]);
        }
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[tn][e] = s16_combine(acc[tn][e], accx[tn][e]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a0 = decode_granule(v[q].x), a1 = decode_granule(v[q].y);
          const float a2 = decode_granule(v[q].z), a3 = decode_granule(v[q].w);
#pragma unroll
          for (int tn = 0; tn < 4; ++tn) {
            acc[tn] = mfma16x16x4(a0, bw[tn][q].x, acc[tn]);
            acc[tn] = mfma16x16x4(a1, bw[tn][q].y, acc[tn]);
            acc[tn] = mfma16x16x4(a2, bw[tn][q].z, acc[tn]);
            acc[tn] = mfma16x16x4(a3, bw[tn][q].w, acc[tn]);
          }
        }
      }
    }
    f32x4 (*rb)[4][64] = red[s & 1];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) rb[w][tn][lane] = acc[tn];
    // step s+1's operands: issued here, after this wave's MFMAs (the wave whose sweep completes
    // last sets the step's pace, and its MFMAs no longer queue behind these loads), still ahead of
    // the next sweep, whose vmcnt wait retires them before the cell uses them
    load_operands(s + 1, gin_n, x_n);
    __syncthreads();
    // the 16 k-chunk partials of this cell and the quit flag in one round of LDS reads (the quit
    // test used to go first: one more LDS round trip on the step chain)
    const int hw = ((rl >> 4) + (RG / 16) * (u >> 4)) * 4, rr = rl & 15;
    const int src_lane = (u & 15) + 16 * (rr >> 2), reg = rr & 3;
    float part[4][4];
#pragma unroll
    for (int tn = 0; tn < 4; ++tn)
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) part[tn][ww] = rb[hw + ((ww - (hw >> 2)) & 3)][tn][src_lane][reg];  // k-chunk ww
    const int quit = s_quit[s & 1];  // acted on below, before the first store of the step
    if (tr && lane == 0) tr[s * 5 + 2] = (uint32_t)__builtin_amdgcn_s_memrealtime();

    // cell (same reduction order as rec_step_kernel: k-chunks 0..3, then + Gin)
    float h2 = 0.f;
    if (act) {
      float gate[4];
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) sum += part[tn][ww];
        gate[tn] = sum + gin_v[tn];
      }
      float c2;
      if constexpr (S16)  // performance arithmetic: hardware-exp cell (casr_common.h, ~1e-7)
        lstm_cell_hw(gate[0], gate[1], gate[2], gate[3], c, h2, c2);
      else  // f32 arithmetic: libm cell, torch's CPU formulas
        lstm_cell(gate[0], gate[1], gate[2], gate[3], c, h2, c2);
      c = c2;
    }
    if (quit) return false;
    // the hand-off word goes out first: the layer outputs below are off the step chain
    if (s + 1 < tmax) store_granule<S16>(hx + (size_t)((s + 1) % 3) * 2 * plane + gi, s + 1, h2, plain_st);
    if (act) {
      const int t = (d == 0) ? s : (len - 1 - s);
      const size_t oi = ((size_t)b * Tp + t) * C + d * H + U;
      if (s == len - 1) hfin[si] = h2;
      const float y = residual ? residual_add(h2, x_res) : h2;
      out[oi] = y;
      // s16x3: the next layer's input row image, written here instead of by split_rows_kernel
      if (S16 && x16) {
        const uint32_t wv = split16_word(y);
        uint16_t* xp = x16 + ((size_t)b * Tp + t) * x16_rs + x16_base;
        xp[0] = (uint16_t)wv;
        xp[x16_lo] = (uint16_t)(wv >> 16);
        const float m = fabsf(y);
        if (m >= 65520.f && m < INFINITY)
          __hip_atomic_fetch_or(err, CASR_DEV_F16_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (tr && lane == 0) {
      tr[s * 5 + 3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
      tr[s * 5 + 4] = npass;
    }
    return true;
  };
  float gA[4] = {0.f, 0.f, 0.f, 0.f}, gB[4] = {0.f, 0.f, 0.f, 0.f}, xA = 0.f, xB = 0.f;
  load_operands(0, gA, xA);
  if (tmax > 0 && step(std::true_type{}, 0, gA, xA, gB, xB)) {
    for (int s = 1; s < tmax; s += 2) {
      if (!step(std::false_type{}, s, gB, xB, gA, xA)) break;
      if (s + 1 < tmax && !step(std::false_type{}, s + 1, gA, xA, gB, xB)) break;
    }
  }
  if (b < B) cst[si] = c;
  // padded frames (t >= len) of the layer output and of the row image are zero (pad_packed_sequence,
  // util.py:1307), written here so the host needs no memset of the output buffers
  if (b < B)
    for (int t = len; t < Tp; ++t) {
      out[((size_t)b * Tp + t) * C + d * H + U] = 0.f;
      if (S16 && x16) {
        uint16_t* xp = x16 + ((size_t)b * Tp + t) * x16_rs + x16_base;
        xp[0] = 0;
        xp[x16_lo] = 0;
      }
    }
}

}  // namespace

// CUs of the current device (the persistent grid wants one workgroup per CU)
static int rec_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return v;
}

// Layout per batch.  32x16 (512 threads: 32 rows x 16 units) while its grid of 16 x ceil(B/32) x 2
// workgroups needs all the CUs (B = 256: one per CU); 16x16 (256 threads) once 16 x ceil(B/16) x 2
// workgroups still fit one per CU (B <= 128): twice the workgroups, each with half the rows, so
// a step's MFMA and cell work per CU halves while the hand-off stays a 16-producer exchange.
// Measured (rec ms per batch, two interleaved rounds): beam B = 128 2.36-2.37 (32x16) -> 2.01-2.02
// (16x16); greedy B = 256 2.67-2.71 (32x16) vs 3.08-3.10 (16x16: two workgroups per CU).
// CASR_OPT_REC_LAYOUT forces one (1 = 32x16, 2 = 16x32, 3 = 16x16).
int rec_layout(int B, const Tuning& t) {
  switch (t[CASR_OPT_REC_LAYOUT]) {
    case 1: return 0;
    case 2: return 1;
    case 3: return 2;
    default: return (H / 16) * ((B + 15) / 16) * 2 <= rec_cus() ? 2 : 0;
  }
}
static int rec_rows(int layout) { return layout == 0 ? 32 : 16; }
static int rec_units(int layout) { return layout == 1 ? 32 : 16; }

// the three granule buffers, then the placement table (one word per workgroup)
static size_t rec_granule_words(int B) { return (size_t)3 * 2 * ((B + 31) / 32 * 32) * H; }

size_t rec_layer_granule_bytes(int B, int layout) {
  return (rec_granule_words(B) + (size_t)rec_layer_grid_blocks(B, layout)) * sizeof(uint32_t);
}

int rec_layer_waves(int layout) { return rec_rows(layout) * rec_units(layout) / 64; }

int rec_layer_producers(int layout) { return H / rec_units(layout); }

int rec_layer_grid_blocks(int B, int layout) {
  return (H / rec_units(layout)) * ((B + rec_rows(layout) - 1) / rec_rows(layout)) * 2;
}

template <int RG, int UW>
static int occ() {
  // both arithmetic variants must fit: the capacity is the smaller of the two
  static const int v = [] {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, rec_layer_kernel<RG, UW, false>, RG * UW, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rec_layer_kernel<RG, UW, true>, RG * UW, 0) != hipSuccess)
      return 0;
    return a < b ? a : b;
  }();
  return v;
}

bool rec_layer_fits(int B, int layout) {
  int per_cu;
  switch (layout) {
    case 1: per_cu = occ<16, 32>(); break;
    case 2: per_cu = occ<16, 16>(); break;
    default: per_cu = occ<32, 16>(); break;
  }
  return rec_layer_grid_blocks(B, layout) <= per_cu * rec_cus();
}

hipError_t reset_rec_layer(uint32_t* hx, int B, int layout, hipStream_t s) {
  // Guideline 16: re-initialise every call.  Buffer j is first read at step j (j = 1, 2) or 3
  // (j = 0), expecting parity 1, 0, 1: fill buffers 0 and 1 with parity 0, buffer 2 with 1.
  // The placement table after them starts at 0 (no id published).
  const size_t per = rec_granule_words(B) / 3;
  FillList fl;
  fl.add32(hx, 0u, 2 * per);
  fl.add32(hx + 2 * per, TAG_BIT, per);
  fl.add32(hx + 3 * per, 0u, (size_t)rec_layer_grid_blocks(B, layout));
  return fill_multi(fl, s);
}

// CASR_OPT_REC_COOP 2 (default, round 6): the persistent layer is an ordinary launch, ordered after
// the previous persistent launch of this process on the same device by one process-wide event per
// device (its stream waits for that event, the launch records it).  The hand-off spins need every
// workgroup of the grid resident: two persistent grids dispatched side by side (batches in flight
// on several streams, casr/pipeline.py) could each hold part of the chip and wait on the other, so
// they never overlap; any other kernel beside a partly placed grid finishes and frees its CUs.  The
// cooperative launch (1) gave the same guarantee at about 25 us per launch (interleaved A/B,
// profiles/r06/rec_launch/: greedy 6.53-6.58 -> 6.43-6.46 ms per batch serially, beam 10.11-10.13
// -> 9.99-10.06 ms with two in flight).  Another process's persistent grid is not ordered: the
// bounded hand-off wait (device flag 32) covers that case, as for the ordinary launch (0).
namespace {
std::mutex g_rec_chain_mu;
constexpr int REC_CHAIN_DEVICES = 64;
hipEvent_t g_rec_chain[REC_CHAIN_DEVICES] = {};
}  // namespace

hipError_t launch_rec_layer(const float* Whh_f, const float* Gin, const float* xin, float* out,
                            uint16_t* x16, uint32_t* hx, float* hfin, float* cst, const int32_t* lens, int B, int Tp,
                            int residual, int s16, int32_t* err, uint32_t* trace, int layout, const Tuning& t,
                            hipStream_t s, int km) {
  int Bp = (B + 31) / 32 * 32;  // granule planes padded to 32 rows for every layout
  const int RG = rec_rows(layout), UW = rec_units(layout);
  int nrg = (B + RG - 1) / RG;
  // (-1, the default: no sleep for grids of 64 workgroups or more, one unit below: B <= 16 in the
  // 16-row layout, 32 workgroups; measured round 6)
  const int nwg = (H / UW) * nrg * 2;
  int sleep = t[CASR_OPT_REC_SLEEP] < 0 ? (nwg >= 64 ? 0 : 1) : t[CASR_OPT_REC_SLEEP] > 16 ? 16 : t[CASR_OPT_REC_SLEEP];
  int gap = t[CASR_OPT_REC_POLL_GAP] < 1 ? 1 : t[CASR_OPT_REC_POLL_GAP] > 8 ? 8 : t[CASR_OPT_REC_POLL_GAP];
  int plain = t[CASR_OPT_REC_STORE_PLAIN] ? 1 : 0;
  const dim3 grid((H / UW) * nrg * 2), block(RG * UW);
  auto go = [&](auto kern) -> hipError_t {
    if (t[CASR_OPT_REC_COOP] == 1) {
      // every workgroup co-resident or an immediate launch error (the hand-off spins need all of them)
      void* args[] = {&Whh_f, &Gin, &xin, &out, &x16, &hx, &hfin, &cst, &lens, &B, &Bp, &Tp, &residual,
                      &err, &trace, &nrg, &sleep, &gap, &plain, &km};
      return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(kern), grid, block, args, 0, s);
    }
    hipEvent_t chain = nullptr;
    std::unique_lock<std::mutex> lk(g_rec_chain_mu, std::defer_lock);
    if (t[CASR_OPT_REC_COOP] == 2) {  // ordered after this process's previous persistent grid (above)
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      int dev = -1;
      hipError_t e = hipStreamIsCapturing(s, &cs);
      if (e == hipSuccess) e = hipGetDevice(&dev);
      if (e != hipSuccess) return e;
      if (cs == hipStreamCaptureStatusNone && dev >= 0 && dev < REC_CHAIN_DEVICES) {
        lk.lock();
        if (!g_rec_chain[dev]) {
          e = hipEventCreateWithFlags(&g_rec_chain[dev], hipEventDisableTiming);
          if (e != hipSuccess) return e;
        }
        chain = g_rec_chain[dev];
        e = hipStreamWaitEvent(s, chain, 0);  // (an event never recorded: no wait)
        if (e != hipSuccess) return e;
      }
    }
    hipLaunchKernelGGL(kern, grid, block, 0, s, Whh_f, Gin, xin, out, x16, hx, hfin, cst, lens, B, Bp, Tp, residual,
                       err, trace, nrg, sleep, gap, plain, km);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && chain) e = hipEventRecord(chain, s);
    return e;
  };
  switch (layout) {
    case 1: return s16 ? go(rec_layer_kernel<16, 32, true>) : go(rec_layer_kernel<16, 32, false>);
    case 2: return s16 ? go(rec_layer_kernel<16, 16, true>) : go(rec_layer_kernel<16, 16, false>);
    default: return s16 ? go(rec_layer_kernel<32, 16, true>) : go(rec_layer_kernel<32, 16, false>);
  }
}

}  // namespace casr
