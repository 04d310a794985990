// Bahdanau additive attention of one decode step on gfx950 (BauAttn.forward, heads == 1,
// attention.py:80-95):
//   q[r]    = h[r] . W_hidden                        (torch.mm, attention.py:92)
//   e[r][t] = sum_a v[a] * tanh(keys[b][t][a] + q[r][a])
//   alpha   = softmax_t(mask + e),   ctx[r] = sum_t alpha[r][t] * enc[b][t]   (:93-95)
// for every decoder row r = b*k + j.  Keys/values are per utterance (the reference tiles
// and re-gathers them per beam, model.py:660-669 / :913-916): a block serves up to KPB
// beam rows of one utterance, so each utterance's keys and values are streamed
// ceil(k / KPB) times per step instead of k times.
//
// HBM/L2-bound streaming + transcendental work, no MFMA.  512 threads: every phase has
// 8 waves with all of a lane's 16 B loads of the phase in flight; partial sums are combined
// through LDS in a fixed order (results are deterministic).  keysT is [B][A][Tq] (Tq = Tp
// rounded up to 4) so a lane reads 4 consecutive time steps of one key row.
#include <stdlib.h>

#include <type_traits>

#include "beam_select.h"
#include "casr_common.h"
#include "casr_internal.h"

// (diagnostic builds only, tools/probes: bit 0 drops the greedy prologue's W_hidden loads, bit 1
// its gate-row gather; the results are then wrong)
#ifndef CASR_AT_DIAG
#define CASR_AT_DIAG 0
#endif

// the split attention's hand-off (TSPLIT) orders its agent-scope stores before the arrival count
// with vmcnt(0) alone, as decoder.hip's k split: gfx9-family only
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "attention.hip: the split hand-off assumes gfx950's vmcnt store counting; build for gfx950 only"
#endif

namespace casr {

constexpr int AT_THREADS = 512;
constexpr int AT_WAVES = AT_THREADS / 64;
constexpr int AT_NQ = HD / 16;  // query partials per row at most (dec_q_slots: one per LSTMCell column block)
constexpr int AT_MAXG = 8;      // a-groups of the score phase
constexpr int AT_CH = 20;       // keys rows in flight per score batch (apg = 19 at Tp = 266)
constexpr int AT_APAD = A + AT_CH;  // q / v rows in LDS, zero-padded so a batch never branches

__host__ __device__ constexpr int attn_tq(int Tp) { return (Tp + 3) & ~3; }

template <int KPB, int MAXG = AT_MAXG>
__host__ __device__ constexpr int attn_scratch_floats(int Tq) {
  // score partials [MAXG][KPB][Tq] | context partials [4][KPB][C]
  return MAXG * KPB * Tq > 4 * KPB * C ? MAXG * KPB * Tq : 4 * KPB * C;
}
// (round 6) the split folded greedy attention (attention_kernel<1, 1, true>): a block takes Tq / S
// steps, so its score phase can use up to 32 a-groups of 4 keys rows (the unsplit form's 8 groups of
// 16 rows would leave most of the block's threads idle on a short range)
constexpr int AT_MAXG_SPLIT = 32;

// the folded step's cell phase (CELL): h [HD] | query slices [AT_QS][A]
constexpr int AT_QS = AT_THREADS / (A / 4);  // 16 unit slices of HD / AT_QS = 32 units
constexpr int AT_CELL_FLOATS = HD + AT_QS * A;
static_assert(AT_QS * A >= 4 * HD, "the token's gate-table row fits the query slice area (CELL 1)");

// LDS: qs, eqs [AT_APAD][KPB] | vs, v2s [A] | (AT_MAXG unused) | scratch | es [Tq][KPB] | (CELL: h,
// query slices) | value rows
// (CELL 2, the beam cell phase, keeps its h rows and query slices in the score scratch instead)
template <int KPB, int CELL = 0, bool TSPLIT = false>
__host__ __device__ constexpr size_t attn_smem_floats(int Tp) {
  return (size_t)2 * KPB * AT_APAD + 2 * A + AT_MAXG +
         attn_scratch_floats<KPB, TSPLIT ? AT_MAXG_SPLIT : AT_MAXG>(attn_tq(Tp)) + KPB * attn_tq(Tp) +
         (CELL == 1 ? AT_CELL_FLOATS : 0);
}

// Split exponential form of the score tanh.  tanh(k + q) = 1 - 2 / (1 + e^{2k} e^{2q}): with
// ek = exp(2k) computed once per encode (KeysEpi, next to the keys) and eq = exp(2q) once per row
// and step, a term costs one fma (d = ek eq + 1), one v_rcp_f32 and one fma into the score,
// against two transcendentals in tanh_fast.  The score of an a-group is
//     sum_a v_a tanh(k_a + q_a) = sum_a v_a  +  sum_a (-2 v_a) / (1 + ek_a eq_a).
// Range: ek and eq are finite normal floats while |k|, |q| < 43 (exp2 of up to 124); their product
// then overflows to +inf only where k + q > 44 (rcp = 0, tanh = 1, as tanh_fast) and underflows
// only where k + q < -51 (d = 1, tanh = -1).  Outside that range ek / eq are stored as NaN, which
// makes the block's score NaN and sends the block back to the direct form (also the path for a
// NaN key or query, whose scores then come out as in tanh_fast).  Error: the exponent products
// round k 2 log2(e) and q 2 log2(e) separately, so e^{2k} e^{2q} carries ~1.2e-7 (|k| + |q|)
// relative error where exp(2(k + q)) carries ~1.2e-7 |k + q|; for the |k|, |q| of a few units of
// the path's activations the score moves by ~1e-6 at most (tests: alignment within 1e-5).
// split_exp2x: casr_common.h (shared with KeysEpi)

// tanh(x) = 1 - 2 / (1 + exp(2x)) on v_exp_f32 / v_rcp_f32: mul, exp, add, rcp, fma (5 VALU
// ops; the libm-style division __fdividef compiles to on gfx950 is an 11-instruction
// div_scale / div_fmas / div_fixup sequence).  exp overflows to +inf for x > ~44 (rcp(inf) = 0,
// tanh = 1) and underflows to 0 for x < ~-44 (tanh = -1).  Absolute error <= ~3e-7 (rcp 1 ulp
// on r <= 1, exp 1 ulp damped by r(1 - r)): every term of the score sum is this times |v[a]|
// (~0.1) and 128 terms are summed, so the scores stay within ~1e-6 of the libm form (tests:
// alignment within 1e-5).
CASR_DEV float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2 log2(e) x
  return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + e), 1.f);
}

// Two at a time: the multiply, the add and the fma as packed f32 (v_pk_mul / v_pk_add /
// v_pk_fma_f32: two lanes' worth per instruction, each element rounded exactly as the scalar
// form), the exp and rcp per element.  Bitwise equal to tanh_fast on each element; the score
// phase is bound by this VALU work (with 4 beam rows per block, 136 K tanh per block and step).
typedef float f32x2 __attribute__((ext_vector_type(2)));
CASR_DEV f32x2 tanh_fast2(f32x2 x) {
  const f32x2 y = x * (f32x2){2.8853900817779268f, 2.8853900817779268f};
  const f32x2 d = (f32x2){1.f, 1.f} + (f32x2){__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
  const f32x2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return __builtin_elementwise_fma((f32x2){-2.f, -2.f}, r, (f32x2){1.f, 1.f});
}

// Memory-level parallelism is the design driver: one block (8 waves) per utterance and step
// streams its keys (A x Tq f32) and values (len x C f32) once per step, so every phase keeps all
// of a lane's loads of that phase in flight at once (one round trip per phase, not one per
// unrolled batch).  The query q = h . W_hidden arrives as HD/16 partials written by the decoder
// LSTM epilogue (decoder.hip DecLstmEpi), so W_hidden is not re-read per block.
// diagnostics (CASR_DG_TRACE, tools/probes/dg_trace.py): per-block phase stamps of the last launch
__device__ uint32_t* g_at_trace = nullptr;

// CELL (the folded step, casr_internal.h KA): before the attention the block runs the LSTM cell of
// its rows on gates_prev + emb_gates[tok] and q = h . W_hidden itself (no query partials); st
// receives h, c (and ctx as always).  CELL 1, greedy (KPB = 1, row r = b): the block first runs the
// select of step l - 1 for its row.  CELL 2, beam (KPB = 4 or 8): tokens and predecessor rows come
// from the beam select; gates_prev and c are read at the predecessor row.  CELL 3, beam with one
// block per utterance (KPB = k = 4 or 8): the block first runs the beam select of step l - 1 for
// its utterance (beam_select.h) and takes the tokens and predecessor rows from it.
// TSPLIT (round 6, CELL 1 only, CASR_OPT_ATTN_SPLIT): the utterance's time steps are split over
// cell.split blocks (blockIdx.y = the split, cell.tc steps each, a multiple of 4).  Every block runs
// the select, the cell and the query (identical values; only split 0 writes the bookkeeping and h / c),
// then the scores, the softmax's maximum m_s and sum z_s and the unnormalised context c_s of its range.
// Each block publishes (m_s, z_s, c_s) with agent-scope stores and counts itself in; the last of the
// utterance's blocks merges in split order: M = max m_s, w_s = exp(m_s - M), Z = sum w_s z_s,
// ctx = (sum w_s c_s) / Z, and writes ctx (and its split words) as the unsplit form does.
template <int KPB, int CELL = 0, bool TSPLIT = false>
__global__ __launch_bounds__(AT_THREADS) void attention_kernel(
    float* __restrict__ st, const float* __restrict__ qpart, const float* __restrict__ keysT,
    const float* __restrict__ ekT, const float* __restrict__ enc, const int32_t* __restrict__ lens,
    const float* __restrict__ vv, int R, int k, int Tp, float* __restrict__ align, const int32_t* __restrict__ newdone,
    int l, int total, int npf, int direct, int nq, int V, AttnCell cell) {
  static_assert(CELL != 1 || KPB == 1, "the folded greedy step: one row per block");
  static_assert(CELL != 2 || KPB >= 2, "the folded beam step: beam rows of one utterance per block");
  static_assert(CELL != 3 || KPB == 4 || KPB == 8, "the fused beam select: one block per utterance, k = 4 or 8");
  static_assert(CELL != 4 || KPB == 4, "the fused beam select, two blocks per utterance: k = 8");
  static_assert(!TSPLIT || CELL == 1, "the split attention: the folded greedy step");
  constexpr int MAXG = TSPLIT ? AT_MAXG_SPLIT : AT_MAXG;
  // CELL 4 (round 5): KPB 4 at k = 8, so two blocks per utterance (B = 128: 256 blocks) run the same
  // select of step l - 1; the first (blockIdx.y == 0) does its global bookkeeping, both read their
  // rows' tokens and predecessor rows from their own copy
  constexpr int KSEL = CELL == 4 ? 2 * KPB : KPB;  // rows of the fused select
  extern __shared__ __attribute__((aligned(16))) float sm[];
  uint32_t* atr = g_at_trace ? g_at_trace + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
  auto stamp = [&](int i) {
    if (atr && threadIdx.x == 0) atr[i] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // (CELL 1: the early exit is decided after the block's own select, below.  CELL 3: the select of
  // step l - 1 skips when every utterance finished before step l - 1; otherwise the block runs it and
  // the attention, whatever this launch's selects add to step l - 1's count)
  if (CELL != 1 && done_before(newdone, CELL >= 3 ? l - 1 : l) >= total) return;
  const int TqG = attn_tq(Tp);                 // keysT / ekT row stride
  const int sp = TSPLIT ? (int)blockIdx.y : 0;  // the block's split
  const int tbase = TSPLIT ? sp * cell.tc : 0;  // its first step
  const int Tq = TSPLIT ? min(cell.tc, TqG - tbase) : TqG;  // its steps (a multiple of 4)
  float* qs = sm;                   // [AT_APAD][KPB]: q transposed, zero past A and for j >= nk
  float* eqs = qs + KPB * AT_APAD;  // [AT_APAD][KPB]: exp(2q) (split form), zero past A
  float* vs = eqs + KPB * AT_APAD;  // [A]
  float* v2s = vs + A;              // [A]: -2 v
  float* xs = v2s + A + AT_MAXG;    // scratch
  float* es = xs + attn_scratch_floats<KPB, MAXG>(Tq);  // [Tq][KPB]: one 4 x KPB-byte read per t
  float* hs = es + KPB * Tq;                       // CELL: [HD] h, then [AT_QS][A] query slices
  float* vl = hs + (CELL == 1 ? AT_CELL_FLOATS : 0);  // [npf][C]: value rows 0..npf-1 (LDS-DMA)
  const int b = blockIdx.x, j0 = TSPLIT ? 0 : blockIdx.y * KPB;
  const int nk = min(KPB, k - j0);
  // CELL 1: wv through readfirstlane, provably wave-uniform, so the prologue's per-wave roles are
  // scalar branches (blocks of their own for hipcc's wait insertion, not exec-masked regions whose
  // pending loads merge); the other instances keep the plain form (their register allocation)
  const int tid = threadIdx.x, wv = CELL == 1 ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6, ln = tid & 63;
  const int len = TSPLIT ? max(0, min(min(lens[b], Tp) - tbase, Tq)) : min(lens[b], Tp);  // (local steps)
  const size_t row0 = (size_t)b * k + j0;

  // score work split (phase 2): G a-groups of apg keys rows x Tq / 4 chunks of 4 steps
  const int nch = Tq / 4;
  const int G = min(MAXG, max(1, AT_THREADS / nch));
  const int apg = (A + G - 1) / G;
  const float* kb = keysT + (size_t)b * A * TqG + tbase;
  const float* ekb = ekT + (size_t)b * A * TqG + tbase;
  constexpr int CH = KPB >= 8 ? AT_CH / 2 : AT_CH;  // KPB 8: half the keys rows per batch (registers)
  // CELL: the first keys batch of this thread's first score item (split form) is loaded before the
  // cell phase, which it does not depend on, so the scores start on landed keys
  constexpr bool PRE = CELL == 1 || (CELL >= 2 && KPB >= 8);  // (KPB 4: 20 keys rows per batch, no registers left)
  float4 kvp[PRE ? CH : 1];
  // CELL 1, 2 (round 4): unconditional loads at clamped addresses, masked at use.  Per-slot
  // conditional loads compile to lane-masked regions, and their joins made hipcc wait for every load
  // in flight (the preload now follows the gathers and W_hidden loads of the cell phase).  CELL 0
  // keeps the conditional form
  auto preload_keys = [&]() {
    const int ag = tid / nch, t0 = 4 * (tid - ag * nch), a0 = ag * apg, a1 = min(A, a0 + apg);
    const bool live = !direct && tid < G * nch && t0 < len;
    if constexpr (CELL != 0) {  // raw values: the slots past a1 / dead items are zeroed at use (score_item)
      const int tc = min(t0, Tq - 4);
#pragma unroll
      for (int i = 0; i < CH; ++i)
        kvp[i] = *reinterpret_cast<const float4*>(ekb + (size_t)min(a0 + i, A - 1) * TqG + tc);
      (void)live;
      (void)a1;
    } else {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        kvp[i] = live && a0 + i < a1 ? *reinterpret_cast<const float4*>(ekb + (size_t)(a0 + i) * Tq + t0)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if constexpr (PRE && CELL == 0) preload_keys();
  if constexpr (CELL == 1) {
    // 0. the folded step's LSTM cell (decoder.py:104-114) and query (attention.py:92) for row r.
    // Load order (round 4): a wave's loads retire in issue order, so whatever a wave issues first is
    // what it waits on first.  Waves 1..7 issue the previous step's gate pre-activations of unit
    // u = tid and its c, their W_hidden slices (rows 32 us .. +31, columns 4 a4 .. +3) and their
    // first keys batch at once, and wait at the barrier.  Wave 0 issues the select's operands
    // first, selects the token, then gathers the token's gate-table row (8 KB) into LDS (the query
    // slice area, free until the query) with nothing else of its own in flight, and only then
    // issues its W_hidden slice and keys.  So the cell reads its gate row from LDS instead of each
    // wave waiting for its own gather behind the keys stream (phase trace, profiles/r04: select
    // 2.8 us, cell 5.2 us, query 0.8 us p50 with the gathers per wave)
    __shared__ int tk_s, skip_s;
    const int r = (int)row0;
    const int a4 = tid & (A / 4 - 1), us = tid / (A / 4);
    constexpr int UPS = HD / AT_QS;  // units per query slice
    const int u = tid;
    auto gcol = [](int g, int u) { return (u >> 4) * 64 + g * 16 + (u & 15); };  // packed_gate_row
    float gprev[4];
    float cold;
    auto load_prev = [&]() {
#pragma unroll
      for (int g = 0; g < 4; ++g) gprev[g] = cell.gates[(size_t)r * (4 * HD) + gcol(g, u)];
      cold = cell.st_old[(size_t)r * ST + C + HD + u];
    };
    // the W_hidden slice (256 KB per block, L2-resident) is the prologue's largest read: issued at
    // the start (wave 0: right after the select's own loads), it lands under the select and the
    // gate-row gather instead of after them (round 4: prologue 9.4 us p50 with it issued after the
    // select)
    float4 wh[UPS];
    auto load_wh = [&]() {
#pragma unroll
      for (int i = 0; i < UPS; ++i)
        wh[i] = (CASR_AT_DIAG & 1) ? make_float4(0.f, 0.f, 0.f, 0.f)
                                   : *reinterpret_cast<const float4*>(cell.w_hidden + (size_t)(UPS * us + i) * A + 4 * a4);
    };
    if (wv == 0) {  // the select of step l - 1 (greedy_select_part_kernel's arithmetic) and its bookkeeping
      // rows finished before step l - 1 (the select's own skip) and before step l (the block's early
      // exit), from one load of the counters issued with the partials: the second misses what this
      // launch's selects add to step l - 1, so a block that sees every row finished skips work nothing
      // downstream reads, and one that does not computes it.
      // (round 4) Every operand load of the select is issued before its first use, in straight-line
      // code (clamped indices and selects instead of lane-masked regions, the sel branch on a kernel
      // argument), then the W_hidden slice: one round trip before the select instead of two, and no
      // wait of hipcc's between the loads (masked regions made it drain the counters' load before
      // the partials' and the partials' before W_hidden's)
      const GreedySel& gs = cell.gs;
      const int lm = max(gs.lsel, l);  // 1 ..max_len, at most 64 (prepare_decode: the fold needs it)
      const int cnt = newdone[min(ln, lm - 1)];
      const int pi = r * GP_NB + min(ln, max(gs.nbp - 1, 0));
      float m = 0.f, se = 0.f;
      int mi = 0, tq = 0, bkv = 0, finv = 0;
      if (cell.sel) {
        m = gs.gp.mx[pi];
        se = gs.gp.se[pi];
        mi = gs.gp.ix[pi];
        // the row's bookkeeping words: accum[r] in lane 1, out_len[r] in the others, from one load
        // (a per-lane address, so hipcc makes no early scalar copy of them, whose wait would sit in
        // front of the W_hidden loads), and fin[r] by a byte load beside it (the caller's B-byte
        // finished buffer: no alignment or padding is assumed)
        const int32_t* bk = ln == 1 ? reinterpret_cast<const int32_t*>(gs.accum + r) : gs.out_len + r;
        bkv = *bk;
        finv = gs.fin[r];
      } else {
        tq = cell.tok[r];
      }
      int dn_sel, dn;
      done_reduce(cnt, gs.lsel, l, dn_sel, dn);
      int t = 0;
      if (cell.sel) {
        const bool in = ln < gs.nbp;
        m = in ? m : -INFINITY;
        se = in ? se : 0.f;
        mi = in ? mi : 0x7fffffff;
        if (dn_sel < total) {  // else nothing downstream runs any more
          float gm = m;
          int gi = mi;
          wave_best(gm, gi);
          t = gi;
          const bool bad_t = (unsigned)t >= (unsigned)V;  // no finite maximum (NaN row)
          if (bad_t) t = 0;
          const float sx = wave_sum((se > 0.f) ? se * expf(m - gm) : 0.f);
          const uint8_t fin0 = (uint8_t)__builtin_amdgcn_readfirstlane(finv);
          const float acc0 = __int_as_float(__builtin_amdgcn_readlane(bkv, 1));
          const int len0 = __builtin_amdgcn_readlane(bkv, 0);
          if (ln == 0 && sp == 0) {  // (split: one block of the utterance writes the bookkeeping)
            if (bad_t) atomicOr(cell.err, CASR_DEV_NAN_LOGITS);
            greedy_book(gs, r, t, gm - (logf(sx) + gm), fin0, acc0, len0);
          }
        }
      } else {
        t = tq;
        if ((unsigned)t >= (unsigned)V) {
          if (ln == 0) atomicOr(cell.err, CASR_DEV_BAD_TOKEN);
          t = 0;
        }
      }
      if (ln == 0) {
        tk_s = t;
        skip_s = dn >= total;
      }
      // the token's gate-table row (4 HD floats, packed gate-row order) into LDS by LDS-DMA: 8 KB,
      // no registers, and wave 0's only loads in flight (the select's operands have landed), so
      // the wait for them is one gather round trip; then wave 0's own W_hidden and keys loads
      {
        const float* src = cell.emb_gates + (size_t)t * (4 * HD);
#pragma unroll
        for (int i = 0; i < 4 * HD / 256; ++i)
          if (!(CASR_AT_DIAG & 2)) lds_dma16(src + 256 * i + 4 * ln, hs + HD + 256 * i);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      load_wh();
      load_prev();
      preload_keys();
    } else {  // (an else branch: wave 0's code is not joined behind these loads)
      load_prev();
      load_wh();
      preload_keys();
    }
    __syncthreads();
    stamp(6);  // (diagnostics) the select, its bookkeeping and the gate-row gather done
    if (skip_s) return;
    float eg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) eg[g] = hs[HD + gcol(g, u)];
    float h2, c2;
    lstm_cell_hw(gprev[0] + eg[0], gprev[1] + eg[1], gprev[2] + eg[2], gprev[3] + eg[3], cold, h2, c2);
    if (sp == 0) {
      st[(size_t)r * ST + C + u] = h2;
      st[(size_t)r * ST + C + HD + u] = c2;
      reinterpret_cast<uint32_t*>(st)[(size_t)r * ST + ST16 + C + u] = split16_word(h2);
    }
    hs[u] = h2;
    __syncthreads();
    stamp(7);  // (diagnostics) the cell done, h in LDS
    float4 qa = make_float4(0.f, 0.f, 0.f, 0.f);  // units in order within the slice
#pragma unroll
    for (int i = 0; i < UPS; ++i) {
      const float hv = hs[UPS * us + i];
      qa.x = fmaf(hv, wh[i].x, qa.x);
      qa.y = fmaf(hv, wh[i].y, qa.y);
      qa.z = fmaf(hv, wh[i].z, qa.z);
      qa.w = fmaf(hv, wh[i].w, qa.w);
    }
    *reinterpret_cast<float4*>(hs + HD + us * A + 4 * a4) = qa;
    __syncthreads();
    for (int a = tid; a < A; a += AT_THREADS) {  // slices added in slice order
      float q = hs[HD + a];
#pragma unroll
      for (int i = 1; i < AT_QS; ++i) q += hs[HD + i * A + a];
      qs[a] = q;
      eqs[a] = split_exp2x(q);
    }
  }
  if constexpr (CELL >= 2) {
    // (CELL 3) the beam select of step l - 1 for utterance b, in the score scratch (free until the
    // scores); its tokens and predecessor rows also go to bs_tok / bs_src, prefilled with what
    // tok / src hold, as the separate launch leaves slots no candidate fills
    __shared__ int bs_tok[CELL >= 3 ? KSEL : 1], bs_src[CELL >= 3 ? KSEL : 1];
    if constexpr (CELL >= 3) {
      using SelLds = BeamSelLds<2 * KSEL, KSEL, AT_WAVES>;
      static_assert(sizeof(SelLds) <= attn_scratch_floats<KPB>(4) * sizeof(float), "the select's LDS fits the scratch");
      if (tid < KSEL) {
        bs_tok[tid] = cell.bs.tok_next[(size_t)b * k + tid];
        bs_src[tid] = cell.bs.src_next[(size_t)b * k + tid];
      }
      SelLds& sl = *reinterpret_cast<SelLds*>(xs);
      const bool writer = CELL == 3 || blockIdx.y == 0;
      if (cell.bs.temperature == 1.0f) beam_select_block<2 * KSEL, true>(cell.bs, b, sl, nullptr, bs_tok, bs_src, writer);
      else beam_select_block<2 * KSEL, false>(cell.bs, b, sl, nullptr, bs_tok, bs_src, writer);
      __syncthreads();  // bs_tok / bs_src written; the scratch is free again
      stamp(6);
    }
    // 0. the folded beam step's LSTM cell for the block's nk rows r = row0 + j: token tok[r],
    // predecessor s = src[r] (clamped and reported like DecLstmA::bind); thread = unit u.  Then
    // q = h . W_hidden for the block's rows as s16x3 MFMAs (the split words of h, rows padded to 16,
    // in the score scratch, free until the scores; W_hidden^T's fragment image wq16): wave w owns
    // attention columns 16 w .. 16 w + 15 over all HD units (16 k-steps of 32), so no partial sums
    // cross waves.  Its fragments are loaded before the cells, under the gathers.
    constexpr int HS16 = HD + 4;  // row stride in words: 16 B skew per row, conflict-free b128 reads
    static_assert(KPB * HS16 <= attn_scratch_floats<KPB>(4), "h rows fit the scratch");
    uint32_t* hs16 = reinterpret_cast<uint32_t*>(xs);
    const int u = tid;
    auto gcol = [](int g, int u) { return (u >> 4) * 64 + g * 16 + (u & 15); };  // packed_gate_row
    int sr[KPB], tk[KPB], bad = 0;
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
      const int r = (int)row0 + min(j, nk - 1);
      int sj, tj;
      if constexpr (CELL >= 3) {
        sj = bs_src[j0 + min(j, nk - 1)];
        tj = bs_tok[j0 + min(j, nk - 1)];
      } else {
        sj = cell.src[r];
        tj = cell.tok[r];
      }
      bad |= (unsigned)sj >= (unsigned)R ? CASR_DEV_BAD_SRC : 0;
      bad |= (unsigned)tj >= (unsigned)V ? CASR_DEV_BAD_TOKEN : 0;
      sr[j] = (unsigned)sj < (unsigned)R ? sj : r;
      tk[j] = (unsigned)tj < (unsigned)V ? tj : 0;
    }
    if (bad && tid == 0) atomicOr(cell.err, bad);
    float gp[KPB][4], eg[KPB][4], co[KPB];
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        gp[j][g] = cell.gates[(size_t)sr[j] * (4 * HD) + gcol(g, u)];
        eg[j][g] = cell.emb_gates[(size_t)tk[j] * (4 * HD) + gcol(g, u)];
      }
      co[j] = cell.st_old[(size_t)sr[j] * ST + C + HD + u];
    }
    constexpr int QKS = HD / 32;  // k-steps of the query MFMAs
    f16x8 bh[QKS], bl[QKS];
    {
      const float* wb = cell.wq16 + (size_t)wv * (HD / 64) * FRAG;
#pragma unroll
      for (int ks = 0; ks < QKS; ++ks) {
        const float* fb = wb + (size_t)(ks >> 1) * FRAG + (ks & 1) * 512 + ln * 4;
        bh[ks] = *reinterpret_cast<const f16x8*>(fb);
        bl[ks] = *reinterpret_cast<const f16x8*>(fb + 256);
      }
    }
    // (round 4) the first keys batch after the gathers and the W_hidden fragments: a wave's loads
    // retire in issue order, so the cells' wait for their gathers no longer covers the block's whole
    // keys batch (the beam prologue took 13.3 us p50 with the keys issued first, profiles/r04)
    if constexpr (PRE) preload_keys();
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
      float h2 = 0.f, c2;
      if (j < nk) {
        const size_t r = row0 + j;
        lstm_cell_hw(gp[j][0] + eg[j][0], gp[j][1] + eg[j][1], gp[j][2] + eg[j][2], gp[j][3] + eg[j][3], co[j], h2,
                     c2);
        st[r * ST + C + u] = h2;
        st[r * ST + C + HD + u] = c2;
        reinterpret_cast<uint32_t*>(st)[r * ST + ST16 + C + u] = split16_word(h2);
      }
      hs16[j * HS16 + u] = j < nk ? split16_word(h2) : 0u;
    }
    __syncthreads();
    f32x4 qh = {0.f, 0.f, 0.f, 0.f}, qx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < QKS; ++ks) {
      // lane (row ln & 15, g = ln >> 4) of k-step ks: units 64 (ks >> 1) + 16 g + 8 (ks & 1) + e
      // (MFMA rows KPB..15 are zero operands)
      const int hr = ln & 15;
      const uint32_t* hp = hs16 + min(hr, KPB - 1) * HS16 + 64 * (ks >> 1) + 16 * (ln >> 4) + 8 * (ks & 1);
      u32x4 w0 = *reinterpret_cast<const u32x4*>(hp), w1 = *reinterpret_cast<const u32x4*>(hp + 4);
      if (hr >= KPB) w0 = w1 = u32x4{0u, 0u, 0u, 0u};
      f16x8 ah, al;
      unpack16(w0, w1, ah, al);
      mfma_s16(ah, al, bh[ks], bl[ks], qh, qx);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * (ln >> 4) + i, c = 16 * wv + (ln & 15);
      if (j < KPB) {
        const float q = s16_combine(qh[i], qx[i]);
        qs[c * KPB + j] = j < nk ? q : 0.f;
        eqs[c * KPB + j] = j < nk ? split_exp2x(q) : 0.f;
      }
    }
    __syncthreads();  // the score phase overwrites the scratch
  }
  // 1. q = sum of the HD/16 partials in partial order (p = 0, 1, ...), v -> LDS.  The block's
  // KPB rows are consecutive, so partial p of all of them is one contiguous KPB x A span: a thread
  // takes one float4 (row j, columns 4 a4..4 a4 + 3) and has its AT_NQ 16-B loads in flight at
  // once (one round trip; the zero pad rows a >= A take no loads)
  for (int f = tid; !CELL && f < KPB * (A / 4); f += AT_THREADS) {
    const int j = f / (A / 4), a4 = f - j * (A / 4);
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < nk) {
      const float4* qp = reinterpret_cast<const float4*>(qpart + (row0 + j) * A) + a4;
      float4 pv[AT_NQ];
#pragma unroll
      for (int p = 0; p < AT_NQ; ++p) pv[p] = p < nq ? qp[(size_t)p * R * (A / 4)] : make_float4(0.f, 0.f, 0.f, 0.f);
      // 16-unit slots are summed in pairs first: a 32-unit slot (dec_q_slots) holds exactly that
      // pair sum, so q has the same bits whichever LSTMCell shape wrote the partials
      if (nq == AT_NQ) {
#pragma unroll
        for (int p = 0; p < AT_NQ; p += 2)
          q.x += pv[p].x + pv[p + 1].x, q.y += pv[p].y + pv[p + 1].y, q.z += pv[p].z + pv[p + 1].z,
              q.w += pv[p].w + pv[p + 1].w;
      } else {
#pragma unroll
        for (int p = 0; p < AT_NQ / 2; ++p)
          if (p < nq) q.x += pv[p].x, q.y += pv[p].y, q.z += pv[p].z, q.w += pv[p].w;
      }
    }
    qs[(4 * a4 + 0) * KPB + j] = q.x;
    qs[(4 * a4 + 1) * KPB + j] = q.y;
    qs[(4 * a4 + 2) * KPB + j] = q.z;
    qs[(4 * a4 + 3) * KPB + j] = q.w;
    eqs[(4 * a4 + 0) * KPB + j] = j < nk ? split_exp2x(q.x) : 0.f;
    eqs[(4 * a4 + 1) * KPB + j] = j < nk ? split_exp2x(q.y) : 0.f;
    eqs[(4 * a4 + 2) * KPB + j] = j < nk ? split_exp2x(q.z) : 0.f;
    eqs[(4 * a4 + 3) * KPB + j] = j < nk ? split_exp2x(q.w) : 0.f;
  }
  for (int i = tid; i < KPB * (AT_APAD - A); i += AT_THREADS) qs[A * KPB + i] = eqs[A * KPB + i] = 0.f;
  if (tid < A) {
    const float v = vv[tid];
    vs[tid] = v;
    v2s[tid] = -2.f * v;
  }
  __syncthreads();
  stamp(1);

  // 2. scores.  Thread = (a-group ag, 4-step chunk c): its APG keys rows' float4 at chunk c are
  // all loaded before use; partial sums per a-group go to LDS and are added in group order.
  // Split form (ekT, see split_exp2x) unless `direct` or a NaN score sends the block back to the
  // direct tanh(k + q) over keysT.
  // this thread's score work: (a-group, 4-step chunk) items it = tid, tid + 512, ...; each in
  // batches of CH keys rows
  bool nan_seen = false;  // a NaN score of this thread's items (split form: leave it to the direct form)
  auto score_item = [&](int it, bool first, auto&& after_loads, auto SPLIT) {
    constexpr bool split = decltype(SPLIT)::value;
    const int ag = it / nch, c = it - ag * nch, t0 = 4 * c;
    const int a0 = ag * apg, a1 = min(A, a0 + apg);
    const bool live = it < G * nch && t0 < len;
    const float* src = split ? ekb : kb;
    float e4[KPB][4];
    float e0 = 0.f;  // split form: the score starts at the group's sum of v (a order, from LDS)
    if (split && live)
      for (int a = a0; a < a1; ++a) e0 += vs[a];
#pragma unroll
    for (int j = 0; j < KPB; ++j) e4[j][0] = e4[j][1] = e4[j][2] = e4[j][3] = e0;
    // branch-free: a slot past the group's last row gets v = 0 (its keys load is zero-filled and
    // q is padded), so it adds an exact zero and the real terms keep their order; rows j >= nk
    // compute on q = 0 and are never stored
    // one fused multiply-add per term (torch multiplies, then sums in its own order: the score
    // is within the attention tolerance either way; hipcc already contracted the former
    // round-to-nearest intrinsic pairs into these FMAs)
    auto batch = [&](const float4 (&kv)[CH], int ab) {
      if constexpr (split) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const float vm = ab + i < a1 ? v2s[ab + i] : 0.f;
#pragma unroll
          for (int j = 0; j < KPB; ++j) {
            const float ea = eqs[(ab + i) * KPB + j];
            const f32x2 e2 = {ea, ea}, v2 = {vm, vm}, one = {1.f, 1.f};
            const f32x2 dlo = __builtin_elementwise_fma((f32x2){kv[i].x, kv[i].y}, e2, one);
            const f32x2 dhi = __builtin_elementwise_fma((f32x2){kv[i].z, kv[i].w}, e2, one);
            const f32x2 rlo = {__builtin_amdgcn_rcpf(dlo.x), __builtin_amdgcn_rcpf(dlo.y)};
            const f32x2 rhi = {__builtin_amdgcn_rcpf(dhi.x), __builtin_amdgcn_rcpf(dhi.y)};
            const f32x2 a01 = __builtin_elementwise_fma(rlo, v2, (f32x2){e4[j][0], e4[j][1]});
            const f32x2 a23 = __builtin_elementwise_fma(rhi, v2, (f32x2){e4[j][2], e4[j][3]});
            e4[j][0] = a01.x, e4[j][1] = a01.y, e4[j][2] = a23.x, e4[j][3] = a23.y;
          }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const float va = ab + i < a1 ? vs[ab + i] : 0.f;
#pragma unroll
        for (int j = 0; j < KPB; ++j) {
          const float qa = qs[(ab + i) * KPB + j];
          const f32x2 q2 = {qa, qa}, v2 = {va, va};
          const f32x2 lo = tanh_fast2((f32x2){kv[i].x, kv[i].y} + q2);
          const f32x2 hi = tanh_fast2((f32x2){kv[i].z, kv[i].w} + q2);
          const f32x2 a01 = __builtin_elementwise_fma(lo, v2, (f32x2){e4[j][0], e4[j][1]});
          const f32x2 a23 = __builtin_elementwise_fma(hi, v2, (f32x2){e4[j][2], e4[j][3]});
          e4[j][0] = a01.x, e4[j][1] = a01.y, e4[j][2] = a23.x, e4[j][3] = a23.y;
        }
      }
    };
    auto load = [&](float4 (&kv)[CH], int ab) {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        kv[i] = live && ab + i < a1 ? *reinterpret_cast<const float4*>(src + (size_t)(ab + i) * TqG + t0)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    int ab = a0;
    if (first) {  // straight-line first batch: no loop join between its wait and its use
      float4 kv[CH];
      if constexpr (PRE && split) {  // preloaded before the cell phase (it == tid)
#pragma unroll
        for (int i = 0; i < CH; ++i)
          kv[i] = CELL == 0 || (live && ab + i < a1) ? kvp[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        load(kv, ab);
      }
      after_loads();
      if (live) batch(kv, ab);
      ab += CH;
    }
    for (; live && ab < a1; ab += CH) {
      float4 kv[CH];
      load(kv, ab);
      batch(kv, ab);
    }
    if (live)
#pragma unroll
      for (int j = 0; j < KPB; ++j)
        if (j < nk) {
          *reinterpret_cast<float4*>(xs + (ag * KPB + j) * Tq + t0) = make_float4(e4[j][0], e4[j][1], e4[j][2], e4[j][3]);
          if (split)  // steps past len are masked (their keysT / ekT slots may hold anything)
#pragma unroll
            for (int q = 0; q < 4; ++q) nan_seen |= t0 + q < len && e4[j][q] != e4[j][q];
        }
  };
  using SplitT = std::true_type;
  using DirectT = std::false_type;
  // The first batch of keys is loaded and waited for by every wave (a wait hipcc sees), then the
  // value rows 0..npf-1 go to LDS by LDS-DMA (inline asm, hipcc does not see it) and stream in
  // while the block computes tanh scores and the softmax: the chip's HBM is otherwise idle in
  // those phases, since every block runs them at the same time.
  const int nv = min(npf, len);
  auto value_dma = [&]() {
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0): the keys batch has landed
    const uint32_t vbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)vl;
    for (int i = wv; i < 2 * nv; i += AT_WAVES) {  // 1 KB (half a row) per wave instruction
      const float* src = enc + ((size_t)b * Tp + tbase + (i >> 1)) * C + (i & 1) * (C / 2) + 4 * ln;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(vbase + (uint32_t)i * (C / 2) * 4);
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };
  if (!direct) {
    score_item(tid, true, value_dma, SplitT{});
    for (int it = tid + AT_THREADS; it < G * nch; it += AT_THREADS) score_item(it, false, [] {}, SplitT{});
  }
  // direct form: requested, or a NaN score in the block (every thread redoes its own items)
  if (__syncthreads_or(direct || nan_seen)) {
    if (direct) score_item(tid, true, value_dma, DirectT{});
    else score_item(tid, false, [] {}, DirectT{});
    for (int it = tid + AT_THREADS; it < G * nch; it += AT_THREADS) score_item(it, false, [] {}, DirectT{});
    __syncthreads();
  }
  stamp(2);

  // 3. masked softmax over t (torch: exp(x - max), sum, then * 1/sum), one wave per row (KPB <= 8
  // waves): the G group partials combined in group order, the row maximum and the sum by wave
  // reductions, no block barrier until the context phase.  Lane ln takes t = ln, ln + 64, ... in
  // every pass, so a row's arithmetic is the same at every KPB.
  // KPB <= 2 (greedy, k = 2): every thread takes a t and the reductions go through LDS (with one
  // or two rows a single wave's three lane-strided passes were slower: 2.3 against 1.2 us)
  static_assert(KPB <= AT_WAVES, "one wave per beam row of the block");
  float m_split = -INFINITY, z_split = 0.f;  // TSPLIT: this block's softmax maximum and sum
  if constexpr (KPB <= 2) {
    __shared__ float wred[2][AT_WAVES][KPB];
    float lmax[KPB];
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
      lmax[j] = -INFINITY;
      if (j < nk)
        for (int t = tid; t < Tq; t += AT_THREADS) {
          float ev = -INFINITY;
          if (t < len) {
            const float* x = xs + j * Tq + t;
            const int gs = KPB * Tq;
            ev = x[0];
            for (int gg = 1; gg < G; ++gg) ev += x[gg * gs];
          }
          es[t * KPB + j] = ev;
          lmax[j] = fmaxf(lmax[j], ev);
        }
    }
#pragma unroll
    for (int j = 0; j < KPB; ++j)
      if (j < nk) {
        const float m = wave_max(lmax[j]);
        if (ln == 0) wred[0][wv][j] = m;
      }
    __syncthreads();
    float rmax[KPB], lsum[KPB];
#pragma unroll
    for (int j = 0; j < KPB; ++j) {
      float m = -INFINITY;
      if (j < nk)
#pragma unroll
        for (int w = 0; w < AT_WAVES; ++w) m = fmaxf(m, wred[0][w][j]);
      rmax[j] = m;
      lsum[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < KPB; ++j)
      if (j < nk)
        for (int t = tid; t < Tq; t += AT_THREADS) {
          const float p = expf(es[t * KPB + j] - rmax[j]);
          es[t * KPB + j] = p;
          lsum[j] += p;
        }
#pragma unroll
    for (int j = 0; j < KPB; ++j)
      if (j < nk) {
        const float s = wave_sum(lsum[j]);
        if (ln == 0) wred[1][wv][j] = s;
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KPB; ++j)
      if (j < nk) {
        const float s = ((wred[1][0][j] + wred[1][1][j]) + (wred[1][2][j] + wred[1][3][j])) +
                        ((wred[1][4][j] + wred[1][5][j]) + (wred[1][6][j] + wred[1][7][j]));
        if constexpr (TSPLIT) {  // the merge normalises: the context sums exp(e - m_s) v over the block's steps
          m_split = len > 0 ? rmax[j] : -INFINITY;  // (a split past the utterance's end contributes nothing)
          z_split = len > 0 ? s : 0.f;
          continue;
        }
        const float rinv = 1.0f / s;
        for (int t = tid; t < Tq; t += AT_THREADS) {
          const float al = es[t * KPB + j] * rinv;
          es[t * KPB + j] = al;
          if (align && t < Tp) align[(size_t)t * R + row0 + j] = al;
        }
      }
  } else if (wv < nk) {
    const int j = wv;
    const int gs = KPB * Tq;
    float m = -INFINITY;
    for (int t = ln; t < Tq; t += 64) {
      float ev = -INFINITY;
      if (t < len) {
        const float* x = xs + j * Tq + t;
        ev = x[0];
        for (int gg = 1; gg < G; ++gg) ev += x[gg * gs];
      }
      es[t * KPB + j] = ev;
      m = fmaxf(m, ev);
    }
    m = wave_max(m);
    float s = 0.f;
    for (int t = ln; t < Tq; t += 64) {
      const float p = expf(es[t * KPB + j] - m);
      es[t * KPB + j] = p;
      s += p;
    }
    const float rinv = 1.0f / wave_sum(s);
    for (int t = ln; t < Tq; t += 64) {
      const float al = es[t * KPB + j] * rinv;
      es[t * KPB + j] = al;
      if (align && t < Tp) align[(size_t)t * R + row0 + j] = al;
    }
  }
  __syncthreads();

  // 4. context: thread = 4 columns x every 4th t (4 partials, combined in a fixed order); 32
  // value rows in flight per lane
  {
    const int c4 = tid & 127, tp = tid >> 7;
    float acc[KPB][4];
#pragma unroll
    for (int j = 0; j < KPB; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.f;
    const float* eb = enc + ((size_t)b * Tp + tbase) * C + 4 * c4;
    // rows 0..nv-1 from LDS (the DMA issued in the score phase; nv is a multiple of 4 or len, so
    // each thread's t sequence continues unchanged into the global rows: same summation order)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(3);
    // alpha of the KPB rows at step t: one LDS read ([Tq][KPB] layout); t is clamped to Tq - 1,
    // which only slots past len reach, and their value rows are zero-filled, so they add exact zeros
    // (alpha is finite everywhere: 0 past len) and the loop needs no exit test per t
    auto alpha = [&](int t, float (&al)[KPB]) {
      const float* ep = es + min(t, Tq - 1) * KPB;
      if constexpr (KPB % 4 == 0) {
#pragma unroll
        for (int q = 0; q < KPB / 4; ++q) {
          const float4 a4 = *reinterpret_cast<const float4*>(ep + 4 * q);
          al[4 * q] = a4.x, al[4 * q + 1] = a4.y, al[4 * q + 2] = a4.z, al[4 * q + 3] = a4.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < KPB; ++j) al[j] = ep[j];
      }
    };
    auto fma4 = [&](const float (&al)[KPB], const float4& v) {
#pragma unroll
      for (int j = 0; j < KPB; ++j) {
        acc[j][0] = fmaf(al[j], v.x, acc[j][0]);
        acc[j][1] = fmaf(al[j], v.y, acc[j][1]);
        acc[j][2] = fmaf(al[j], v.z, acc[j][2]);
        acc[j][3] = fmaf(al[j], v.w, acc[j][3]);
      }
    };
    int t = tp;
    for (; t < nv; t += 4) {
      const float4 v = *reinterpret_cast<const float4*>(vl + (size_t)t * C + 4 * c4);
      float al[KPB];
      alpha(t, al);
      fma4(al, v);
    }
    constexpr int CT = KPB >= 8 ? 16 : 32;  // value rows in flight per lane (KPB 8: fewer, the accumulators double)
    for (int tb = t; tb < len; tb += 4 * CT) {
      float4 v4[CT];
#pragma unroll
      for (int i = 0; i < CT; ++i) {
        const int t = tb + 4 * i;
        v4[i] = t < len ? *reinterpret_cast<const float4*>(eb + (size_t)t * C) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < CT; ++i) {
        float al[KPB];
        alpha(tb + 4 * i, al);
        fma4(al, v4[i]);
      }
    }
#pragma unroll
    for (int j = 0; j < KPB; ++j)
      if (j < nk)
        *reinterpret_cast<float4*>(xs + (tp * KPB + j) * C + 4 * c4) =
            make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
  }
  stamp(4);
  __syncthreads();
  if constexpr (TSPLIT) {
    // publish (m_s, z_s, c_s) with agent-scope 8-byte stores (coherent across the XCDs' L2s), count
    // in; the last of the utterance's cell.split blocks merges in split order (see the template note)
    __shared__ int last_s;
    const int S = cell.split;
    auto slot = [&](int q) { return reinterpret_cast<uint64_t*>(cell.spart + ((size_t)b * AT_SPLIT_MAX + q) * (C + 4)); };
    uint64_t* mine = slot(sp);
    for (int i = tid; i < C / 4; i += AT_THREADS) {
      const float4 p0 = *reinterpret_cast<const float4*>(xs + (0 * KPB) * C + 4 * i);
      const float4 p1 = *reinterpret_cast<const float4*>(xs + (1 * KPB) * C + 4 * i);
      const float4 p2 = *reinterpret_cast<const float4*>(xs + (2 * KPB) * C + 4 * i);
      const float4 p3 = *reinterpret_cast<const float4*>(xs + (3 * KPB) * C + 4 * i);
      const f32x2 lo = {(p0.x + p1.x) + (p2.x + p3.x), (p0.y + p1.y) + (p2.y + p3.y)};
      const f32x2 hi = {(p0.z + p1.z) + (p2.z + p3.z), (p0.w + p1.w) + (p2.w + p3.w)};
      __hip_atomic_store(mine + 2 * i, __builtin_bit_cast(uint64_t, lo), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mine + 2 * i + 1, __builtin_bit_cast(uint64_t, hi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0)
      __hip_atomic_store(mine + C / 2, __builtin_bit_cast(uint64_t, (f32x2){m_split, z_split}), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store retired before the count (gfx950: vmcnt
                                                      // counts stores; decoder.hip's k-split note)
    __syncthreads();
    if (tid == 0) last_s = __hip_atomic_fetch_add(cell.scnt + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
    __syncthreads();
    if (!last_s) {
      stamp(5);  // (diagnostics) published and counted in
      return;
    }
    float w[AT_SPLIT_MAX];
    float M = -INFINITY, Z = 0.f;
#pragma unroll
    for (int q = 0; q < AT_SPLIT_MAX; ++q)
      if (q < S) {
        const f32x2 mz = __builtin_bit_cast(f32x2, __hip_atomic_load(slot(q) + C / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        w[q] = mz.x;
        M = fmaxf(M, mz.x);
      }
#pragma unroll
    for (int q = 0; q < AT_SPLIT_MAX; ++q)
      if (q < S) {
        const f32x2 mz = __builtin_bit_cast(f32x2, __hip_atomic_load(slot(q) + C / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        w[q] = expf(w[q] - M);  // exp(-inf) = 0 for a split past the end
        Z = q == 0 ? w[q] * mz.y : Z + w[q] * mz.y;
      }
    const float zinv = 1.0f / Z;
    for (int i = tid; i < C / 4; i += AT_THREADS) {
      f32x2 lo = {0.f, 0.f}, hi = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < AT_SPLIT_MAX; ++q)
        if (q < S) {
          const f32x2 a = __builtin_bit_cast(f32x2, __hip_atomic_load(slot(q) + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          const f32x2 c = __builtin_bit_cast(f32x2, __hip_atomic_load(slot(q) + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          lo = q == 0 ? w[q] * a : lo + w[q] * a;
          hi = q == 0 ? w[q] * c : hi + w[q] * c;
        }
      const float4 cv = make_float4(lo.x * zinv, lo.y * zinv, hi.x * zinv, hi.y * zinv);
      *reinterpret_cast<float4*>(st + row0 * ST + 4 * i) = cv;
      *reinterpret_cast<u32x4*>(st + row0 * ST + ST16 + 4 * i) =
          u32x4{split16_word(cv.x), split16_word(cv.y), split16_word(cv.z), split16_word(cv.w)};
    }
    if (tid == 0) __hip_atomic_store(cell.scnt + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    stamp(5);
    return;
  }
  for (int i = tid; i < nk * (C / 4); i += AT_THREADS) {
    const int j = i / (C / 4), c4 = i - j * (C / 4);
    const float4 p0 = *reinterpret_cast<const float4*>(xs + (0 * KPB + j) * C + 4 * c4);
    const float4 p1 = *reinterpret_cast<const float4*>(xs + (1 * KPB + j) * C + 4 * c4);
    const float4 p2 = *reinterpret_cast<const float4*>(xs + (2 * KPB + j) * C + 4 * c4);
    const float4 p3 = *reinterpret_cast<const float4*>(xs + (3 * KPB + j) * C + 4 * c4);
    const float4 cv = make_float4((p0.x + p1.x) + (p2.x + p3.x), (p0.y + p1.y) + (p2.y + p3.y),
                                  (p0.z + p1.z) + (p2.z + p3.z), (p0.w + p1.w) + (p2.w + p3.w));
    *reinterpret_cast<float4*>(st + (row0 + j) * ST + 4 * c4) = cv;
    // the s16 split words of ctx for the next step's decoder GEMMs (casr_internal.h ST16)
    *reinterpret_cast<u32x4*>(st + (row0 + j) * ST + ST16 + 4 * c4) =
        u32x4{split16_word(cv.x), split16_word(cv.y), split16_word(cv.z), split16_word(cv.w)};
  }
  stamp(5);
}

// value rows prefetched into LDS by each block: what fits beside the block's other LDS (156 KiB
// of the 160 KiB per CU, one block per CU), a multiple of 4 rows.  Round 2 measured a smaller
// budget (two blocks per CU) unchanged; the knob was removed in round 3.
static size_t attn_lds_budget() { return (size_t)156 * 1024; }

template <int KPB, int CELL = 0, bool TSPLIT = false>
static int attn_npf(int Tp) {
  const size_t fixed = attn_smem_floats<KPB, CELL, TSPLIT>(Tp) * sizeof(float);
  const size_t budget = attn_lds_budget();
  const size_t room = fixed < budget ? budget - fixed : 0;
  const int rows = (int)(room / (C * sizeof(float))) & ~3;
  return rows < Tp ? rows : (Tp + 3) & ~3;
}

template <int KPB, int CELL = 0>
static hipError_t launch_kpb(const DecodeArgs& a, float* st, const float* qpart, float* align, int32_t* newdone,
                             int l, int total, hipStream_t s, const AttnCell& cell = AttnCell{}) {
  const int npf = attn_npf<KPB, CELL>(a.Tp);
  const size_t shm = (attn_smem_floats<KPB, CELL>(a.Tp) + (size_t)npf * C) * sizeof(float);
  static size_t raised = 0;  // allow > 64 KiB of dynamic LDS (160 KiB per CU on gfx950)
  if (shm > raised) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(attention_kernel<KPB, CELL>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    raised = shm;
  }
  dim3 grid(a.B, (a.k + KPB - 1) / KPB);
  const float* ekT = a.keysT + (size_t)a.B * A * attn_tq(a.Tp);  // KeysEpi: [keys | exp(2 keys)]
  hipLaunchKernelGGL((attention_kernel<KPB, CELL>), grid, dim3(AT_THREADS), shm, s, st, qpart, a.keysT, ekT, a.enc,
                     a.lens, a.W + a.L.v, a.B * a.k, a.k, a.Tp, align, newdone, l, total, npf, a.attn_direct,
                     dec_q_slots(a.B * a.k), a.V, cell);
  return hipGetLastError();
}

// the split folded greedy attention (TSPLIT): cell.split blocks of cell.tc steps per utterance; the
// LDS is sized for cell.tc steps
static hipError_t launch_greedy_split(const DecodeArgs& a, float* st, int32_t* newdone, int l, int total,
                                      hipStream_t s, const AttnCell& cell) {
  if (cell.split < 2 || cell.split > AT_SPLIT_MAX || cell.tc < 4 || cell.tc % 4 || !cell.spart || !cell.scnt)
    return hipErrorInvalidValue;
  const int npf = attn_npf<1, 1, true>(cell.tc);
  const size_t shm = (attn_smem_floats<1, 1, true>(cell.tc) + (size_t)npf * C) * sizeof(float);
  static size_t raised = 0;
  if (shm > raised) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(attention_kernel<1, 1, true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return e;
    raised = shm;
  }
  const float* ekT = a.keysT + (size_t)a.B * A * attn_tq(a.Tp);
  hipLaunchKernelGGL((attention_kernel<1, 1, true>), dim3(a.B, cell.split), dim3(AT_THREADS), shm, s, st, nullptr,
                     a.keysT, ekT, a.enc, a.lens, a.W + a.L.v, a.B, 1, a.Tp, nullptr, newdone, l, total, npf,
                     a.attn_direct, dec_q_slots(a.B), a.V, cell);
  return hipGetLastError();
}

hipError_t launch_attention_cell_step(const DecodeArgs& a, float* st, const AttnCell& cell, float* align,
                                      int32_t* newdone, int l, int total, hipStream_t s) {
  if (a.k == 1 && cell.split > 1 && !align) return launch_greedy_split(a, st, newdone, l, total, s, cell);
  if (a.k == 1) return launch_kpb<1, 1>(a, st, nullptr, align, newdone, l, total, s, cell);
  switch (attention_kpb(a.B, a.k, a.attn_kpb)) {
    case 4:
      if (cell.bsel)
        return a.k == 4 ? launch_kpb<4, 3>(a, st, nullptr, align, newdone, l, total, s, cell)
               : a.k == 8 ? launch_kpb<4, 4>(a, st, nullptr, align, newdone, l, total, s, cell)
                          : hipErrorInvalidValue;
      return launch_kpb<4, 2>(a, st, nullptr, align, newdone, l, total, s, cell);
    case 8:
      if (cell.bsel) return a.k == 8 ? launch_kpb<8, 3>(a, st, nullptr, align, newdone, l, total, s, cell) : hipErrorInvalidValue;
      return launch_kpb<8, 2>(a, st, nullptr, align, newdone, l, total, s, cell);
    default: return hipErrorInvalidValue;  // the folded beam step needs 4 or 8 rows per block
  }
}

// beam rows per block at k > 2 (CASR_OPT_ATTN_KPB, 0 = auto).  4 rows per block at B < 256: 8 rows
// per block (one block per utterance, half the grid at B = 128) measured 3.68 ms vs 2.87 ms per
// B = 128, k = 8 batch, and 2 or 1 rows per block 2.81 / 3.57 ms against 2.80 (round 2).  At B >= 256
// one block per utterance already covers the CUs and streams each utterance's keys and values once
// per step instead of k / 4 times (auto: 8 rows per block there).
int attention_kpb(int B, int k, int opt) {
  if (k == 1) return 1;
  if (k == 2) return 2;
  if (opt == 4 || opt == 8) return opt;
  return B >= 256 && k >= 8 ? 8 : 4;
}

hipError_t launch_attention_step(const DecodeArgs& a, float* st, const float* qpart, float* align,
                                 int32_t* newdone, int l, int total, hipStream_t s) {
  switch (attention_kpb(a.B, a.k, a.attn_kpb)) {
    case 1: return launch_kpb<1>(a, st, qpart, align, newdone, l, total, s);
    case 2: return launch_kpb<2>(a, st, qpart, align, newdone, l, total, s);
    case 8: return launch_kpb<8>(a, st, qpart, align, newdone, l, total, s);
    default: return launch_kpb<4>(a, st, qpart, align, newdone, l, total, s);
  }
}

// the kernel's static LDS (its __shared__ words: 256-336 B), read once from the code object
template <int KPB, int CELL = 0>
static size_t attn_static_bytes() {
  static const size_t v = [] {
    hipFuncAttributes fa{};
    const hipError_t e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(attention_kernel<KPB, CELL>));
    return e == hipSuccess ? (size_t)fa.sharedSizeBytes : (size_t)1024;
  }();
  return v;
}

// LDS of one attention block without the value prefetch (which takes what is left): the dynamic
// area plus the kernel's static words, against the 160 KiB a workgroup may hold
size_t attention_smem_bytes(int B, int k, int Tp, int opt, int cell) {
  switch (attention_kpb(B, k, opt)) {
    case 1:
      return cell == 1 ? attn_smem_floats<1, 1>(Tp) * sizeof(float) + attn_static_bytes<1, 1>()
                       : attn_smem_floats<1>(Tp) * sizeof(float) + attn_static_bytes<1>();
    case 2: return attn_smem_floats<2>(Tp) * sizeof(float) + attn_static_bytes<2>();
    case 8: return attn_smem_floats<8>(Tp) * sizeof(float) + attn_static_bytes<8>();
    default: return attn_smem_floats<4>(Tp) * sizeof(float) + attn_static_bytes<4>();
  }
}

void attn_trace_bind(uint32_t* buf) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_at_trace), &buf, sizeof(buf)); }

}  // namespace casr
