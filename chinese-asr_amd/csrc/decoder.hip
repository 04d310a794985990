// Attention decoder + greedy / beam-search loop on gfx950.
//
// Per decode step l (R = B*k rows, row r = b*k + j as tile_batch lays them out,
// util.py:41-56) four launches, all reading only device state:
//   1. dec_lstm  RNNDecoder.forward cell part (decoder.py:104-114): gates =
//      [embed(tok) | ctx_prev | h_prev] . [W_ih | W_hh]^T + b  (K = 1280), LSTMCell in the
//      epilogue.  Beam reordering (model.py:913-926) is an index: row r reads its
//      predecessor state from row src[r]; nothing is copied.
//   2. attention BauAttn.forward heads == 1 (attention.py:91-95): one block per utterance
//      serves its k beams, so each utterance's keys/values are streamed once per step
//      (the reference re-gathers them per beam: model.py:913-916).
//   3. proj      logit = [h | ctx] . W_p^T + b (decoder.py:129-135).
//   4. select    greedy: log-softmax + first-index argmax + the finished/score bookkeeping of
//      model.py:554-578; beam: top-2k over k*V per utterance with wave shuffles + an LDS
//      merge and the finished/active rules of model.py:834-929.
// The GEMMs use v_mfma_f32_16x16x4_f32 (exact fp32) with weights in MFMA-fragment-major
// order, staged by LDS-DMA (dgemm_kernel).  Early exit (model.py:578 / :897-901) is a
// device-side per-step counter every kernel checks, so the host never synchronises.
#include <float.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "beam_select.h"
#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

// ------------------------------------------------------------------ decode GEMM (LDS-DMA ring)
// C[R][N] = A[R][K] . W^T for the decoder LSTMCell (K = 1280, N = 2048 gate rows) and the
// vocabulary projection (K = 1024, N = 5056).  Block = BM = 16 WR rows x 16 NT columns, 8 waves:
// WR row slabs of 16 x KQ = 8 / WR slices of every 64-deep k tile; the slices are added once at
// the end in a fixed order.  Operand tiles are staged global -> LDS by LDS-DMA
// (global_load_lds_dwordx4) through a ring of S stage buffers, so S - 1 k tiles are in flight
// while one is multiplied:
//   * W tile: NT MFMA-fragment-major blocks (16 rows x 64 k, [q][lane][4]) copied verbatim; a
//     lane's fragment read is lane-linear, conflict-free;
//   * A tile: BM rows x 64 k, 256-B rows, 16-B chunk c of row r at c ^ (r & 15) (XOR on the
//     per-lane DMA source address, same XOR on the read).  The per-lane source address also
//     performs the decoder's row gather (embedding row of tok[r], state row of src[r]).
// At M = R = 256 rows this GEMM is bound by the bytes each CU pulls from L2 / MALL per k tile and
// by their latency (compute per tile is a few hundred cycles), so the ring depth, not the MFMA,
// sets its speed (cdna_hip_programming.md "Pipelining across barriers"):
//   * the S stage buffers are S distinct __shared__ arrays and the k loop is unrolled by S, so
//     each ds_read names one of them and hipcc's own wait before it counts only the DMA into
//     that array (one array with a runtime offset waits for every DMA in flight: the prefetch
//     is serialised);
//   * no __syncthreads() inside the loop (its fence drains every DMA in flight with vmcnt(0)):
//     each wave retires its own DMA of tile kt with a counted s_waitcnt vmcnt, then a raw
//     s_barrier makes everyone's part of tile kt visible and proves tile kt-1's buffer is no
//     longer read, and only then is tile kt+S-1 issued into that buffer.
// Grid: 1-D, XCD-aware.  Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// "Workgroup dispatch": speed only, never correctness), so linear id L runs on XCD L % 8.  All
// NR row blocks of one weight column slice get ids with the same L % 8: the slice is fetched into
// one XCD's L2 once and re-read from there by every row block.
constexpr int DG_BK = 64;
typedef float ks_f2 __attribute__((ext_vector_type(2)));  // (the k split's 8-byte exchange words)
#ifndef CASR_DG_DIAG
#define CASR_DG_DIAG 0
#endif
// (round 5) the projection epilogue's row partials take exp(x - max) as v_exp_f32 of (x - max)
// log2(e) instead of the libm expf (about 15 instructions each, 7 x 16 per lane and block in the beam
// shape); 0 restores expf (diagnostic builds, tools/probes/ab_libs.sh)
// (round 5) the beam logits rows go out with the non-temporal hint: the select re-reads only the
// few tiles that can hold a top-2k candidate (about 16 of 313 per row), so the 41 MB per step need
// no cache residency (three interleaved rounds: beam fused GEMM 3.61-3.63 -> 3.54-3.55 ms per beam
// batch, profiles/r05/logits_nt/); 0 restores plain stores (diagnostic builds)
#ifndef CASR_LOGITS_NT
#define CASR_LOGITS_NT 1
#endif
// NUMERICS (documented in include/casr.h): with CASR_FAST_PART_EXP = 1 every row's Σexp partial,
// hence the greedy accum and each beam row's log-sum-exp, differs from the expf form in the last
// bits (v_exp_f32 is within 1 ulp); tokens are pinned by the oracle tests in both arithmetics
#ifndef CASR_FAST_PART_EXP
#define CASR_FAST_PART_EXP 1
#endif

// The k-split hand-off (dgemm_kernel KS > 1, CASR_OPT_DEC_KSPLIT) orders its agent-scope partial-sum
// stores before the arrival count with vm_wait<0>() alone: on gfx9-family CDNA (gfx950 here) vmcnt
// counts stores as well as loads, so the wait retires the sc1 stores at the coherence point before
// the count is issued.  On gfx10+ stores are counted by vscnt and this would need a release/acquire
// pair (a device-scope fence measured 33 against 19.5 us per step), so any other target is refused.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "decoder.hip: the k-split hand-off assumes gfx950's vmcnt store counting; build for gfx950 only"
#endif

__device__ __forceinline__ bool xcd_tile(int NB, int NR, int& nb, int& rb, int L = -1) {
  if (L < 0) L = blockIdx.x;
  const int x = L & 7, j = L >> 3;
  nb = (j / NR) * 8 + x;
  rb = j % NR;
  return nb < NB;
}

inline unsigned xcd_grid(int NB, int NR) { return (unsigned)(8 * ((NB + 7) / 8) * NR); }

// lds_dma16 (casr_common.h): global_load_lds_dwordx4 from inline asm

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt[3:0], expcnt 7, lgkmcnt 15, vmcnt[5:4] << 14)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// wait until at most n (wave-uniform, 0 <= n) of this wave's vector-memory operations remain
template <int MAXN>
__device__ __forceinline__ void vm_wait_le(int n) {
  if constexpr (MAXN == 0) {
    vm_wait<0>();
  } else {
    if (n >= MAXN) vm_wait<MAXN>();
    else vm_wait_le<MAXN - 1>(n);
  }
}

// diagnostics (CASR_DG_TRACE=<file>, tools/probes/dg_trace.py): per-block s_memrealtime stamps of
// the last decode GEMM launch of each class; null otherwise (one scalar load per block)
__device__ uint32_t* g_dg_trace = nullptr;

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// S16: A rows are split words (split16_word: [emb16 | ctx16 | h16]) and W is the s16 fragment
// image (pack_frag16); a 64-deep tile is 2 k-steps of v_mfma_f32_16x16x32_f16 (s16x3), k-step
// js = 2 kt + j going to wave kq = js % KQ.  Lane (r, g) of step j reads A words 16g + 8j .. +7
// (two swizzled 16-B chunks) and W block [j][hi|lo][lane].
// ntiles: 16-row W fragment blocks that exist; a block's tiles past it re-read the last one (their
// columns are discarded by the epilogue).
// RS, WC (beam shapes): each wave multiplies RS 16-row slabs (so every W fragment it reads from
// LDS feeds RS MFMA rows) by NT / WC of the block's column tiles; KQ = 8 / (WR WC) k slices.
// IL (s16): the next tile's DMA slots are issued between this tile's MFMA groups (one per column
// tile of the wave's first k-step) instead of in one burst after the barrier.
// BKW = 32 (s16 only): each ring stage holds ONE 32-deep k-step instead of a 64-deep tile, so the
// same LDS carries twice the rows or columns (the 256 x 160 beam projection block) or twice the
// stages in flight.  Stage kt is k-step js = kt of the 64-deep form: the same wave (kq = kt % KQ)
// multiplies the same operands in the same order, so both forms give the same bits.  A stage of
// a row is its 8 16-B pieces of words 64 (kt >> 1) + 16 p' + 8 (kt & 1) + {0, 4} (p = 2 p' + {0,1}),
// piece p stored at slot p ^ (row & 7); the W stage is half j = kt & 1 of the fragment block.
// ONE (s16, weights |w| < 16: blob info word 4): one accumulator per tile carrying the whole s16x3
// sum scaled by 2^11, acc += a_hi (w_hi 2^11) + a_hi w_lo' + a_lo' w_hi (w_hi 2^11 formed by one
// v_pk_mul_f16, exact while |w| < 32), as the encoder's input projection (gemm16.hip): half the
// accumulator registers of the (hi.hi, cross) pair, which the 256 x 160 block cannot hold.
// SA > S (the 256-row beam blocks; S = 2): the A tiles get a deeper ring of their own (SA stage
// buffers of A, S of W) and each step issues the next W stage BEFORE the A stage SA - 1 ahead, so the
// counted wait for stage kt retires only W(kt) (and what preceded it) while A(kt + SA - 2) stays in
// flight: the chain waits on a 28 KB W stage instead of a 60 KB [A | W] one.  Same operands, same
// order per element: bitwise equal to SA = S.
// KS > 1 (the greedy folded GEMM at R <= 32, CASR_OPT_DEC_KSPLIT: its 63 blocks of 32 x 112 would
// leave three quarters of the CUs idle): KS blocks per output block, block q of them multiplies the
// 64-deep tiles q nkt / KS .. (q + 1) nkt / KS - 1 (the in-block k slices as usual).  Each epilogue
// wave stores its k-range sum to kspart, and the wave that arrives last at its counter (kscnt,
// agent-scope fences around an atomic add) adds the KS sums in q order, resets the counter and runs
// the epilogue: a fixed order, so the bits do not depend on which block arrives last.
template <int WR, int NT, int S, class ASrc, class Epi, bool S16 = false, int RS = 1, int WC = 1, bool IL = false,
          int BKW = 64, bool ONE = false, int SA = S, int KS = 1>
__global__ __launch_bounds__(512, 2) void dgemm_kernel(int NB, int NR, int ntiles, int nkt,
                                                    const float* __restrict__ Wf, ASrc asrc, Epi epi,
                                                    f32x4* __restrict__ kspart, int* __restrict__ kscnt) {
  constexpr int KQ = 8 / (WR * WC), QPW = 4 / KQ, BM = 16 * WR * RS, NTW = NT / WC;
  static_assert(WR * WC * KQ == 8 && NT % WC == 0 && KQ <= 4, "8 waves = row groups x column groups x k slices");
  constexpr bool B32 = BKW == 32;
  static_assert(BKW == 64 || (B32 && S16), "32-deep stages: s16 images only");
  static_assert(!ONE || S16, "one accumulator: s16 images only");
  constexpr int WFR = B32 ? FRAG / 2 : FRAG;       // W floats of one column tile per stage
  constexpr int RPI = B32 ? 8 : 4, WPI = B32 ? 2 : 4;  // A rows / W DMA instructions per 1 KB DMA
  constexpr int ATILE = BM * BKW, WTILE = NT * WFR;
  constexpr int STG = ATILE + WTILE;          // floats per stage: [A tile | W tile]
  constexpr int NA = BM / RPI, NDMA = NA + WPI * NT;  // DMA instructions per stage: A + W
  constexpr int NSLOT = (NDMA + 7) / 8;      // per wave (at most)
  const int nkb = B32 ? nkt / 2 : nkt;        // 64-deep fragment blocks per W column tile
  static_assert(S >= 2 && S <= 6, "ring of 2..6 stage buffers");
  static_assert((S * STG + (SA - S) * ATILE) * 4 <= 160 * 1024, "ring fits the LDS");
  static_assert((S - 2) * NSLOT < 64, "vmcnt range");
  constexpr bool ASYM = SA > S;
  constexpr int JA = NA / 8;  // ASYM: slots j < JA are A DMAs in every wave, the rest W
  static_assert(!ASYM || (S == 2 && SA <= 4 && NA % 8 == 0 && JA < NSLOT), "deeper A ring: S = 2, whole A slots");
  static_assert(KS == 1 || (!ASYM && !B32 && KQ > 1), "k split: the 64-deep ring, k slices exchanged in LDS");
  __shared__ __attribute__((aligned(16))) float lb0[STG];
  __shared__ __attribute__((aligned(16))) float lb1[STG];
  __shared__ __attribute__((aligned(16))) float lb2[S > 2 ? STG : 4];
  __shared__ __attribute__((aligned(16))) float lb3[S > 3 ? STG : 4];
  __shared__ __attribute__((aligned(16))) float lb4[S > 4 ? STG : 4];
  __shared__ __attribute__((aligned(16))) float lb5[S > 5 ? STG : 4];
  __shared__ __attribute__((aligned(16))) float lx0[SA > S ? ATILE : 4];  // ASYM: A stage buffers S, S + 1
  __shared__ __attribute__((aligned(16))) float lx1[SA > S + 1 ? ATILE : 4];
  // ASYM: A slot a of the A ring (A part of lb0 / lb1, then lx0, lx1); W slot of the W ring: lb0 / lb1
  auto abuf = [&](auto I) -> float* {
    if constexpr (I == 0) return lb0;
    else if constexpr (I == 1) return lb1;
    else if constexpr (I == 2) return lx0;
    else return lx1;
  };
  auto buf = [&](auto I) -> float* {
    if constexpr (I == 0) return lb0;
    else if constexpr (I == 1) return lb1;
    else if constexpr (I == 2) return lb2;
    else if constexpr (I == 3) return lb3;
    else if constexpr (I == 4) return lb4;
    else return lb5;
  };
  int nb, rb;
  const int ksq = KS > 1 ? (int)(blockIdx.x % KS) : 0;  // this block's k range of the output block
  if (!xcd_tile(NB, NR, nb, rb, KS > 1 ? (int)(blockIdx.x / KS) : -1)) return;
  const int nktl = nkt / KS, kofs = ksq * nktl;  // 64-deep tiles of this block, the first one
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, ws = w % WR, wc = (w / WR) % WC, kq = w / (WR * WC);
  uint32_t* dtr = g_dg_trace ? g_dg_trace + ((size_t)Epi::kTraceClass * 4096 + blockIdx.x) * 8 : nullptr;
  auto stamp = [&](int i) {
    if (dtr && tid == 0) dtr[i] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (dtr && tid == 0) {  // the block's tile (words 5, 6) and the launch's column block count (7)
    dtr[5] = (uint32_t)nb;
    dtr[6] = (uint32_t)rb;
    dtr[7] = (uint32_t)NB;
  }
  const int r = lane & 15, g = lane >> 4;
  const int cnt_w = w < NDMA ? (NDMA - w + 7) / 8 : 0;  // DMA instructions this wave issues per stage

  // the A source's own prologue (DecLstmA with a fused greedy select: the tokens of this block's
  // rows, into LDS, before any row is bound); block-uniform, ends with a barrier when it runs
  asrc.template prologue<BM>(rb * BM, nb == 0);
  // per-lane DMA sources that do not depend on k: A row segment bases, W fragment block bases
  int bad = 0;
  // (a source with one segment (kSeg == 0) keeps one pointer per slot; W sources are 32-bit
  // offsets from Wf: registers the 256 x 160 block needs for its accumulators)
  // (one-segment sources: 32-bit offsets from the source's row 0 as well)
  constexpr int NSEG = ASrc::kSeg > 0 ? 2 : 1;
  constexpr bool AOFF = NSEG == 1;
  const float* aseg[AOFF ? 1 : NSLOT][NSEG];
  uint32_t aoff[AOFF ? NSLOT : 1];
  const float* abase = nullptr;
  if constexpr (AOFF) {
    const float* s1;
    int unused = 0;
    asrc.bind(0, abase, s1, unused);
  }
  uint32_t woff[NSLOT];
#pragma unroll
  for (int j = 0; j < NSLOT; ++j) {
    const int i = w + 8 * j;
    woff[j] = 0;
    if constexpr (AOFF) aoff[j] = 0;
    else
#pragma unroll
      for (int q = 0; q < NSEG; ++q) aseg[j][q] = nullptr;
    if (i < NA) {
      const float* s0;
      const float* s1;
      asrc.bind(rb * BM + RPI * i + lane / (64 / RPI), s0, s1, bad);
      if constexpr (AOFF) {
        aoff[j] = (uint32_t)(s0 - abase);
      } else {
        aseg[j][0] = s0;
        aseg[j][NSEG - 1] = s1;
      }
    } else if (i < NDMA) {
      const int tn = (i - NA) / WPI, qq = (i - NA) % WPI;
      int t = nb * NT + tn;
      t = t < ntiles ? t : ntiles - 1;
      woff[j] = (uint32_t)(t * nkb * FRAG + qq * 256 + lane * 4);
    }
  }
  // dst: the stage's [A | W] buffer, or (ASYM) da / dw: its A and W buffers
  auto stage_slot2 = [&](float* la, float* lw, int kt, auto J) {
    constexpr int j = decltype(J)::value;
    if constexpr (j < NSLOT) {
      const int kb = (B32 ? kt >> 1 : kt) + kofs, k0 = kb * 64;
      const int i = w + 8 * j;
      if (i < NA) {
        const float* seg;
        if constexpr (AOFF) seg = abase + aoff[j] + k0;
        else seg = k0 < ASrc::kSeg ? aseg[j][0] + k0 : aseg[j][NSEG - 1] + (k0 - ASrc::kSeg);
        if constexpr (B32) {
          const int row = 8 * i + (lane >> 3), p = (lane & 7) ^ (row & 7);
          if constexpr ((CASR_DG_DIAG & 128) != 0)  // diagnostic: the stage's 128 B of a row contiguous (wrong data)
            lds_dma16(seg + 32 * (kt & 1) + 4 * p, la + i * 256);
          else
            lds_dma16(seg + 16 * (p >> 1) + 8 * (kt & 1) + 4 * (p & 1), la + i * 256);
        } else {
          const int row = 4 * i + (lane >> 4), c = (lane & 15) ^ (row & 15);
          lds_dma16(seg + c * 4, la + i * 256);
        }
      } else if (i < NDMA) {
        const int tn = (i - NA) / WPI, qq = (i - NA) % WPI;
        lds_dma16(Wf + woff[j] + (size_t)kb * FRAG + (B32 ? (kt & 1) * 512 : 0), lw + tn * WFR + qq * 256);
      }
    }
  };
  auto stage_slot = [&](float* dst, int kt, auto J) { stage_slot2(dst, dst + ATILE, kt, J); };
  auto stage = [&](float* dst, int kt) { static_for<0, NSLOT>([&](auto J) { stage_slot(dst, kt, J); }); };
  constexpr bool ILS = IL && S16;

  f32x4 acc[RS][NTW], accx[ONE ? 1 : RS][ONE ? 1 : NTW];
#pragma unroll
  for (int rs = 0; rs < RS; ++rs)
#pragma unroll
    for (int tn = 0; tn < NTW; ++tn) {
      acc[rs][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (!ONE) accx[rs][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  auto arow = [&](int rs) { return (ws * RS + rs) * 16 + r; };
  auto compute2 = [&](const float* la, const float* lw0, int kt, auto&& issue) {
    const float* lw = lw0 + wc * NTW * WFR;
    if constexpr (S16) {
      bool pend = ILS;  // DMA slots of the next tile not issued yet (wave-uniform)
#pragma unroll
      for (int j = 0; j < (B32 ? 1 : 2); ++j) {
        if ((B32 ? kt : 2 * kt + j) % KQ != kq) continue;
        f16x8 ah[RS], al[RS];
#pragma unroll
        for (int rs = 0; rs < RS; ++rs) {
          const int ar = arow(rs);
          u32x4 w0, w1;
          if constexpr (B32) {  // pieces 2g, 2g + 1 of the row's stage
            w0 = *reinterpret_cast<const u32x4*>(la + ar * 32 + (((2 * g) ^ (ar & 7)) << 2));
            w1 = *reinterpret_cast<const u32x4*>(la + ar * 32 + (((2 * g + 1) ^ (ar & 7)) << 2));
          } else {
            const int c0 = 4 * g + 2 * j;
            w0 = *reinterpret_cast<const u32x4*>(la + ar * DG_BK + ((c0 ^ (ar & 15)) << 2));
            w1 = *reinterpret_cast<const u32x4*>(la + ar * DG_BK + (((c0 + 1) ^ (ar & 15)) << 2));
          }
          unpack16(w0, w1, ah[rs], al[rs]);
        }
        static_for<0, NTW>([&](auto TN) {
          constexpr int tn = decltype(TN)::value;
          const int jw = B32 ? 0 : 2 * j;  // the stage's W half: [hi | lo][lane][8 halves]
          const f16x8 bh = *reinterpret_cast<const f16x8*>(lw + tn * WFR + jw * 256 + lane * 4);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(lw + tn * WFR + (jw + 1) * 256 + lane * 4);
          if constexpr (ONE) {
            const f16x8 b1 = bh * (_Float16)2048.0f;
#pragma unroll
            for (int rs = 0; rs < RS; ++rs) {
              acc[rs][tn] = mfma16x16x32h(ah[rs], b1, acc[rs][tn]);
              if constexpr (kS16Cross) {
                acc[rs][tn] = mfma16x16x32h(ah[rs], bl, acc[rs][tn]);
                acc[rs][tn] = mfma16x16x32h(al[rs], bh, acc[rs][tn]);
              }
            }
          } else {
#pragma unroll
            for (int rs = 0; rs < RS; ++rs) mfma_s16(ah[rs], al[rs], bh, bl, acc[rs][tn], accx[rs][tn]);
          }
          if constexpr (ILS) {
            if (pend) issue(TN);
          }
        });
        if constexpr (ILS) {
          if (pend) static_for<NTW, NSLOT>(issue);
          pend = false;
        }
      }
      if constexpr (ILS) {
        if (pend) static_for<0, NSLOT>(issue);  // no k-step of this tile is this wave's
      }
      return;
    }
#pragma unroll
    for (int qh = 0; qh < QPW; ++qh) {
      const int q = kq * QPW + qh;
      float4 a[RS];
#pragma unroll
      for (int rs = 0; rs < RS; ++rs) {
        const int ar = arow(rs);
        a[rs] = *reinterpret_cast<const float4*>(la + ar * DG_BK + (((4 * g + q) ^ (ar & 15)) << 2));
      }
      float4 b[NTW];
#pragma unroll
      for (int tn = 0; tn < NTW; ++tn) b[tn] = *reinterpret_cast<const float4*>(lw + tn * FRAG + q * 256 + lane * 4);
#pragma unroll
      for (int rs = 0; rs < RS; ++rs)
#pragma unroll
        for (int tn = 0; tn < NTW; ++tn) {
          acc[rs][tn] = mfma16x16x4(a[rs].x, b[tn].x, acc[rs][tn]);
          acc[rs][tn] = mfma16x16x4(a[rs].y, b[tn].y, acc[rs][tn]);
          acc[rs][tn] = mfma16x16x4(a[rs].z, b[tn].z, acc[rs][tn]);
          acc[rs][tn] = mfma16x16x4(a[rs].w, b[tn].w, acc[rs][tn]);
        }
    }
  };
  auto compute = [&](const float* src, int kt, auto&& issue) { compute2(src, src + ATILE, kt, issue); };

  if constexpr (ASYM) {
    // issue order A(0), W(0), A(1) .. A(SA - 2): each later step issues W(kt + 1), then A(kt + SA - 1)
    static_for<0, JA>([&](auto J) { stage_slot2(abuf(std::integral_constant<int, 0>{}), lb0, 0, J); });
    static_for<JA, NSLOT>([&](auto J) { stage_slot2(lb0, lb0 + ATILE, 0, J); });
    static_for<1, SA - 1>([&](auto I) {
      if (I < nkt) static_for<0, JA>([&](auto J) { stage_slot2(abuf(I), lb0, I, J); });
    });
  } else {
    static_for<0, S - 1>([&](auto I) {
      if (I < nktl) stage(buf(I), I);
    });
  }
  // after the first ring stages are in flight: the epilogue's operands (bias, predecessor rows,
  // W_hidden), loaded under the k loop, and the early-exit check (its wait also retires those
  // stages: a skipped block leaves no DMA behind)
  auto erow0 = [&](int rs) { return rb * BM + (ws * RS + rs) * 16 + 4 * (lane >> 4); };
  const int nbw = nb * WC + wc;  // the wave's column block in units of NTW tiles (the epilogue's nb)
  // (an epilogue whose prefetched operands do not depend on the rows (kPreRowFree: the column biases)
  // loads them once for all RS slabs: registers the 256-row blocks need for their accumulators)
  constexpr int NPRE = Epi::kPreRowFree ? 1 : RS;
  typename Epi::Pre pre[NPRE];
  if (kq == 0)
#pragma unroll
    for (int rs = 0; rs < NPRE; ++rs) epi.template prefetch<NTW>(pre[rs], erow0(rs), nbw, lane & 15, bad);
  if (epi.skip()) return;
  if (bad) atomicOr(epi.err_flags(), bad);
  stamp(1);
  if constexpr (ASYM) {
    // unrolled by the W ring's period; the A buffer is picked at run time (wave-uniform): the DMAs are
    // inline asm, so hipcc adds no wait for them whatever it can prove about the buffers
    auto abuf_rt = [&](int a) -> float* { return a == 0 ? lb0 : a == 1 ? lb1 : a == 2 ? lx0 : lx1; };
    for (int kt0 = 0; kt0 < nkt; kt0 += 2) {
      static_for<0, 2>([&](auto I) {
        const int kt = kt0 + I;
        if (kt >= nkt) return;
        // W(kt) was issued at step kt - 1, followed only by that step's A(kt + SA - 2)
        vm_wait_le<JA>(kt + SA - 2 < nkt ? JA : 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // issue position p: W slots first (p < NSLOT - JA), then A
        auto issue = [&](auto P) {
          constexpr int p = decltype(P)::value, j = (p + JA) % NSLOT;
          if constexpr (j >= JA) {
            if (kt + 1 < nkt && !(CASR_DG_DIAG & 1))
              stage_slot2(lb0, buf(std::integral_constant<int, (I + 1) % 2>{}) + ATILE, kt + 1,
                          std::integral_constant<int, j>{});
          } else {
            if (kt + SA - 1 < nkt && !(CASR_DG_DIAG & 1))
              stage_slot2(abuf_rt((kt + SA - 1) % SA), lb0, kt + SA - 1, std::integral_constant<int, j>{});
          }
        };
        if constexpr (!ILS) static_for<0, NSLOT>(issue);
        if (kt == 0) stamp(2);
        if (!(CASR_DG_DIAG & 2))
          compute2(abuf_rt(kt % SA), buf(std::integral_constant<int, I % 2>{}) + ATILE, kt, issue);
        else if constexpr (ILS) static_for<0, NSLOT>(issue);
      });
    }
  }
  for (int kt0 = 0; !ASYM && kt0 < nktl; kt0 += S) {
    static_for<0, S>([&](auto I) {
      const int kt = kt0 + I;
      if (kt >= nktl) return;
      // this wave's DMA of tile kt is done once at most (tiles issued after it) x cnt_w remain
      const int ahead = min(S - 2, nktl - 1 - kt);
      vm_wait_le<(S - 2) * NSLOT>(ahead * cnt_w);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of tile kt-1 are done
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");  // no LDS read of tile kt moves above the barrier
      // CASR_DG_DIAG (diagnostic builds, tools/probes): bit 0 drops the k loop's DMA, bit 1 the MFMAs
      auto issue = [&](auto J) {
        if (kt + S - 1 < nktl && !(CASR_DG_DIAG & 1))
          stage_slot(buf(std::integral_constant<int, (I + S - 1) % S>{}), kt + S - 1, J);
      };
      if constexpr (!ILS) static_for<0, NSLOT>(issue);
      if (kt == 0) stamp(2);
      if (!(CASR_DG_DIAG & 2)) compute(buf(I), kt, issue);
      else if constexpr (ILS) static_for<0, NSLOT>(issue);
    });
  }
  __syncthreads();  // nothing in flight any more: every wave is done reading the ring
  stamp(3);
  if (kq == 0)
#pragma unroll
    for (int rs = 0; rs < NPRE; ++rs) epi.template late<NTW>(pre[rs], erow0(rs), nbw, lane & 15);  // under the k-slice exchange
  if constexpr (S16) {
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
      for (int tn = 0; tn < NTW; ++tn)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (ONE) acc[rs][tn][e] *= S16_LO_INV;
          else acc[rs][tn][e] = s16_combine(acc[rs][tn][e], accx[rs][tn][e]);
        }
  }
  // k slices 1..KQ-1 hand their partial sums to slice 0 through LDS (the ring is free now)
  if constexpr (KQ > 1) {
    // partial slots in lb0, continued in lb2 when they outgrow one stage buffer (32-row
    // projection blocks: 3 x 2 x 5 tiles); the epilogue below uses lb1 (and lb0 for waves >= 4)
    constexpr int CAP = STG * 4 / 16, NPART = (KQ - 1) * WR * WC * RS * NTW * 64;
    static_assert(NPART <= CAP || (S > 2 && NPART <= 2 * CAP), "partials fit lb0 (+ lb2)");
    static_assert(NPART <= CAP || WR * WC <= 4, "with lb2 in use the epilogue waves stay on lb1");
    auto part = [&](int j, int rs, int tn) -> f32x4& {
      const int i = ((((j * WR + ws) * WC + wc) * RS + rs) * NTW + tn) * 64 + lane;
      if constexpr (NPART <= CAP) return reinterpret_cast<f32x4*>(lb0)[i];
      else return i < CAP ? reinterpret_cast<f32x4*>(lb0)[i] : reinterpret_cast<f32x4*>(lb2)[i - CAP];
    };
    if (kq > 0) {
#pragma unroll
      for (int rs = 0; rs < RS; ++rs)
#pragma unroll
        for (int tn = 0; tn < NTW; ++tn) part(kq - 1, rs, tn) = acc[rs][tn];
    }
    __syncthreads();
    if (kq > 0) return;
#pragma unroll
    for (int j = 0; j < KQ - 1; ++j)
#pragma unroll
      for (int rs = 0; rs < RS; ++rs)
#pragma unroll
        for (int tn = 0; tn < NTW; ++tn) acc[rs][tn] += part(j, rs, tn);
  }
  if constexpr (KS > 1) {  // the KS k ranges of this wave's rows and columns, summed in q order
    // agent-scope (sc1) 8-byte stores and loads, as the recurrence's hand-off words: coherent across
    // the XCDs' L2s without the L2 write-back / invalidate a device-scope fence costs (measured: the
    // fenced form took 33 us per step against 19.5 for the unsplit GEMM)
    const size_t gi = ((size_t)rb * NB + nb) * (WR * WC) + ws * WC + wc;
    uint64_t* pk = reinterpret_cast<uint64_t*>(kspart + gi * (KS * RS * NTW * 64)) + 2 * lane;
    auto slot = [&](int qq, int rs, int tn) { return pk + (size_t)((qq * RS + rs) * NTW + tn) * 128; };
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
      for (int tn = 0; tn < NTW; ++tn) {
        const f32x4 v = acc[rs][tn];
        uint64_t* p = slot(ksq, rs, tn);
        __hip_atomic_store(p, __builtin_bit_cast(uint64_t, (ks_f2){v[0], v[1]}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p + 1, __builtin_bit_cast(uint64_t, (ks_f2){v[2], v[3]}), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    vm_wait<0>();  // the sums are stored before the count (gfx9 vmcnt counts stores: see the #error above)
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(kscnt + gi, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0);
    if (old != KS - 1) return;
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
      for (int tn = 0; tn < NTW; ++tn) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int qq = 0; qq < KS; ++qq) {
          const uint64_t* p = slot(qq, rs, tn);
          const ks_f2 lo = __builtin_bit_cast(ks_f2, __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          const ks_f2 hi = __builtin_bit_cast(ks_f2, __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          const f32x4 w = {lo[0], lo[1], hi[0], hi[1]};
          v = qq == 0 ? w : v + w;
        }
        acc[rs][tn] = v;
      }
    if (lane == 0) __hip_atomic_store(kscnt + gi, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  }
  // lane holds rows erow0(rs) + e (e = 0..3), column (nbw*NTW + tn)*16 + r
  // per-wave LDS scratch for the epilogue (ring buffers are free now; the k-slice exchange
  // above used lb0 (only when KQ > 1, i.e. at most 4 epilogue waves, all on lb1)): 16 rows x
  // (16 NTW + 4) floats per epilogue wave, reused by its RS slabs in turn (LDS is in order per wave)
  static_assert(!Epi::kScratch || 4 * 16 * (16 * NTW + 4) <= STG, "epilogue slabs fit a stage buffer");
  const int ew = ws * WC + wc;
  float* escr = (ew < 4 ? lb1 : lb0) + (ew & 3) * 16 * (16 * NTW + 4);
#pragma unroll
  for (int rs = 0; rs < RS; ++rs) epi.template run<NTW>(acc[rs], erow0(rs), nbw, r, pre[NPRE == 1 ? 0 : rs], escr);
  stamp(4);
}

template <int WR, int NT, int S, int RS = 1, int WC = 1, bool IL = false, int BKW = 64, bool ONE = false, int SA = S,
          int KS = 1, class ASrc, class Epi>
static void launch_dg(int NB, int R, int ntiles, int nkt, const float* Wf, const ASrc& asrc, const Epi& epi,
                      int s16, hipStream_t s, f32x4* kspart = nullptr, int* kscnt = nullptr) {
  constexpr int BM = 16 * WR * RS;
  const int NR = (R + BM - 1) / BM;
  if constexpr (KS > 1) {  // (64-deep stages, nkt % KS == 0: the host's check)
    if (s16)
      hipLaunchKernelGGL((dgemm_kernel<WR, NT, S, ASrc, Epi, true, RS, WC, IL, 64, false, S, KS>),
                         dim3(xcd_grid(NB, NR) * KS), dim3(512), 0, s, NB, NR, ntiles, nkt, Wf, asrc, epi, kspart, kscnt);
    else
      hipLaunchKernelGGL((dgemm_kernel<WR, NT, S, ASrc, Epi, false, RS, WC, false, 64, false, S, KS>),
                         dim3(xcd_grid(NB, NR) * KS), dim3(512), 0, s, NB, NR, ntiles, nkt, Wf, asrc, epi, kspart, kscnt);
    return;
  }
  if constexpr (BKW == 32 || ONE) {  // s16 only (the f32 form of the same shape does not fit the LDS)
    hipLaunchKernelGGL((dgemm_kernel<WR, NT, S, ASrc, Epi, true, RS, WC, IL, BKW, ONE, SA>), dim3(xcd_grid(NB, NR)),
                       dim3(512), 0, s, NB, NR, ntiles, nkt * (64 / BKW), Wf, asrc, epi, nullptr, nullptr);
  } else {
    if (s16)
      hipLaunchKernelGGL((dgemm_kernel<WR, NT, S, ASrc, Epi, true, RS, WC, IL>), dim3(xcd_grid(NB, NR)), dim3(512), 0,
                         s, NB, NR, ntiles, nkt, Wf, asrc, epi, nullptr, nullptr);
    else
      hipLaunchKernelGGL((dgemm_kernel<WR, NT, S, ASrc, Epi, false, RS, WC>), dim3(xcd_grid(NB, NR)), dim3(512), 0, s,
                         NB, NR, ntiles, nkt, Wf, asrc, epi, nullptr, nullptr);
  }
}

// A rows of the decoder LSTM: [embed(tok[r]) | st_old[src[r]][0:1024] = ctx | h]; a 64-deep
// k tile lies in one segment (E = 256 is a multiple of 64).  Rows >= R read row R-1 (unused).
// s16: emb is the split-word table (emb16) and the state segment starts at ST16 ([ctx16 | h16]).
// Greedy select of step lsel fused into the next step's LSTMCell (run_greedy): the partials of
// the projection (GreedyPart, one per 80-column block) are reduced by the LSTMCell blocks
// themselves, each for its own rows, so no select launch (and no kernel boundary) sits between
// the projection and the next LSTMCell.  Every column block of a row block computes its rows'
// tokens (32 rows x 64 partials); the block with nb == 0 also does the bookkeeping of
// greedy_select_part_kernel (tokens, finished, lengths, score, newdone), with the same
// arithmetic, so both forms give the same bits.
// (GreedySel, greedy_book: casr_internal.h)
__device__ __forceinline__ int* sel_tok_lds() {
  __shared__ int t[128];
  return t;
}

struct DecLstmA {
  static constexpr int kSeg = E;  // k < kSeg: embedding row, else state row
  const float* emb;
  const float* st_old;
  const int32_t* tok;
  const int32_t* src;
  int32_t* err;
  int R, V, s16;
  int sel = 0;  // 1: tokens from the fused greedy select of step gs.lsel (prologue)
  GreedySel gs = {};
  // every load of the wave's BM / 8 rows (partials, and for the writer the bookkeeping state) is
  // issued before the first reduction: one round trip for the block, not one per row
  template <int BM>
  __device__ __forceinline__ void prologue(int row0, bool writer) const {
    static_assert(128 % BM == 0, "row blocks tile the fused select's 128 token slots");
    if (!sel) return;
    constexpr int RPW = BM / 8;  // rows per wave
    int* st = sel_tok_lds();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float m[RPW], se[RPW], acc0[RPW];
    int mi[RPW], len0[RPW];
    uint8_t fin0[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = row0 + w + 8 * i;
      m[i] = -INFINITY, se[i] = 0.f, mi[i] = 0x7fffffff;
      acc0[i] = 0.f, len0[i] = 0, fin0[i] = 0;
      if (r < R && lane < gs.nbp) {
        m[i] = gs.gp.mx[(size_t)r * GP_NB + lane];
        se[i] = gs.gp.se[(size_t)r * GP_NB + lane];
        mi[i] = gs.gp.ix[(size_t)r * GP_NB + lane];
      }
      if (writer && r < R && lane == 0) {
        fin0[i] = gs.fin[r];
        acc0[i] = gs.accum[r];
        len0[i] = gs.out_len[r];
      }
    }
    const bool all_done = done_before(gs.newdone, gs.lsel) >= R;  // greedy_select_part_kernel's skip
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = row0 + w + 8 * i;
      if (r >= R) break;
      if (all_done) {  // every row finished before step lsel: nothing downstream runs any more
        if (lane == 0) st[r & 127] = 0;
        continue;
      }
      float gm = m[i];
      int gi = mi[i];
      wave_best(gm, gi);
      int t = gi;
      const bool bad_t = (unsigned)t >= (unsigned)V;  // no finite maximum (NaN row)
      if (bad_t) t = 0;
      if (lane == 0) st[r & 127] = t;  // BM divides 128 and row0: distinct slots
      if (!writer) continue;
      const float sx = wave_sum((se[i] > 0.f) ? se[i] * expf(m[i] - gm) : 0.f);
      if (lane != 0) continue;
      if (bad_t) atomicOr(err, CASR_DEV_NAN_LOGITS);
      const float lp = gm - (logf(sx) + gm);
      greedy_book(gs, r, t, lp, fin0[i], acc0[i], len0[i]);
    }
    __syncthreads();
  }
  // branch-free (a branch on a loaded index would serialise the prologue's loads: one round
  // trip each); bad indices are clamped and reported through `bad` (CASR_DEV_* bits)
  __device__ __forceinline__ void bind(int row, const float*& seg0, const float*& seg1, int& bad) const {
    row = row < R ? row : R - 1;
    const int t = sel ? sel_tok_lds()[row & 127] : tok[row];
    const bool bt = (unsigned)t >= (unsigned)V;
    bad |= bt ? CASR_DEV_BAD_TOKEN : 0;
    seg0 = emb + (size_t)(bt ? 0 : t) * E;
    seg1 = st_old + (size_t)safe_src(row, bad) * ST + (s16 ? ST16 : 0);
  }
  __device__ __forceinline__ int safe_src(int row, int& bad) const {
    const int s = src[row];
    const bool bs = (unsigned)s >= (unsigned)R;
    bad |= bs ? CASR_DEV_BAD_SRC : 0;
    return bs ? row : s;
  }
};

struct DecLstmEpi {
  static constexpr int kTraceClass = 0;
  static constexpr bool kPreRowFree = false;  // predecessor rows and c per row slab
  static constexpr bool kScratch = false;  // the epilogue's LDS: its own h tiles (ht), no slab
  const float* bias;  // packed [4HD]
  const float* st_old;
  float* st_new;
  DecLstmA rows;      // guarded predecessor lookup
  const int32_t* newdone;
  const float* w_hidden;  // [HD][A]
  float* qpart;           // [dec_q_slots(R)][R][A]
  int R, l, total;
  int hw = 0;  // s16x3 arithmetic: the hardware-exp cell (casr_common.h lstm_cell_hw, as the encoder's)
  // operands loaded before the k loop: gate biases, predecessor rows, this lane's W_hidden
  // fragments of the query partial (A/16 x 4 MFMA steps); c of the predecessor after it.  A block
  // of NTN = 4 UG column tiles holds UG 16-unit groups (4 gate tiles each): [i f g o] of units
  // 16 (nb UG + ug) ..+15 (the packed gate-row order)
  static constexpr int UGMAX = 2;
  struct Pre {
    float bg[UGMAX][4];
    int srow[4];
    float wh[UGMAX][A / 16][4];
    float cold[UGMAX][4];
  };
  __device__ __forceinline__ bool skip() const { return done_before(newdone, l) >= total; }
  __device__ __forceinline__ int32_t* err_flags() const { return rows.err; }
  template <int NTN>
  __device__ __forceinline__ void prefetch(Pre& p, int row0, int nb, int u, int& bad) const {
    constexpr int UG = NTN / 4;
    const int lane = threadIdx.x & 63, g = lane >> 4;
#pragma unroll
    for (int ug = 0; ug < UG; ++ug)
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) p.bg[ug][gt] = bias[(nb * UG + ug) * 64 + gt * 16 + u];
#pragma unroll
    for (int e = 0; e < 4; ++e) p.srow[e] = rows.safe_src(min(row0 + e, R - 1), bad);
#pragma unroll
    for (int ug = 0; ug < UG; ++ug) {
      const float* wp = w_hidden + (size_t)((nb * UG + ug) * 16 + g) * A + (lane & 15);
#pragma unroll
      for (int at = 0; at < A / 16; ++at)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) p.wh[ug][at][kk] = wp[(size_t)(4 * kk) * A + at * 16];
    }
  }
  template <int NTN = 4>
  __device__ __forceinline__ void late(Pre& p, int row0, int nb, int u) const {
    constexpr int UG = NTN / 4;
#pragma unroll
    for (int ug = 0; ug < UG; ++ug) {
      const int U = (nb * UG + ug) * 16 + u;
#pragma unroll
      for (int e = 0; e < 4; ++e) p.cold[ug][e] = st_old[(size_t)p.srow[e] * ST + C + HD + U];
    }
  }
  template <int NTN = 4>
  __device__ __forceinline__ void run(const f32x4 (&acc)[NTN], int row0, int nb, int u, const Pre& p, float*) const {
    static_assert(NTN % 4 == 0 && NTN / 4 <= UGMAX, "the LSTM cell needs the 4 gate tiles of each 16-unit group");
    constexpr int UG = NTN / 4;
    // per row-slab wave (<= 8 per block): the h tile [row][unit] of its UG unit groups.  The query
    // partial of each 16-unit group is its own MFMA chain; a two-group block stores their sum in
    // slot nb (dec_q_slots), which is the pair sum the attention forms from two 16-unit slots, so
    // q has the same bits at every R
    __shared__ float ht[8][16][16 * UG + 1];
    const int lane = threadIdx.x & 63, ws = (row0 >> 4) & 7, g = lane >> 4;
    const int rbase = row0 - 4 * g;  // first row of this wave's slab
#pragma unroll
    for (int ug = 0; ug < UG; ++ug) {
      const int U = (nb * UG + ug) * 16 + u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + e;
        float h2 = 0.f, c2;
        if (row < R) {
          const f32x4* ag = acc + 4 * ug;
          if (hw)  // performance arithmetic (~1e-7 absolute, like the encoder's s16x3 cell)
            lstm_cell_hw(ag[0][e] + p.bg[ug][0], ag[1][e] + p.bg[ug][1], ag[2][e] + p.bg[ug][2],
                         ag[3][e] + p.bg[ug][3], p.cold[ug][e], h2, c2);
          else  // f32 arithmetic: libm cell, torch's CPU formulas
            lstm_cell(ag[0][e] + p.bg[ug][0], ag[1][e] + p.bg[ug][1], ag[2][e] + p.bg[ug][2], ag[3][e] + p.bg[ug][3],
                      p.cold[ug][e], h2, c2);
          st_new[(size_t)row * ST + C + U] = h2;
          st_new[(size_t)row * ST + C + HD + U] = c2;
          reinterpret_cast<uint32_t*>(st_new)[(size_t)row * ST + ST16 + C + U] = split16_word(h2);
        }
        ht[ws][4 * g + e][16 * ug + u] = h2;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile is read back by other lanes of this wave
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int at = 0; at < A / 16; ++at) {
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ug = 0; ug < UG; ++ug) {
        f32x4 qg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) qg = mfma16x16x4(ht[ws][lane & 15][16 * ug + 4 * kk + g], p.wh[ug][at][kk], qg);
        if (ug == 0) q = qg;
        else q += qg;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + 4 * g + e;
        if (row < R) qpart[((size_t)nb * R + row) * A + at * 16 + (lane & 15)] = q[e];
      }
    }
  }
};

struct ProjA {  // A rows of the projection: st_new[r][0:1024] = [ctx | h] (s16: [ctx16 | h16])
  static constexpr int kSeg = 0;
  const float* st;
  int R, s16;
  template <int BM>
  __device__ __forceinline__ void prologue(int, bool) const {}
  __device__ __forceinline__ void bind(int row, const float*& seg0, const float*& seg1, int&) const {
    seg0 = seg1 = st + (size_t)(row < R ? row : R - 1) * ST + (s16 ? ST16 : 0);
  }
};

// Greedy decoding needs, per row, only the first-index argmax of the logits and their
// logsumexp (model.py:554-560), so in greedy mode the projection epilogue does not store the
// R x V logits: each block reduces its 80 columns of each row to (max, first argmax, sum of
// exp(x - max)) and writes that partial (GreedyPart); greedy_select_part_kernel combines the
// 64 partials of a row.  Beam search keeps the full logits (logits != nullptr).

// Projection epilogue pieces (ProjEpi, FoldEpi).  Lane (g, u) holds rows row0 + e (e = 0..3) of
// column tiles nb * NTN + tn, column 16 (nb NTN + tn) + u; bn: the columns' biases.
// Beam logits: the wave's 16 rows x 16 NTN columns go through its LDS slab (row stride padded by 4
// floats: the four row groups of a column write hit different banks), then out as float4 row
// segments (one instruction covers 64 consecutive float4 of the tile, row-major: up to 640
// contiguous bytes per row), and each 16-column tile's maximum (tmx, for the beam select's
// threshold and candidate tiles; tiles < ntl only) is reduced over the quad of lanes that hold it.
template <int NTN>
__device__ __forceinline__ void proj_logits_out(const f32x4 (&acc)[NTN], const float (&bn)[16], int row0, int nb,
                                                int u, float* scr, float* logits, float* tmx, int R, int V,
                                                int ntl, float* gates = nullptr, int gcol0 = 0) {
  constexpr int RWS = 16 * NTN + 4, CH = 4 * NTN;  // slab row stride; float4 per tile row
  const int lane = threadIdx.x & 63, g = lane >> 4;
#pragma unroll
  for (int tn = 0; tn < NTN; ++tn)
#pragma unroll
    for (int e = 0; e < 4; ++e) scr[(4 * g + e) * RWS + tn * 16 + u] = acc[tn][e] + bn[tn];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int rb0 = row0 - 4 * g, c0 = nb * 16 * NTN;
  const bool vec = (V & 3) == 0;
#pragma unroll
  for (int i = 0; i < CH / 4; ++i) {
    const int f = i * 64 + lane, rr = f / CH, ch = f - rr * CH;
    const float4 v = *reinterpret_cast<const float4*>(scr + rr * RWS + 4 * ch);
    const int row = rb0 + rr, col = c0 + 4 * ch;
    if (gates && col >= gcol0) {  // (FoldEpi) the next step's gate pre-activations: raw, no bias
      if (row < R && col - gcol0 < 4 * HD) *reinterpret_cast<float4*>(gates + (size_t)row * (4 * HD) + (col - gcol0)) = v;
      continue;
    }
    if (!logits) continue;
    if (row < R && !(CASR_DG_DIAG & 256)) {  // (diagnostic bit 256: no logits stores, wrong data)
      float* dst = logits + (size_t)row * V + col;
      if (vec && col + 3 < V) {
#if CASR_LOGITS_NT
        __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(dst));
#else
        *reinterpret_cast<float4*>(dst) = v;
#endif
      } else {
        if (col < V) dst[0] = v.x;
        if (col + 1 < V) dst[1] = v.y;
        if (col + 2 < V) dst[2] = v.z;
        if (col + 3 < V) dst[3] = v.w;
      }
    }
    if (tmx) {
      float m = fmaxf(fmaxf(col < V ? v.x : -INFINITY, col + 1 < V ? v.y : -INFINITY),
                      fmaxf(col + 2 < V ? v.z : -INFINITY, col + 3 < V ? v.w : -INFINITY));
      m = fmaxf(m, dpp_f<DPP_XOR1>(m));
      m = fmaxf(m, dpp_f<DPP_XOR2>(m));
      if ((lane & 3) == 0 && row < R && (col >> 4) < ntl) tmx[(size_t)row * GP_NT + (col >> 4)] = m;
    }
  }
}

// per-row partials over the block's columns n < V (greedy, and beam at temperature 1): lane (g, u)
// holds columns 16 (nb NTN + tn) + u; the 16 lanes of one g share the rows
// IX: also the first column of the maximum (the greedy select's token; the beam select reads only
// the maximum and the sum)
template <int NTN, bool IX = true>
__device__ __forceinline__ void proj_row_partials(const f32x4 (&acc)[NTN], const float (&bn)[16], int row0, int nb,
                                                  int u, const GreedyPart& gp, int R, int V) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float x[NTN];
    float m = -INFINITY;
    int mi = 0x7fffffff;
#pragma unroll
    for (int tn = 0; tn < NTN; ++tn) {
      const int n = (nb * NTN + tn) * 16 + u;
      x[tn] = acc[tn][e] + bn[tn];
      if constexpr (IX) {
        if (n < V && x[tn] > m) {  // columns ascend with tn: first index within the lane
          m = x[tn];
          mi = n;
        }
      } else if (n < V) {
        m = fmaxf(m, x[tn]);
      }
    }
    {  // the row's (max, lowest column among equal maxima) over the 16 lanes of this g
      const float rm = row16_max(m);
      if constexpr (IX) mi = row16_min(m == rm ? mi : 0x7fffffff);
      m = rm;
    }
    // sum of exp(x - max): v_exp_f32 (1 ulp) of (x - max) log2(e), whose product rounding adds at most
    // |x - max| 2^-24 relative to a term (<= 1e-6 for the terms above 4e-8), so the row's logsumexp
    // moves by ~1e-6: the select's values x - lse + score move together per row, and the scores stay
    // far inside their 2e-3 tolerance (the GPU suite passes unchanged; A/B: fused GEMM 3.9 -> 3.8 ms
    // per beam batch, profiles/r05/fastexp/)
    float sx = 0.f;
#pragma unroll
    for (int tn = 0; tn < NTN; ++tn) {
      const int n = (nb * NTN + tn) * 16 + u;
      if (n < V) sx += CASR_FAST_PART_EXP ? __builtin_amdgcn_exp2f((x[tn] - m) * 1.4426950408889634f) : expf(x[tn] - m);
    }
    sx = row16_sum(sx);  // lane u == 0 (the row's first quad) writes it
    const int row = row0 + e;
    if (u == 0 && row < R) {
      gp.mx[(size_t)row * GP_NB + nb] = m;
      gp.se[(size_t)row * GP_NB + nb] = sx;
      if constexpr (IX) gp.ix[(size_t)row * GP_NB + nb] = mi;
    }
  }
}

struct ProjEpi {
  static constexpr int kTraceClass = 1;
  static constexpr bool kPreRowFree = true;  // the column biases
  static constexpr bool kScratch = true;  // beam logits go out through per-wave LDS slabs
  const float* bias;
  float* logits;  // [R][V] (beam); nullptr in greedy mode
  // per-block row partials (greedy; beam at temperature 1 for its logsumexp and threshold), or
  // gp.mx == nullptr
  const int32_t* newdone;
  int R, V, l, total;
  int32_t* err;
  GreedyPart gp;
  struct Pre {
    float bn[16];
  };
  __device__ __forceinline__ int32_t* err_flags() const { return err; }
  __device__ __forceinline__ bool skip() const { return done_before(newdone, l) >= total; }
  template <int NTN>
  __device__ __forceinline__ void prefetch(Pre& p, int, int nb, int u, int&) const {
    static_assert(NTN <= 16, "bias prefetch slots");
#pragma unroll
    for (int tn = 0; tn < NTN; ++tn) {
      const int n = (nb * NTN + tn) * 16 + u;
      p.bn[tn] = n < V ? bias[n] : 0.f;
    }
  }
  template <int NTN>
  __device__ __forceinline__ void late(Pre&, int, int, int) const {}
  template <int NTN = 4>
  __device__ __forceinline__ void run(const f32x4 (&acc)[NTN], int row0, int nb, int u, const Pre& p,
                                      float* scr) const {
    static_assert(NTN <= 16, "bias prefetch slots");
    if (logits) proj_logits_out<NTN>(acc, p.bn, row0, nb, u, scr, logits, gp.tmx, R, V, GP_NT);
    if (gp.mx) {
      if (logits) proj_row_partials<NTN, false>(acc, p.bn, row0, nb, u, gp, R, V);  // beam
      else proj_row_partials<NTN>(acc, p.bn, row0, nb, u, gp, R, V);
    }
  }
};

// Epilogue of the folded step's GEMM (casr_internal.h KB): columns are 16-column tiles of the
// fused image, vocabulary tiles T < VT first (greedy partials exactly as ProjEpi's, over the
// tile's columns n < V), then the LSTM gate tiles gt = T - VT of the next step, stored raw into
// gates[row][gt * 16 + u] (packed gate-row order; the biases are in the per-token table).  A block
// whose tiles are all gate tiles writes no partial; nbp = ceil(VT / NT) blocks do.
struct FoldEpi {
  static constexpr int kTraceClass = 1;
  static constexpr bool kPreRowFree = true;  // the column biases
  static constexpr bool kScratch = true;  // beam logits go out through per-wave LDS slabs
  const float* bias;  // proj_b [VP]
  const int32_t* newdone;
  int R, V, VT, l, total;
  int32_t* err;
  GreedyPart gp;   // row partials (greedy; beam at temperature 1) or gp.mx == nullptr
  float* gates;    // [R][4 HD]
  float* logits;   // [R][V] (beam), or nullptr
  int VG;          // first gate tile (fold_gtile0: VT rounded up to a whole wave column)
  struct Pre {
    float bn[16];
  };
  __device__ __forceinline__ int32_t* err_flags() const { return err; }
  __device__ __forceinline__ bool skip() const { return done_before(newdone, l) >= total; }
  template <int NTN>
  __device__ __forceinline__ void prefetch(Pre& p, int, int nb, int u, int&) const {
    static_assert(NTN <= 16, "bias prefetch slots");
#pragma unroll
    for (int tn = 0; tn < NTN; ++tn) {
      const int n = (nb * NTN + tn) * 16 + u;
      p.bn[tn] = n < V ? bias[n] : 0.f;
    }
  }
  template <int NTN>
  __device__ __forceinline__ void late(Pre&, int, int, int) const {}
  template <int NTN>
  __device__ __forceinline__ void run(const f32x4 (&acc)[NTN], int row0, int nb, int u, const Pre& p,
                                      float* scr) const {
    // logits (beam) and the gate columns through the wave's LDS slab as float4 row segments (the
    // gate columns of consecutive tiles are consecutive in gates[row]; VT 16 is a multiple of 4, so
    // no segment straddles the two); the biases of the gate tiles are 0 (Pre), the stored values raw
    const bool has_gates = (nb + 1) * NTN > VG;
    if (logits || has_gates)
      proj_logits_out<NTN>(acc, p.bn, row0, nb, u, scr, logits, gp.tmx, R, V, VT, has_gates ? gates : nullptr,
                           16 * VG);
    if (nb * NTN >= VT) return;  // no vocabulary tile in this block
    if (gp.mx) {
      if (logits) proj_row_partials<NTN, false>(acc, p.bn, row0, nb, u, gp, R, V);  // beam
      else proj_row_partials<NTN>(acc, p.bn, row0, nb, u, gp, R, V);
    }
  }
};

// ------------------------------------------------------------------ fold tables (bind time)
// the fused fragment image: vocabulary tiles 0..VT-1 of proj_w16, zero tiles up to VG (a whole wave
// column), then the 128 LSTM gate tiles of dec_w16 restricted to its k blocks 4..19 (the [ctx | h]
// part of [emb | ctx | h]: E = 256 = 4 x 64)
__global__ void fold_image_kernel(const float* __restrict__ proj16, const float* __restrict__ dec16, int VT, int VG,
                                  float* __restrict__ out) {
  const int T = blockIdx.x / (KPROJ / 64), kc = blockIdx.x % (KPROJ / 64);
  const float* src = T < VT   ? proj16 + ((size_t)T * (KPROJ / 64) + kc) * FRAG
                     : T < VG ? nullptr
                              : dec16 + ((size_t)(T - VG) * (KDEC / 64) + E / 64 + kc) * FRAG;
  float* dst = out + (size_t)blockIdx.x * FRAG;
  for (int i = threadIdx.x; i < FRAG / 4; i += blockDim.x)
    reinterpret_cast<float4*>(dst)[i] = src ? reinterpret_cast<const float4*>(src)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// the per-token gate table: emb_gates[v][n] = sum_k emb[v][k] W_dec[n][k] (k < E, f32 fma chain
// in k order, from the f32 fragment image) + (b_ih + b_hh)[n], n in packed gate-row order.
// Block = 64 tokens x 256 gate rows (the embedding rows in LDS), thread = one gate row.
constexpr int FOLD_EV = 64;
__global__ __launch_bounds__(256) void fold_emb_gates_kernel(const float* __restrict__ emb, const float* __restrict__ decw,
                                                             const float* __restrict__ decb, int V,
                                                             float* __restrict__ out) {
  __shared__ float es[FOLD_EV][E];
  const int v0 = blockIdx.x * FOLD_EV, n = blockIdx.y * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < FOLD_EV * E; i += 256) {
    const int v = v0 + i / E;
    es[i / E][i % E] = v < V ? emb[(size_t)v * E + i % E] : 0.f;
  }
  __syncthreads();
  float acc[FOLD_EV];
#pragma unroll
  for (int j = 0; j < FOLD_EV; ++j) acc[j] = 0.f;
  const int nt = n >> 4, rr = n & 15;
  for (int k = 0; k < E; ++k) {
    // pack_frag: block (nt, kc), [q][lane][4] with lane = row + 16 ((k % 64) / 16), q = (k % 16) / 4
    const int kc = k >> 6, kk = k & 63;
    const int lane = rr + 16 * (kk >> 4), q = (kk & 15) >> 2;
    const float w = decw[((size_t)nt * (KDEC / 64) + kc) * FRAG + (q * 64 + lane) * 4 + (kk & 3)];
#pragma unroll
    for (int j = 0; j < FOLD_EV; ++j) acc[j] = fmaf(es[j][k], w, acc[j]);
  }
  const float b = decb[n];
#pragma unroll
  for (int j = 0; j < FOLD_EV; ++j)
    if (v0 + j < V) out[(size_t)(v0 + j) * (4 * HD) + n] = acc[j] + b;
}

// W_hidden^T ([A][HD]: n = attention column, k = decoder unit) as an s16 fragment image (the layout
// of casr_capi.hip pack_frag16: block (nt, kc) = [j][hi | lo][lane][8 halves], n = 16 nt + (lane & 15),
// k = 64 kc + 16 (lane >> 4) + 8 j + e): the B operand of the beam cell's query MFMAs
__global__ void fold_wq16_kernel(const float* __restrict__ w_hidden, float* __restrict__ out) {
  const int blk = blockIdx.x, nt = blk / (HD / 64), kc = blk % (HD / 64);
  uint16_t* o = reinterpret_cast<uint16_t*>(out) + (size_t)blk * FRAG * 2;
  for (int i = threadIdx.x; i < 2 * 64 * 8; i += blockDim.x) {  // (j, lane, e)
    const int j = i / 512, lane = (i / 8) % 64, e = i % 8;
    const int n = nt * 16 + (lane & 15), k = kc * 64 + 16 * (lane >> 4) + 8 * j + e;
    const uint32_t w = split16_word(w_hidden[(size_t)k * A + n]);
    o[((j * 2 + 0) * 64 + lane) * 8 + e] = (uint16_t)(w & 0xFFFFu);
    o[((j * 2 + 1) * 64 + lane) * 8 + e] = (uint16_t)(w >> 16);
  }
}

hipError_t build_fold(const float* W, const Layout& L, int V, float* wfold, float* emb_gates, float* wq16,
                      float* wfold32, hipStream_t s) {
  const int VT = fold_vtiles(V), VG = fold_gtile0(V);
  if (VT > L.VP / 16) return hipErrorInvalidValue;
  // the f32 and s16 fragment images share their tiling and k order (Layout), so one copy kernel
  // assembles either fused image
  if (wfold)
    hipLaunchKernelGGL(fold_image_kernel, dim3((VG + FOLD_GT) * (KPROJ / 64)), dim3(256), 0, s, W + L.proj_w16,
                       W + L.dec_w16, VT, VG, wfold);
  if (wfold32)
    hipLaunchKernelGGL(fold_image_kernel, dim3((VG + FOLD_GT) * (KPROJ / 64)), dim3(256), 0, s, W + L.proj_w,
                       W + L.dec_w, VT, VG, wfold32);
  if (emb_gates)
    hipLaunchKernelGGL(fold_emb_gates_kernel, dim3((V + FOLD_EV - 1) / FOLD_EV, 4 * HD / 256), dim3(256), 0, s,
                       W + L.emb, W + L.dec_w, W + L.dec_b, V, emb_gates);
  if (wq16) hipLaunchKernelGGL(fold_wq16_kernel, dim3((A / 16) * (HD / 64)), dim3(256), 0, s, W + L.w_hidden, wq16);
  return hipGetLastError();
}

// ------------------------------------------------------------------ init
// st0[r] = [ctx 0 | h_fin(b) | c_fin(b)], tok = sos, src = r, score = 0 (model.py:531-535,
// :660-669, :684-690).
// src2 (greedy with the fused select, else null): the second predecessor buffer, also identity
__global__ void decode_init_kernel(float* __restrict__ st0, const float* __restrict__ hfin,
                                   const float* __restrict__ cfin, int B, int k, int sos,
                                   int32_t* __restrict__ tok, int32_t* __restrict__ src,
                                   float* __restrict__ score, int32_t* __restrict__ src2) {
  const int r = blockIdx.x, b = r / k;
  float* o = st0 + (size_t)r * ST;
  for (int i = threadIdx.x; i < ST16; i += blockDim.x) {
    float v;
    if (i < C) {
      v = 0.f;
    } else if (i < C + HD) {
      const int u = i - C;  // [fw | bw]
      v = hfin[((size_t)(u / H) * B + b) * H + (u % H)];
    } else {
      const int u = i - C - HD;
      v = cfin[((size_t)(u / H) * B + b) * H + (u % H)];
    }
    o[i] = v;
    if (i < C + HD) reinterpret_cast<uint32_t*>(o)[ST16 + i] = split16_word(v);
  }
  if (threadIdx.x == 0) {
    tok[r] = sos;
    src[r] = r;
    score[r] = 0.f;
    if (src2) src2[r] = r;
  }
}

// ------------------------------------------------------------------ greedy select
struct ArgMax {
  float v;
  int i;
};
__global__ __launch_bounds__(256) void greedy_select_kernel(
    const float* __restrict__ logits, int V, int R, int l, int L, int eos, int32_t* __restrict__ tok_next,
    int32_t* __restrict__ src_next, uint8_t* __restrict__ fin, int32_t* __restrict__ out_len, float* __restrict__ accum,
    int32_t* __restrict__ tokens, int32_t* __restrict__ newdone, int32_t* __restrict__ err) {
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ float ss[4];
  if (done_before(newdone, l) >= R) return;
  const int r = blockIdx.x, tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
  const float* x = logits + (size_t)r * V;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  if ((V & 3) == 0) {  // rows are 16 B aligned: 4 logits per load, 4 loads in flight
    const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll 4
    for (int i = tid; i < V / 4; i += 256) {
      const float4 q = x4[i];
      if (q.x > m) { m = q.x; mi = 4 * i; }
      if (q.y > m) { m = q.y; mi = 4 * i + 1; }
      if (q.z > m) { m = q.z; mi = 4 * i + 2; }
      if (q.w > m) { m = q.w; mi = 4 * i + 3; }
    }
  } else {
    for (int v = tid; v < V; v += 256) {
      const float xv = x[v];
      if (xv > m) {
        m = xv;
        mi = v;
      }
    }
  }
  wave_best(m, mi);
  if (ln == 0) {
    sv[wv] = m;
    si[wv] = mi;
  }
  __syncthreads();
  m = sv[0];
  mi = si[0];
#pragma unroll
  for (int w = 1; w < 4; ++w)
    if (better(sv[w], si[w], m, mi)) {
      m = sv[w];
      mi = si[w];
    }
  float s = 0.f;
  if ((V & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll 4
    for (int i = tid; i < V / 4; i += 256) {
      const float4 q = x4[i];
      s += expf(q.x - m) + expf(q.y - m) + expf(q.z - m) + expf(q.w - m);
    }
  } else {
    for (int v = tid; v < V; v += 256) s += expf(x[v] - m);
  }
  s = wave_sum(s);
  if (ln == 0) ss[wv] = s;
  __syncthreads();
  if (tid == 0) {
    const float sum = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    const float lse = logf(sum) + m;  // torch.logsumexp: log(sum(exp(x - max))) + max
    const float lp = m - lse;
    int tok = mi;
    if ((unsigned)tok >= (unsigned)V) {  // no finite maximum (NaN row)
      atomicOr(err, CASR_DEV_NAN_LOGITS);
      tok = 0;
    }
    tokens[(size_t)r * L + l] = tok;
    tok_next[r] = tok;
    src_next[r] = r;  // greedy never reorders
    const bool was = fin[r] != 0;
    const bool cur = tok == eos;
    float acc = accum[r];
    if (!was && cur) acc = acc + lp;  // model.py:567
    const bool now = was || cur;
    if (!now) {
      out_len[r] += 1;  // model.py:573
      acc = acc + lp;   // model.py:576
    }
    accum[r] = acc;
    if (now && !was) {
      fin[r] = 1;
      atomicAdd(&newdone[l], 1);
    }
  }
}

// Greedy step from the projection's per-block partials (ProjEpi greedy mode): one wave per row,
// lane b holds block b's (max, first argmax, sum exp(x - max)); the row's maximum takes the
// lowest column among equal maxima (torch.argmax: first index), and the sum of exp(x - max) is
// rebuilt as sum_b se_b exp(m_b - max) by a fixed shuffle tree.  Bookkeeping exactly as
// greedy_select_kernel (model.py:540-590).
__global__ __launch_bounds__(256) void greedy_select_part_kernel(
    GreedyPart gp, int nbp, int V, int R, int l, int L, int eos, int32_t* __restrict__ tok_next,
    int32_t* __restrict__ src_next, uint8_t* __restrict__ fin, int32_t* __restrict__ out_len, float* __restrict__ accum,
    int32_t* __restrict__ tokens, int32_t* __restrict__ newdone, int32_t* __restrict__ err) {
  if (done_before(newdone, l) >= R) return;
  const int ln = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  float m = -INFINITY, se = 0.f;
  int mi = 0x7fffffff;
  if (ln < nbp) {
    m = gp.mx[(size_t)r * GP_NB + ln];
    se = gp.se[(size_t)r * GP_NB + ln];
    mi = gp.ix[(size_t)r * GP_NB + ln];
  }
  float gm = m;
  int gi = mi;
  wave_best(gm, gi);
  const float s = wave_sum((se > 0.f) ? se * expf(m - gm) : 0.f);
  if (ln != 0) return;
  const float lse = logf(s) + gm;
  const float lp = gm - lse;
  int tok = gi;
  if ((unsigned)tok >= (unsigned)V) {  // no finite maximum (NaN row)
    atomicOr(err, CASR_DEV_NAN_LOGITS);
    tok = 0;
  }
  tokens[(size_t)r * L + l] = tok;
  tok_next[r] = tok;
  src_next[r] = r;
  const bool was = fin[r] != 0;
  const bool cur = tok == eos;
  float acc = accum[r];
  if (!was && cur) acc = acc + lp;  // model.py:567
  const bool now = was || cur;
  if (!now) {
    out_len[r] += 1;  // model.py:573
    acc = acc + lp;   // model.py:576
  }
  accum[r] = acc;
  if (now && !was) {
    fin[r] = 1;
    atomicAdd(&newdone[l], 1);
  }
}

// ------------------------------------------------------------------ beam select (beam_select.h)
template <int K2, bool UNIT_T>
__global__ __launch_bounds__(64 * bs_waves<K2>()) void beam_select_kernel(BeamSelArgs a) {
  constexpr int NWV = bs_waves<K2>();
  __shared__ BeamSelLds<K2, KMAX_BEAM, NWV> lds;
  uint32_t* btr = g_dg_trace ? g_dg_trace + ((size_t)2 * 4096 + blockIdx.x) * 8 : nullptr;
  if (btr && threadIdx.x == 0) btr[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  if (done_before(a.newdone, a.l) >= a.B) return;
  beam_select_block<K2, UNIT_T>(a, blockIdx.x, lds, btr, nullptr, nullptr);
}

// executed loop steps: the step at which the cumulative count reached `total`, + 1
__device__ __forceinline__ int executed_steps(const int32_t* newdone, int L, int total) {
  int cum = 0;
  for (int s = 0; s < L; ++s) {
    cum += newdone[s];
    if (cum >= total) return s + 1;
  }
  return L;
}

// one thread per utterance: first-max finished record (model.py:765) or the unfinished
// fallback (model.py:961-972); tokens recovered by walking the back-pointers.
__global__ void beam_finalize_kernel(int B, int k, int L, float lm_weight, float length_weight,
                                     const float* __restrict__ score0,
                                     const float* __restrict__ score1,
                                     const int32_t* __restrict__ bp, const int32_t* __restrict__ tk,
                                     const float* __restrict__ rec_score,
                                     const int32_t* __restrict__ rec_src,
                                     const uint8_t* __restrict__ rec_valid,
                                     const int32_t* __restrict__ newdone, int32_t* __restrict__ best_tokens,
                                     int32_t* __restrict__ best_len, float* __restrict__ best_score,
                                     int32_t* __restrict__ steps_out, int32_t* __restrict__ err) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int steps = executed_steps(newdone, L, B);
  if (b == 0) steps_out[0] = steps;
  if (b >= B) return;
  const int R = B * k;
  // the select of step l writes score[(l+1)&1]; the last executed step is steps-1
  const float* score_final = (steps & 1) ? score1 : score0;
  int bl = -1, bc = -1;
  float bs = 0.f;
  for (int l = 0; l < steps; ++l)
    for (int c = 0; c < k; ++c) {
      const size_t ri = ((size_t)b * L + l) * k + c;
      if (rec_valid[ri] && (bl < 0 || rec_score[ri] > bs)) {
        bl = l;
        bc = c;
        bs = rec_score[ri];
      }
    }
  int32_t* out = best_tokens + (size_t)b * L;
  int len, slot, from;
  if (bl >= 0) {
    len = bl;
    slot = rec_src[((size_t)b * L + bl) * k + bc];
    from = bl - 1;
  } else {
    const int ll = steps - 1;
    const float lw = (float)((double)length_weight * (double)(ll + 1));
    int bj = 0;
    float bsv = 0.f;
    for (int j = 0; j < k; ++j) {
      const float s = (score_final[b * k + j] + lm_weight * 0.f) + lw;
      if (j == 0 || s > bsv) {
        bsv = s;
        bj = j;
      }
    }
    bs = bsv;
    len = ll + 1;
    slot = bj;
    from = ll;
  }
  for (int s = from; s >= 0; --s) {
    if ((unsigned)slot >= (unsigned)k) {
      atomicOr(err, CASR_DEV_BAD_BACKPTR);
      slot = 0;
    }
    const size_t ix = (size_t)s * R + b * k + slot;
    out[s] = tk[ix];
    slot = bp[ix];
  }
  for (int s = len; s < L; ++s) out[s] = -1;
  best_len[b] = len;
  best_score[b] = bs;
}

// One wave per utterance (round 5): the same choice and walk as beam_finalize_kernel, with the
// utterance's records, back-pointers and tokens staged in LDS first (one coalesced pass) and the
// executed-step count from a wave prefix scan of newdone.  beam_finalize_kernel's thread per
// utterance paid a memory round trip per back-pointer hop and per newdone word (68 us per beam
// batch at B = 256, L = 40); here lane 0 walks LDS.  Same sequential order: the same bits.
__global__ __launch_bounds__(64) void beam_finalize_wave_kernel(
    int B, int k, int L, float lm_weight, float length_weight, const float* __restrict__ score0,
    const float* __restrict__ score1, const int32_t* __restrict__ bp, const int32_t* __restrict__ tk,
    const float* __restrict__ rec_score, const int32_t* __restrict__ rec_src, const uint8_t* __restrict__ rec_valid,
    const int32_t* __restrict__ newdone, int32_t* __restrict__ best_tokens, int32_t* __restrict__ best_len,
    float* __restrict__ best_score, int32_t* __restrict__ steps_out, int32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) int32_t fsm[];
  const int b = blockIdx.x, ln = threadIdx.x, R = B * k, LK = L * k, LKp = (LK + 7) & ~7;
  int32_t* sbp = fsm;
  int32_t* stk = sbp + LKp;
  float* srs = reinterpret_cast<float*>(stk + LKp);
  uint8_t* srv = reinterpret_cast<uint8_t*>(srs + LKp);
  // executed_steps(): the first s whose running sum of newdone reaches B (else L)
  int steps = L, carry = 0;
  for (int s0 = 0; s0 < L; s0 += 64) {
    const int sl = s0 + ln;
    int v = sl < L ? newdone[sl] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o);
      if (ln >= o) v += t;
    }
    v += carry;
    const unsigned long long hit = __ballot(sl < L && v >= B);
    if (hit) {
      steps = s0 + __ffsll((long long)hit);
      break;
    }
    carry = __shfl(v, 63);
  }
  if (b == 0 && ln == 0) steps_out[0] = steps;
  const int n = steps * k;
  for (int i = ln; i < n; i += 64) {
    const int st = i / k, c = i - st * k;
    sbp[i] = bp[(size_t)st * R + b * k + c];
    stk[i] = tk[(size_t)st * R + b * k + c];
    srs[i] = rec_score[(size_t)b * LK + i];
    srv[i] = rec_valid[(size_t)b * LK + i];
  }
  for (int i = n + ln; i < ((n + 7) & ~7); i += 64) srv[i] = 0;  // the scan reads 8 at a time
  __syncthreads();
  int len = 0;
  if (ln == 0) {
    const float* score_final = (steps & 1) ? score1 : score0;
    int bl = -1, bc = -1;
    float bs = 0.f;
    // records in (step, slot) order, 8 per LDS round trip, compared in that order
    for (int i0 = 0; i0 < n; i0 += 8) {
      const uint2 v8 = *reinterpret_cast<const uint2*>(srv + i0);
      const float4 s0 = *reinterpret_cast<const float4*>(srs + i0);
      const float4 s1 = *reinterpret_cast<const float4*>(srs + i0 + 4);
      const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool valid = ((e < 4 ? v8.x : v8.y) >> (8 * (e & 3))) & 0xFFu;
        if (valid && (bl < 0 || sv[e] > bs)) {
          bl = (i0 + e) / k;
          bc = (i0 + e) - bl * k;
          bs = sv[e];
        }
      }
    }
    int32_t* out = best_tokens + (size_t)b * L;
    int slot, from;
    if (bl >= 0) {
      len = bl;
      slot = rec_src[((size_t)b * L + bl) * k + bc];
      from = bl - 1;
    } else {
      const int ll = steps - 1;
      const float lw = (float)((double)length_weight * (double)(ll + 1));
      int bj = 0;
      float bsv = 0.f;
      for (int j = 0; j < k; ++j) {
        const float sv = (score_final[b * k + j] + lm_weight * 0.f) + lw;
        if (j == 0 || sv > bsv) {
          bsv = sv;
          bj = j;
        }
      }
      bs = bsv;
      len = ll + 1;
      slot = bj;
      from = ll;
    }
    for (int st = from; st >= 0; --st) {
      if ((unsigned)slot >= (unsigned)k) {
        atomicOr(err, CASR_DEV_BAD_BACKPTR);
        slot = 0;
      }
      out[st] = stk[st * k + slot];
      slot = sbp[st * k + slot];
    }
    best_len[b] = len;
    best_score[b] = bs;
  }
  len = __shfl(len, 0);
  for (int st = len + ln; st < L; st += 64) best_tokens[(size_t)b * L + st] = -1;
}

// grid (B, L), block 64: expand every finished record's token sequence.
__global__ void beam_records_kernel(int B, int k, int L, const int32_t* __restrict__ bp,
                                    const int32_t* __restrict__ tk, const float* __restrict__ rec_score,
                                    const int32_t* __restrict__ rec_src,
                                    const uint8_t* __restrict__ rec_valid,
                                    const int32_t* __restrict__ newdone, int32_t* __restrict__ out_tok,
                                    float* __restrict__ out_score, uint8_t* __restrict__ out_valid,
                                    int32_t* __restrict__ err) {
  const int b = blockIdx.x, l = blockIdx.y, c = threadIdx.x;
  if (c >= k) return;
  const int steps = executed_steps(newdone, L, B);
  const size_t ri = ((size_t)b * L + l) * k + c;
  const bool valid = l < steps && rec_valid[ri];
  out_valid[ri] = valid;
  int32_t* o = out_tok + ri * L;
  if (!valid) {
    for (int s = 0; s < L; ++s) o[s] = -1;
    out_score[ri] = 0.f;
    return;
  }
  out_score[ri] = rec_score[ri];
  int slot = rec_src[ri];
  const int R = B * k;
  for (int s = l - 1; s >= 0; --s) {
    if ((unsigned)slot >= (unsigned)k) {
      atomicOr(err, CASR_DEV_BAD_BACKPTR);
      slot = 0;
    }
    const size_t ix = (size_t)s * R + b * k + slot;
    o[s] = tk[ix];
    slot = bp[ix];
  }
  for (int s = l; s < L; ++s) o[s] = -1;
}

// ------------------------------------------------------------------ decode GEMM launch shapes
// Tile choice per row count (one 512-thread block per CU, 256 blocks at R = 256):
//   LSTMCell (N = 2048, 16 units x 4 gates per block): R <= 256: 32 rows, ring 4; R <= 512:
//   64 rows, ring 4; else 128 rows, ring 3.
//   projection (N = 5056 = 316 16-column tiles): R <= 256: 64 rows x 80 columns, ring 4;
//   R <= 512: 128 x 80, ring 3 (<= 156 KB of LDS each); else 128 x 160, ring 2, each wave 32 rows
//   (RS = 2: every W fragment it reads feeds two MFMA row slabs) x 80 columns (WC = 2).
// At R > 512 (beam) both GEMMs issue the next tile's DMA between their MFMA groups (IL).
// Beam ablations at R = 1024 (k loop per block, us; tools/probes/dg_diag.sh): projection 27.9
// full, 19.8 without the k loop's DMA, 13.8 without its MFMAs; LSTMCell 18.6 / 13.0 / 7.1.  The
// compute phase (s16x3: 3 MFMAs per product) and the DMA overlapped poorly: all 8 waves issued
// their 9 DMA instructions in one burst after each barrier, with the MFMA pipes idle.  Interleaved
// (A/B, ms per beam batch): projection 1.75 -> 1.67, with the 32 x 80 wave tiles 1.61; LSTMCell
// 1.27 -> 1.24.  The greedy shapes (R = 256, 2-3 DMA instructions per wave and tile) measured
// slower interleaved (0.82 -> 0.86-0.88 ms each) and keep the burst.
// Measured at R = 256 (bench, ms per greedy batch of 40 steps): projection 64 x 80 ring 4 0.88
// against 1.11 for the 32 x 64 two-buffer tile of 640 blocks, 1.19 for 64 x 64 ring 4 (316
// blocks), 1.59 for 32 x 64 ring 6 (LDS then admits one of its 2.5 blocks per CU); the LSTMCell
// is 0.92 at ring 2, 4 and 6 alike: past one tile in flight a CU's intake from MALL/HBM-latency
// sources does not grow with depth (about 26-35 GB/s per CU in every variant).
template <class ASrc, class Epi>
static void launch_dec_lstm(int R, const float* Wf, const ASrc& asrc, const Epi& epi, int s16, hipStream_t s) {
  const int NB = HD / 16, ntiles = 4 * NB, nkt = KDEC / DG_BK;
  if (R <= 256) launch_dg<2, 4, 4>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (R <= 512) launch_dg<4, 4, 4>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (!dec_wide(R)) launch_dg<8, 4, 3, 1, 1, true>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  // R >= 2048: 128 rows x 128 columns (two 16-unit groups), two 64-deep stages: at R = 2048 one
  // round of 256 blocks, 1.3 MB per block, instead of two rounds of 128 x 64 blocks (ring 3) at
  // 0.98 MB each (at R = 1024 the 128 x 64 blocks are one round: 256 blocks)
  else launch_dg<8, 8, 2, 1, 1, true>(NB / 2, R, ntiles, nkt, Wf, asrc, epi, s16, s);
}

template <class ASrc, class Epi>
static void launch_proj(int R, int ntiles, const float* Wf, const ASrc& asrc, const Epi& epi, int s16, int small_w,
                        hipStream_t s) {
  const int nkt = KPROJ / DG_BK, NB = (ntiles + 4) / 5;  // 5 column tiles per block (10 at R > 512)
  // R <= 32 (BASELINE config 2): 32-row blocks, so no block stages and multiplies 32 padding rows
  if (R <= 32) launch_dg<2, 5, 4>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (R <= 256) launch_dg<4, 5, 4>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (R <= 512) launch_dg<8, 5, 3>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (!s16 || !small_w) launch_dg<4, 10, 2, 2, 2, true>((ntiles + 9) / 10, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  else if (!dec_wide(R)) launch_dg<4, 10, 2, 2, 2, true, 64, true>((ntiles + 9) / 10, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  // s16 at R >= 2048 with |W_p| < 16: 256 x 160 blocks of 32-deep stages, ring 3, one accumulator
  // (one round of 256 blocks at R = 2048, 1.7 MB per block, against two rounds of 128 x 160 blocks
  // at 1.2 MB each; at R = 1024 the 128 x 160 blocks are one round: 256 blocks)
  else launch_dg<4, 10, 3, 4, 2, true, 32, true>((ntiles + 9) / 10, R, ntiles, nkt, Wf, asrc, epi, s16, s);
}

// the folded step's GEMM (KB) over the 441 tiles (313 vocabulary + 128 gate) of the fused image.
// Greedy: 64 x 112 blocks (R <= 32: 32 x 112), ring of three 64-deep stages (44 KB each); at R = 256,
// 4 x 63 = 252 blocks in one round, 721 KB per block against 590 KB (projection) + 491 KB
// (LSTMCell) for the three-launch step (a ring of six 32-deep stages, the same bits, measured
// 1.29-1.34 against 1.00 ms per greedy batch).  Beam (one-accumulator s16x3, 32-deep stages, wave tiles of
// 16 RS rows x 112 columns, the 7-tile column blocks of the greedy shapes): 256 x 224 blocks, a W ring
// of two 28 KB stages and an A ring of three 32 KB stages (dgemm_kernel SA), at R >= 2048 (8 x 32 = 256 blocks at R = 2048, 1.97 MB each against 1.7 MB
// + 1.3 MB); 128 x 224, ring of three, below (R = 1024: 256 blocks)
constexpr int FOLD_NT_BEAM = 2 * FOLD_NT;
template <class ASrc, class Epi>
static void launch_fold_gemm(int R, bool beam, int NB, int ntiles, const float* Wf, const ASrc& asrc, const Epi& epi,
                             int s16, hipStream_t s, f32x4* kspart = nullptr, int* kscnt = nullptr) {
  const int nkt = KPROJ / DG_BK;
  if (!beam) {  // (greedy: s16x3, or the exact-f32 MFMAs on the f32 fused image)
    // R <= 32 with a k-split buffer (CASR_OPT_DEC_KSPLIT): DG_KS blocks per 32 x 112 output block
    if (R <= 32 && kspart && NB <= DG_KS_GROUPS && nkt % DG_KS == 0)
      launch_dg<2, FOLD_NT, 3, 1, 1, false, 64, false, 3, DG_KS>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s, kspart, kscnt);
    else if (R <= 32) launch_dg<2, FOLD_NT, 3>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
    else launch_dg<4, FOLD_NT, 3>(NB, R, ntiles, nkt, Wf, asrc, epi, s16, s);
  } else if (dec_wide(R)) {  // (128 x 224 in two rounds at R = 2048 measured 12.07 against 11.47 ms per batch)
    // A ring of three beside the W ring of two (152 KB): fused GEMM 3.96-4.02 -> 3.88-3.92 ms per beam
    // batch (interleaved A/B, two rounds; a version unrolled by 6 with static A buffers spilled 11 VGPRs)
    launch_dg<4, FOLD_NT_BEAM, 2, 4, 2, true, 32, true, 3>(NB, R, ntiles, nkt, Wf, asrc, epi, 1, s);
  } else {
    launch_dg<4, FOLD_NT_BEAM, 3, 2, 2, true, 32, true>(NB, R, ntiles, nkt, Wf, asrc, epi, 1, s);
  }
}

// ------------------------------------------------------------------ host drivers
// per-block row partials from the projection epilogue: the vocabulary must fit the 64 partial
// blocks; beam search uses them at temperature 1 only (they are of x, not x / T)
static int fold_col_blocks(int V) { return (fold_vtiles(V) + FOLD_NT - 1) / FOLD_NT; }
static int proj_col_blocks(const DecodeArgs& a) {
  // the folded step's partials: one per 7-tile wave column in every shape
  if (a.fold) return fold_col_blocks(a.V);
  const int nt = a.L.VP / 16, R = a.B * a.k;
  // the column block of a wave (ProjEpi's partial index): 5 tiles in every launch_proj shape (the
  // beam blocks' two wave columns), so the select's partial sums do not depend on R
  (void)R;
  return (nt + 4) / 5;
}
static bool row_partials(const DecodeArgs& a) {
  return proj_col_blocks(a) <= GP_NB && (a.greedy_run || a.temperature == 1.0f);
}

// proj = false: LSTMCell and attention only (the folded step's step 0: its GEMM follows)
static hipError_t decode_step(const DecodeArgs& a, DecodeBufs& d, int l, int total, float* align,
                              hipStream_t s, const GreedySel* gsel = nullptr, bool proj = true) {
  const int R = a.B * a.k;
  const float* st_old = d.st[l & 1];
  float* st_new = d.st[(l + 1) & 1];
  {
    ProfScope ps(a.prof, CASR_K_DEC_LSTM, s);
    DecLstmA asrc{a.W + (a.s16 ? a.L.emb16 : a.L.emb), st_old, d.tok[l & 1], d.src[l & 1], d.err, R, a.V, a.s16};
    if (gsel) {
      asrc.sel = 1;
      asrc.gs = *gsel;
    }
    DecLstmEpi epi{a.W + a.L.dec_b, st_old, st_new, asrc, d.newdone, a.W + a.L.w_hidden, d.qpart, R, l, total};
    epi.hw = a.s16;
    launch_dec_lstm(R, a.W + (a.s16 ? a.L.dec_w16 : a.L.dec_w), asrc, epi, a.s16, s);
  }
  hipError_t e;
  {
    ProfScope ps(a.prof, CASR_K_ATTENTION, s);
    e = launch_attention_step(a, st_new, d.qpart, align, d.newdone, l, total, s);
  }
  if (e != hipSuccess) return e;
  if (proj) {
    ProfScope ps(a.prof, CASR_K_PROJ, s);
    ProjA asrc{st_new, R, a.s16};
    // greedy: per-block partials instead of logits; beam at temperature 1: logits and partials
    const bool parts = row_partials(a);
    GreedyPart gp = parts ? d.part : GreedyPart{nullptr, nullptr, nullptr, nullptr};
    if (a.greedy_run || a.V > 16 * GP_NT) gp.tmx = nullptr;  // tile maxima: beam only
    ProjEpi epi{a.W + a.L.proj_b, a.greedy_run && parts ? nullptr : d.logits, d.newdone, R, a.V, l, total, d.err, gp};
    launch_proj(R, a.L.VP / 16, a.W + (a.s16 ? a.L.proj_w16 : a.L.proj_w), asrc, epi, a.s16, a.proj_small, s);
  }
  return hipGetLastError();
}

// CASR_DG_TRACE=<file>: allocate the stamp buffer once and point g_dg_trace at it (diagnostics)
static uint32_t* dg_trace_buffer() {
  static uint32_t* buf = nullptr;
  static bool init = false;
  if (!init) {
    init = true;
    if (std::getenv("CASR_DG_TRACE") && hipMalloc(&buf, 4 * 4096 * 8 * sizeof(uint32_t)) == hipSuccess) {
      (void)hipMemset(buf, 0, 4 * 4096 * 8 * sizeof(uint32_t));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dg_trace), &buf, sizeof(buf));
      attn_trace_bind(buf + 3 * 4096 * 8);  // class 3: attention (attention.hip)
    }
  }
  return buf;
}

void dg_trace_init() { dg_trace_buffer(); }

// CASR_DG_TRACE_STEP=<l> (diagnostics): the fused decode GEMM records its stamps at step l only
// (before: every launch, the last one's surviving)
static void dg_trace_step_gate(int l, bool before, hipStream_t s) {
  static const int step = std::getenv("CASR_DG_TRACE_STEP") ? std::atoi(std::getenv("CASR_DG_TRACE_STEP")) : -1;
  uint32_t* buf = dg_trace_buffer();
  if (!buf || step < 0) return;
  // a pageable host-to-device copy inside a stream capture could be refused or invalidate the
  // graph: the step gate applies to eager decodes only (diagnostics)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return;
  static uint32_t* on = nullptr;
  static uint32_t* const off = nullptr;
  on = buf;
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_dg_trace), (before && l != step) ? &off : &on, sizeof(on), 0,
                               hipMemcpyHostToDevice, s);
}

void dg_trace_dump() {
  uint32_t* buf = dg_trace_buffer();
  const char* path = std::getenv("CASR_DG_TRACE");
  if (!buf || !path) return;
  std::vector<uint32_t> h(4 * 4096 * 8);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h.data(), buf, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (FILE* f = std::fopen(path, "wb")) {
    std::fwrite(h.data(), 4, h.size(), f);
    std::fclose(f);
  }
}

// the folded greedy step's GEMM (KB) on st_new = [ctx | h] of step l: partials of step l and, unless
// l is the last step, the next step's gate pre-activations
// beam: logits, and at temperature 1 the row partials and tile maxima, as decode_step's projection
static void fold_gemm_step(const DecodeArgs& a, DecodeBufs& d, int l, int total, hipStream_t s) {
  const int R = a.B * a.k;
  const bool beam = !a.greedy_run;
  const int VT = fold_vtiles(a.V), VG = fold_gtile0(a.V), NT = beam ? FOLD_NT_BEAM : FOLD_NT;
  const bool gates = l + 1 < a.max_len;
  const int ntiles = VG + FOLD_GT;
  const int NB = ((gates ? ntiles : VT) + NT - 1) / NT;
  ProfScope ps(a.prof, CASR_K_PROJ, s);
  ProjA asrc{d.st[(l + 1) & 1], R, a.s16};
  GreedyPart gp = row_partials(a) ? d.part : GreedyPart{nullptr, nullptr, nullptr, nullptr};
  if (!beam || a.V > 16 * GP_NT) gp.tmx = nullptr;  // tile maxima: beam only
  FoldEpi epi{a.W + a.L.proj_b, d.newdone, R, a.V, VT, l, total, d.err, gp, a.fb.gates, beam ? d.logits : nullptr, VG};
  dg_trace_step_gate(l, true, s);
  launch_fold_gemm(R, beam, NB, ntiles, a.fb.wfold, asrc, epi, a.s16, s, beam ? nullptr : reinterpret_cast<f32x4*>(d.kspart), d.kscnt);
  dg_trace_step_gate(l, false, s);
}

// the folded step's attention with its cell prologue (steps l >= 1): greedy with the fused select
// of step l - 1 (sel), beam with the beam select's tokens and predecessor rows
static hipError_t fold_attention_step(const DecodeArgs& a, DecodeBufs& d, int l, int total, float* align,
                                      bool sel, const GreedySel& gs, hipStream_t s, const BeamSelArgs* bs = nullptr) {
  ProfScope ps(a.prof, CASR_K_ATTENTION, s);
  AttnCell cell{};
  cell.st_old = d.st[l & 1];
  cell.gates = a.fb.gates;
  cell.emb_gates = a.fb.emb_gates;
  cell.w_hidden = a.W + a.L.w_hidden;
  cell.wq16 = a.fb.wq16;
  cell.tok = d.tok[l & 1];
  cell.src = d.src[l & 1];
  cell.err = d.err;
  cell.sel = sel ? 1 : 0;
  cell.gs = gs;
  if (bs) {
    cell.bsel = 1;
    cell.bs = *bs;
  } else if (d.aspart && !align) {  // greedy, CASR_OPT_ATTN_SPLIT: d.asplit ranges of a multiple of 4 steps
    const int tq = (a.Tp + 3) & ~3;  // (attention.hip's attn_tq)
    cell.tc = ((tq + d.asplit - 1) / d.asplit + 3) & ~3;
    cell.split = (tq + cell.tc - 1) / cell.tc;  // (< 2 at short inputs: the unsplit form)
    cell.spart = d.aspart;
    cell.scnt = d.ascnt;
  }
  return launch_attention_cell_step(a, d.st[(l + 1) & 1], cell, align, d.newdone, l, total, s);
}

// CASR_OPT_DEC_FOLD (casr_internal.h): step 0 as before (LSTMCell GEMM + attention from the query
// partials), then the fused GEMM at every step and the cell inside the attention from step 1 on
static hipError_t run_greedy_fold(const DecodeArgs& a, DecodeBufs& d, int32_t* tokens, int32_t* out_len,
                                  uint8_t* finished, float* accum, float* align, hipStream_t s) {
  const int R = a.B;
  const int nbp = fold_col_blocks(a.V);
  if (nbp > GP_NB) return hipErrorInvalidValue;
  const bool fuse = a.fuse_select != 0;
  hipLaunchKernelGGL(decode_init_kernel, dim3(R), dim3(256), 0, s, d.st[0], a.hfin, a.cfin, a.B, 1, a.sos, d.tok[0],
                     d.src[0], d.score[0], nullptr);
  for (int l = 0; l < a.max_len; ++l) {
    float* al = align ? align + (size_t)l * a.Tp * R : nullptr;
    const GreedySel gs{d.part, nbp, l - 1, a.max_len, a.eos, finished, out_len, accum, tokens, d.newdone};
    const hipError_t e = l == 0 ? decode_step(a, d, 0, R, al, s, nullptr, false)
                                : fold_attention_step(a, d, l, R, al, fuse, gs, s);
    if (e != hipSuccess) return e;
    fold_gemm_step(a, d, l, R, s);
    if (fuse && l + 1 < a.max_len) continue;
    ProfScope ps(a.prof, CASR_K_SELECT, s);
    hipLaunchKernelGGL(greedy_select_part_kernel, dim3((R + 3) / 4), dim3(256), 0, s, d.part, nbp, a.V, R, l,
                       a.max_len, a.eos, d.tok[(l + 1) & 1], d.src[(l + 1) & 1], finished, out_len, accum, tokens,
                       d.newdone, d.err);
  }
  return hipGetLastError();
}

hipError_t run_greedy(const DecodeArgs& a_in, DecodeBufs& d, int32_t* tokens, int32_t* out_len,
                      uint8_t* finished, float* accum, float* align, hipStream_t s) {
  DecodeArgs a = a_in;
  a.greedy_run = 1;
  const int R = a.B;
  // fill kernels, not hipMemsetAsync: this sequence is captured into a replayed graph
  FillList fl;
  fl.add32(d.newdone, 0, a.max_len);
  fl.add8(finished, 0, R);
  fl.add32(out_len, 0, R);
  fl.add32(accum, 0, R);
  fl.add32(tokens, 0xffffffffu, (size_t)R * a.max_len);
  if (d.kscnt) fl.add32(d.kscnt, 0, DG_KS_COUNTERS);
  if (d.ascnt) fl.add32(d.ascnt, 0, R);
  hipError_t e0 = fill_multi(fl, s);
  if (e0 != hipSuccess) return e0;
  if (a.fold) return run_greedy_fold(a, d, tokens, out_len, finished, accum, align, s);
  // the select of step l runs inside step l+1's LSTMCell (GreedySel) when the projection writes
  // per-block partials; the last step's select is a launch of its own.  CASR_OPT_FUSE_SELECT = 0
  // keeps every select a launch (the same bits either way)
  const bool fuse = a.fuse_select && row_partials(a);
  hipLaunchKernelGGL(decode_init_kernel, dim3(R), dim3(256), 0, s, d.st[0], a.hfin, a.cfin, a.B, 1,
                     a.sos, d.tok[0], d.src[0], d.score[0], fuse ? d.src[1] : nullptr);
  for (int l = 0; l < a.max_len; ++l) {
    GreedySel gs{d.part, proj_col_blocks(a), l - 1, a.max_len, a.eos, finished, out_len, accum, tokens, d.newdone};
    hipError_t e = decode_step(a, d, l, R, align ? align + (size_t)l * a.Tp * R : nullptr, s,
                               fuse && l > 0 ? &gs : nullptr);
    if (e != hipSuccess) return e;
    if (fuse && l + 1 < a.max_len) continue;
    ProfScope ps(a.prof, CASR_K_SELECT, s);
    if (row_partials(a)) {
      hipLaunchKernelGGL(greedy_select_part_kernel, dim3((R + 3) / 4), dim3(256), 0, s, d.part, proj_col_blocks(a), a.V,
                         R, l, a.max_len, a.eos, d.tok[(l + 1) & 1], d.src[(l + 1) & 1], finished, out_len, accum,
                         tokens, d.newdone, d.err);
    } else {
      hipLaunchKernelGGL(greedy_select_kernel, dim3(R), dim3(256), 0, s, d.logits, a.V, R, l,
                         a.max_len, a.eos, d.tok[(l + 1) & 1], d.src[(l + 1) & 1], finished, out_len,
                         accum, tokens, d.newdone, d.err);
    }
  }
  return hipGetLastError();
}

// the select of step l: logits and partials of step l's GEMM, scores of step l in, step l + 1's
// tokens / predecessors / scores out
static BeamSelArgs beam_sel_args(const DecodeArgs& a, const DecodeBufs& d, int l) {
  return BeamSelArgs{d.logits, a.V, a.B, a.k, l, a.max_len, a.eos, a.temperature, d.score[l & 1],
                     d.score[(l + 1) & 1], d.tok[(l + 1) & 1], d.src[(l + 1) & 1], d.topfin, d.bp, d.tk,
                     d.rec_score, d.rec_src, d.rec_valid, d.newdone, d.err, d.part,
                     row_partials(a) ? proj_col_blocks(a) : 0};
}

template <int K2>
static void launch_beam_select(const DecodeArgs& a, DecodeBufs& d, int l, hipStream_t s) {
  auto kern = a.temperature == 1.0f ? beam_select_kernel<K2, true> : beam_select_kernel<K2, false>;
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(64 * bs_waves<K2>()), 0, s, beam_sel_args(a, d, l));
}

hipError_t run_beam(const DecodeArgs& a, DecodeBufs& d, float lm_weight, float length_weight,
                    int32_t* best_tokens, int32_t* best_len, float* best_score, int32_t* steps,
                    hipStream_t s) {
  const int R = a.B * a.k;
  FillList fl;
  fl.add32(d.newdone, 0, a.max_len);
  fl.add8(d.topfin, 0, a.B);
  hipError_t e0 = fill_multi(fl, s);
  if (e0 != hipSuccess) return e0;
  hipLaunchKernelGGL(decode_init_kernel, dim3(R), dim3(256), 0, s, d.st[0], a.hfin, a.cfin, a.B, a.k,
                     a.sos, d.tok[0], d.src[0], d.score[0], nullptr);
  // the folded step with one attention block per utterance (k = 4 or 8 rows per block): the select
  // of step l - 1 runs in step l's attention prologue (CASR_OPT_FUSE_SELECT; the last step's select
  // is a launch of its own)
  // (k = 8 at 4 rows per attention block: both blocks of an utterance run the select, CELL 4)
  const int fkpb = attention_kpb(a.B, a.k, a.attn_kpb);
  const bool fsel = a.fold && a.fuse_select && (a.k == 4 || a.k == 8) && (fkpb == a.k || (a.k == 8 && fkpb == 4));
  for (int l = 0; l < a.max_len; ++l) {
    // the folded step (CASR_OPT_DEC_FOLD): step 0's LSTMCell + attention, then per step the
    // attention with the cell prologue (l >= 1) and the fused GEMM
    hipError_t e;
    if (!a.fold) {
      e = decode_step(a, d, l, a.B, nullptr, s);
    } else if (l == 0) {
      e = decode_step(a, d, 0, a.B, nullptr, s, nullptr, false);
    } else {
      const BeamSelArgs bs = beam_sel_args(a, d, l - 1);
      e = fold_attention_step(a, d, l, a.B, nullptr, false, GreedySel{}, s, fsel ? &bs : nullptr);
    }
    if (e != hipSuccess) return e;
    if (a.fold) fold_gemm_step(a, d, l, a.B, s);
    if (fsel && l + 1 < a.max_len) continue;
    ProfScope ps(a.prof, CASR_K_SELECT, s);
    if (a.k <= 2) launch_beam_select<4>(a, d, l, s);
    else if (a.k <= 4) launch_beam_select<8>(a, d, l, s);
    else if (a.k <= 8) launch_beam_select<16>(a, d, l, s);
    else launch_beam_select<32>(a, d, l, s);
  }
  const size_t fin_lds = (size_t)((a.max_len * a.k + 7) & ~7) * (3 * sizeof(int32_t) + 1) + 16;
  if (fin_lds <= 64 * 1024)
    hipLaunchKernelGGL(beam_finalize_wave_kernel, dim3(a.B), dim3(64), fin_lds, s, a.B, a.k, a.max_len,
                       lm_weight, length_weight, d.score[0], d.score[1], d.bp, d.tk, d.rec_score, d.rec_src,
                       d.rec_valid, d.newdone, best_tokens, best_len, best_score, steps, d.err);
  else  // (a max_len x k past the LDS: the thread-per-utterance form)
    hipLaunchKernelGGL(beam_finalize_kernel, dim3((a.B + 63) / 64), dim3(64), 0, s, a.B, a.k, a.max_len,
                       lm_weight, length_weight, d.score[0], d.score[1], d.bp, d.tk, d.rec_score, d.rec_src,
                       d.rec_valid, d.newdone, best_tokens, best_len, best_score, steps, d.err);
  return hipGetLastError();
}

hipError_t run_beam_records(const DecodeArgs& a, DecodeBufs& d, int32_t* rec_tokens,
                            float* rec_score, uint8_t* rec_valid, hipStream_t s) {
  hipLaunchKernelGGL(beam_records_kernel, dim3(a.B, a.max_len), dim3(64), 0, s, a.B, a.k, a.max_len,
                     d.bp, d.tk, d.rec_score, d.rec_src, d.rec_valid, d.newdone, rec_tokens,
                     rec_score, rec_valid, d.err);
  return hipGetLastError();
}

}  // namespace casr
