// Beam select of one utterance and step (model.py:834-929), shared by beam_select_kernel
// (decoder.hip, a launch of its own per step) and the folded beam attention, which runs the select
// of step l - 1 in its prologue when one block serves all k rows of an utterance (attention.hip
// CELL 3).  The block's NWV waves and the LDS area S are the caller's; both callers run the same
// code, so the bits are the same either way.
#pragma once
#include "casr_common.h"
#include "casr_internal.h"

namespace casr {

__device__ __forceinline__ bool better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

template <int K2>
struct TopList {
  float v[K2];
  int i[K2];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int p = 0; p < K2; ++p) {
      v[p] = -INFINITY;
      i[p] = 0x7fffffff;
    }
  }
  __device__ __forceinline__ void insert(float xv, int xi) {
    if (!better(xv, xi, v[K2 - 1], i[K2 - 1])) return;
    v[K2 - 1] = xv;
    i[K2 - 1] = xi;
#pragma unroll
    for (int p = K2 - 1; p > 0; --p) {
      if (better(v[p], i[p], v[p - 1], i[p - 1])) {
        const float tv = v[p];
        v[p] = v[p - 1];
        v[p - 1] = tv;
        const int ti = i[p];
        i[p] = i[p - 1];
        i[p - 1] = ti;
      }
    }
  }
  __device__ __forceinline__ void pop() {
#pragma unroll
    for (int p = 0; p < K2 - 1; ++p) {
      v[p] = v[p + 1];
      i[p] = i[p + 1];
    }
    v[K2 - 1] = -INFINITY;
    i[K2 - 1] = 0x7fffffff;
  }
};

// Extract the top n (<= K2) of the union of the 64 lanes' sorted lists; lane 0 writes them.
template <int K2>
__device__ __forceinline__ void wave_merge(TopList<K2>& L, int n, float* outv, int* outi) {
  for (int c = 0; c < n; ++c) {
    float bv = L.v[0];
    int bi = L.i[0];
    wave_best(bv, bi);
    if (L.i[0] == bi && L.v[0] == bv) L.pop();
    if ((threadIdx.x & 63) == 0) {
      outv[c] = bv;
      outi[c] = bi;
    }
  }
}

// One block per utterance, one wave per beam row (rows j = w, w + 8): three exact passes
// over the row (max, sum of exp -> lse; then val = (x/T - lse) + score inserted into a
// per-lane sorted list), the lane lists merged with wave shuffles to the row's top-2k, then
// wave 0 merges the k rows' lists from LDS into the utterance's top-2k (torch.topk over
// the k*V flattened scores, model.py:860-865; ties -> lower flat index).
constexpr int BS_CAP = 256;  // threshold candidates kept per row (beyond: full selection)

// UNIT_T: temperature == 1 (the reference default, gpd['temperature']): x / T is x exactly, so the
// three per-element divisions of each pass are skipped (bitwise the same values)
// 8 waves, one per beam row (k = 16: two rows each).  Measured at k = 16 (B = 128): 16 waves
// of one row each (1024 threads, <= 128 VGPRs: the register-resident row does not fit, so they
// take the two-pass path) 45.7 us per step against 38.7 us for 8 waves on the register path.
template <int K2>
constexpr int bs_waves() {
  return 8;
}


// LDS of one select: NR rows' sorted lists (and the merge tree's other buffer), the utterance's
// list, and per wave its threshold candidates
template <int K2, int NR, int NWV>
struct BeamSelLds {
  float rv[NR][K2];
  int ri[NR][K2];
  float rv2[(NR + 1) / 2][K2];  // block-merge tree: the other buffer of each level
  int ri2[(NR + 1) / 2][K2];
  float cv[K2];
  int ci[K2];
  float cvs[NWV][BS_CAP];  // per-wave threshold candidates
  int cis[NWV][BS_CAP];
  int cnt[NWV];
};

// The select for utterance b (rows b k .. b k + k - 1, k <= NR) by the calling block's NWV waves;
// the caller has checked the early exit (done_before(newdone, l) < B).  tok_l / src_l (or null):
// the block's LDS copy of the tokens and predecessor rows it writes to tok_next / src_next (slots
// no candidate fills keep what the caller put there).  No barrier after the bookkeeping: a caller
// that reads S, tok_l or src_l afterwards synchronises first.  writer = false (the second of two
// blocks that run the same select, attention.hip CELL 4): the same choice into tok_l / src_l, no
// global bookkeeping (its finished-count increment must happen once).
template <int K2, bool UNIT_T, int NR, int NWV>
__device__ __forceinline__ void beam_select_block(const BeamSelArgs& a, int b, BeamSelLds<K2, NR, NWV>& S,
                                                  uint32_t* btr, int32_t* tok_l, int32_t* src_l,
                                                  bool writer = true) {
  constexpr int NTH = 64 * NWV;
  const float* __restrict__ logits = a.logits;
  const int V = a.V, B = a.B, k = a.k, l = a.l, L = a.L, eos = a.eos;
  const float temperature = a.temperature;
  const float* __restrict__ score_cur = a.score_cur;
  const GreedyPart& gp = a.gp;
  const int nbp = a.nbp;
  (void)B;
  auto stamp = [&](int i, uint32_t v) {
    if (btr && threadIdx.x == 0) btr[i] = v;
  };
  const int tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
  const int R = B * k;
  const int nrows = (l == 0) ? 1 : k;  // model.py:862-863: step 0 ranks beam 0 only
  const int n2k = 2 * k;
  const bool vec = (V & 3) == 0;
  auto xt = [&](float x) { return UNIT_T ? x : x / temperature; };

  for (int j = wv; j < nrows; j += NWV) {
    const float* x = logits + (size_t)(b * k + j) * V;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float sc = score_cur[b * k + j];
    constexpr int TPL = GP_NT / 64;  // tile maxima per lane
    int nc;
    float lse;  // the row's logsumexp
    if (UNIT_T && nbp > 0 && gp.tmx && vec) {
      // From the projection's partials: block (max, sum exp) -> logsumexp, and the maximum of
      // every 16-column tile.  tau = the exact 2k-th largest tile maximum (in candidate value,
      // monotone in x): the tile maxima are distinct elements, so tau bounds the row's 2k-th best
      // value from below, and every element of the top 2k lies in a tile whose maximum is >= tau.
      // Only those tiles (2k of them, ties aside) are read: 16 logits each instead of the row.
      const size_t row = (size_t)(b * k + j);
      float mb = -INFINITY, sb = 0.f;
      if (ln < nbp) {
        mb = gp.mx[row * GP_NB + ln];
        sb = gp.se[row * GP_NB + ln];
      }
      const int ntile = (V + 15) / 16;
      float tm[TPL];
      int tt[TPL];
#pragma unroll
      for (int c = 0; c < TPL; ++c) {
        tt[c] = ln + 64 * c;
        tm[c] = tt[c] < ntile ? gp.tmx[row * GP_NT + tt[c]] : -INFINITY;
      }
      const float M = wave_max(mb);
      const float s = wave_sum((sb > 0.f) ? sb * expf(mb - M) : 0.f);
      lse = logf(s) + M;
      // this lane's tiles in descending maximum (a 5-element sorting network of swaps)
#pragma unroll
      for (int i = 0; i < TPL; ++i)
#pragma unroll
        for (int c = 0; c + 1 < TPL - i; ++c)
          if (tm[c + 1] > tm[c]) {
            const float fv = tm[c];
            tm[c] = tm[c + 1];
            tm[c + 1] = fv;
            const int iv = tt[c];
            tt[c] = tt[c + 1];
            tt[c + 1] = iv;
          }
      // each lane's best tile is read ahead, under the tau rounds (the qualifying tiles are the
      // 2k best, most of them each the best of its lane); the rest only if they qualify.  Reading
      // the two best ahead measured the same.
      constexpr int PRE = 1;
      float4 xq[TPL][4];
#pragma unroll
      for (int c = 0; c < PRE; ++c)
#pragma unroll
        for (int h = 0; h < 4; ++h) xq[c][h] = x4[min(tt[c], ntile - 1) * 4 + h];
      if (j == 0) stamp(1, (uint32_t)__builtin_amdgcn_s_memrealtime());
      float tau = -INFINITY;
      {
        float hd[TPL];  // this lane's remaining tile maxima, head first
#pragma unroll
        for (int c = 0; c < TPL; ++c) hd[c] = (tm[c] - lse) + sc;
        for (int c = 0; c < n2k; ++c) {
          const float mx = wave_max(hd[0]);
          tau = mx;
          const unsigned long long hit = __ballot(hd[0] == mx);
          if (hit && ln == __ffsll((long long)hit) - 1) {
#pragma unroll
            for (int i = 0; i + 1 < TPL; ++i) hd[i] = hd[i + 1];
            hd[TPL - 1] = -INFINITY;
          }
        }
      }
      // the qualifying tiles' logits (all loads issued before any use), then the candidates
      // val >= tau compacted per wave without atomics: per-lane counts, their exclusive prefix over
      // the wave from bit-sliced ballots (counts <= 80 < 128), each lane writing from its offset
      bool qual[TPL];
#pragma unroll
      for (int c = 0; c < TPL; ++c) {
        qual[c] = (tm[c] - lse) + sc >= tau;
        if (c >= PRE) {
#pragma unroll
          for (int h = 0; h < 4; ++h)
            xq[c][h] = qual[c] ? x4[tt[c] * 4 + h] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
        }
      }
      // per-slot 16-bit hit masks; a slot no lane of the wave qualifies in (the usual case past the
      // lanes' best tiles) is skipped by a wave-uniform branch
      uint32_t hm[TPL];
      int cnt = 0;
#pragma unroll
      for (int c = 0; c < TPL; ++c) {
        hm[c] = 0u;
        if (__ballot(qual[c])) {
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int n0 = tt[c] * 16 + 4 * h;
            const float xs[4] = {xq[c][h].x, xq[c][h].y, xq[c][h].z, xq[c][h].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              hm[c] |= (qual[c] && n0 + e < V && (xs[e] - lse) + sc >= tau) ? (1u << (4 * h + e)) : 0u;
          }
          cnt += __popc(hm[c]);
        }
      }
      const unsigned long long below = (1ull << ln) - 1ull;
      int slot = 0, total = 0;
#pragma unroll
      for (int bit = 0; bit < 7; ++bit) {
        const unsigned long long mk = __ballot((cnt >> bit) & 1);
        slot += __popcll(mk & below) << bit;
        total += __popcll(mk) << bit;
      }
#pragma unroll
      for (int c = 0; c < TPL; ++c) {
        if (__ballot(hm[c] != 0u)) {
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int n0 = tt[c] * 16 + 4 * h;
            const float xs[4] = {xq[c][h].x, xq[c][h].y, xq[c][h].z, xq[c][h].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if ((hm[c] >> (4 * h + e)) & 1u) {
                if (slot < BS_CAP) {
                  S.cvs[wv][slot] = (xs[e] - lse) + sc;  // model.py:834-836
                  S.cis[wv][slot] = j * V + n0 + e;
                }
                ++slot;
              }
          }
        }
      }
      nc = total;
    } else {
    // the row read whole (temperature != 1, or a vocabulary beyond the tile-maxima table): the
    // row's logsumexp and this lane's largest and second-largest candidate values (for tau)
    float lt, lt2;
    {
      float lm = -INFINITY, lm2 = -INFINITY;  // this lane's two largest x / T (distinct elements)
      auto top2 = [&](float y) {
        lm2 = fmaxf(lm2, fminf(lm, y));
        lm = fmaxf(lm, y);
      };
      if (vec) {
#pragma unroll 4
        for (int i = ln; i < V / 4; i += 64) {
          const float4 q = x4[i];
          top2(xt(q.x));
          top2(xt(q.y));
          top2(xt(q.z));
          top2(xt(q.w));
        }
      } else {
        for (int v = ln; v < V; v += 64) top2(xt(x[v]));
      }
      const float m = wave_max(lm);
      float s = 0.f;
      if (vec) {
#pragma unroll 4
        for (int i = ln; i < V / 4; i += 64) {
          const float4 q = x4[i];
          s += expf(xt(q.x) - m) + expf(xt(q.y) - m) + expf(xt(q.z) - m) + expf(xt(q.w) - m);
        }
      } else {
        for (int v = ln; v < V; v += 64) s += expf(xt(x[v]) - m);
      }
      s = wave_sum(s);
      lse = logf(s) + m;
      lt = (lm - lse) + sc;
      lt2 = (lm2 - lse) + sc;
    }
    if (j == 0) stamp(1, (uint32_t)__builtin_amdgcn_s_memrealtime());
    // tau = the 2k-th largest of the lanes' candidate values: each round takes the largest and
    // exposes that lane's next one
    float tau = -INFINITY;
    for (int c = 0; c < n2k; ++c) {
      const float mx = wave_max(lt);
      tau = mx;
      const unsigned long long hit = __ballot(lt == mx);
      if (hit && ln == __ffsll((long long)hit) - 1) {
        lt = lt2;
        lt2 = -INFINITY;
      }
    }
    if (ln == 0) S.cnt[wv] = 0;
    __builtin_amdgcn_wave_barrier();
    auto offer = [&](float val, int idx) {
      if (val >= tau) {
        const int slot = atomicAdd(&S.cnt[wv], 1);
        if (slot < BS_CAP) {
          S.cvs[wv][slot] = val;
          S.cis[wv][slot] = idx;
        }
      }
    };
    if (vec) {
      // all of a lane's row loads in flight at once (20 float4 cover V = 5004), not two per
      // round trip
      constexpr int QB = 20;
      for (int i0 = ln; i0 < V / 4; i0 += 64 * QB) {
        float4 q[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int i = i0 + 64 * u;
          q[u] = i < V / 4 ? x4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int i = i0 + 64 * u;
          if (i >= V / 4) break;
          offer((xt(q[u].x) - lse) + sc, j * V + 4 * i);
          offer((xt(q[u].y) - lse) + sc, j * V + 4 * i + 1);
          offer((xt(q[u].z) - lse) + sc, j * V + 4 * i + 2);
          offer((xt(q[u].w) - lse) + sc, j * V + 4 * i + 3);
        }
      }
    } else {
      for (int v = ln; v < V; v += 64) offer((xt(x[v]) - lse) + sc, j * V + v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    nc = S.cnt[wv];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's candidates are in S.cvs / S.cis
    __builtin_amdgcn_wave_barrier();
    if (j == 0) {
      stamp(2, (uint32_t)__builtin_amdgcn_s_memrealtime());
      stamp(7, (uint32_t)nc);
    }
    if (nc <= BS_CAP) {
      // rank selection over the row's threshold candidates (a few dozen): a candidate's slot is
      // the number of candidates better than it (better(): value, then lower flat index; indices
      // are distinct, so ranks are too); slots no candidate reaches keep the (-inf, INT_MAX)
      // sentinel the sorted-list merge (wave_merge) produces for them.  Same list, in sorted
      // order, as the per-lane insertion + wave_merge below, without its 2k shuffle rounds.
      if (ln < n2k) {
        S.rv[j][ln] = -INFINITY;
        S.ri[j][ln] = 0x7fffffff;
      }
      __builtin_amdgcn_wave_barrier();
      if (nc <= 64) {  // one candidate per lane, the others read from registers (readlane)
        const float pv = ln < nc ? S.cvs[wv][ln] : -INFINITY;
        const int pi = ln < nc ? S.cis[wv][ln] : 0x7fffffff;
        int rank = 0;
        for (int q = 0; q < nc; ++q)
          rank += better(readlane_f(pv, q), __builtin_amdgcn_readlane(pi, q), pv, pi) ? 1 : 0;
        if (ln < nc && rank < n2k) {
          S.rv[j][rank] = pv;
          S.ri[j][rank] = pi;
        }
      } else {
        for (int p = ln; p < nc; p += 64) {
          const float pv = S.cvs[wv][p];
          const int pi = S.cis[wv][p];
          int rank = 0;
          for (int q = 0; q < nc; ++q) rank += better(S.cvs[wv][q], S.cis[wv][q], pv, pi) ? 1 : 0;
          if (rank < n2k) {
            S.rv[j][rank] = pv;
            S.ri[j][rank] = pi;
          }
        }
      }
      if (j == 0) {
        stamp(3, (uint32_t)__builtin_amdgcn_s_memrealtime());
        stamp(4, (uint32_t)__builtin_amdgcn_s_memrealtime());
      }
    } else {  // more ties at tau than the buffer holds: every element through sorted lane lists
      TopList<K2> tl;
      tl.init();
      if (vec) {
        for (int i = ln; i < V / 4; i += 64) {
          const float4 q = x4[i];
          tl.insert((xt(q.x) - lse) + sc, j * V + 4 * i);  // model.py:834-836
          tl.insert((xt(q.y) - lse) + sc, j * V + 4 * i + 1);
          tl.insert((xt(q.z) - lse) + sc, j * V + 4 * i + 2);
          tl.insert((xt(q.w) - lse) + sc, j * V + 4 * i + 3);
        }
      } else {
        for (int v = ln; v < V; v += 64) tl.insert((xt(x[v]) - lse) + sc, j * V + v);
      }
      if (j == 0) stamp(3, (uint32_t)__builtin_amdgcn_s_memrealtime());
      wave_merge<K2>(tl, n2k, S.rv[j], S.ri[j]);
      if (j == 0) stamp(4, (uint32_t)__builtin_amdgcn_s_memrealtime());
    }
  }
  __syncthreads();  // every row's sorted list is in S.rv / S.ri
  // block merge: the rows' sorted lists are merged pairwise in a tree (nrows -> 1 in
  // ceil(log2 nrows) levels), each level keeping the top 2k of every pair.  An entry's slot in its
  // pair's merged list is its position in its own list + the number of entries of the other list
  // better than it (better(): value, then lower flat index; a binary search over that sorted list),
  // one thread per entry, every wave taking part.  Real candidates have distinct indices, so
  // distinct slots; the (-inf, INT_MAX) sentinels that fill short lists land on slots only
  // sentinels reach.  Same list, in the same order, as the one-wave sorted-list merge (TopList +
  // wave_merge) this replaces.
  // (round 5) K2 = 16 (k <= 8: at most 8 lists of 16): wave 0 merges them in registers instead, a
  // bitonic network over 128 slots (2 per lane, lists of n2k padded with sentinels to 16): per level
  // (32, 64, 128 slots) a flip step (slot s against its mirror in the block) and half-cleaners, each
  // compare-exchange keeping the better (better()) in the lower slot.  better() is a total order on
  // the real candidates (distinct indices) and the sentinels are identical, so the merged order, and
  // with it the top 2k, is the tree's.  No block barrier after the row phase.
  if constexpr (K2 == 16) {
    if (wv == 0) {
      float v0, v1;
      int i0, i1;
      auto ld = [&](int s, float& v, int& i) {
        const int j = s >> 4, p = s & 15;
        const bool ok = j < nrows && p < n2k;
        v = ok ? S.rv[j][p] : -INFINITY;
        i = ok ? S.ri[j][p] : 0x7fffffff;
      };
      ld(ln, v0, i0);
      ld(64 + ln, v1, i1);
      // compare-exchange of (v, i) with the same register of lane ln ^ mask; lo keeps the better
      auto cx = [&](float& v, int& i, int mask, bool lo) {
        const float pv = __shfl_xor(v, mask);
        const int pi = __shfl_xor(i, mask);
        if (lo == better(pv, pi, v, i)) {
          v = pv;
          i = pi;
        }
      };
      auto cleaners = [&](int d0) {
        for (int d = d0; d >= 1; d >>= 1) {
          cx(v0, i0, d, (ln & d) == 0);
          cx(v1, i1, d, (ln & d) == 0);
        }
      };
      cx(v0, i0, 31, (ln & 16) == 0);  // 32-slot blocks (list pairs): flip, then cleaners
      cx(v1, i1, 31, (ln & 16) == 0);
      cleaners(8);
      cx(v0, i0, 63, (ln & 32) == 0);  // 64-slot blocks (one register each)
      cx(v1, i1, 63, (ln & 32) == 0);
      cleaners(16);
      {  // 128 slots: slot s of register 0 against slot 127 - s (register 1 of lane 63 - ln)
        const float p0v = __shfl_xor(v1, 63), p1v = __shfl_xor(v0, 63);
        const int p0i = __shfl_xor(i1, 63), p1i = __shfl_xor(i0, 63);
        if (better(p0v, p0i, v0, i0)) {
          v0 = p0v;
          i0 = p0i;
        }
        if (!better(p1v, p1i, v1, i1)) {
          v1 = p1v;
          i1 = p1i;
        }
      }
      cleaners(32);
      if (ln < n2k) {
        S.cv[ln] = v0;
        S.ci[ln] = i0;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  } else {
    float(*sv)[K2] = S.rv;
    int(*si)[K2] = S.ri;
    float(*dv)[K2] = S.rv2;
    int(*di)[K2] = S.ri2;
    int nl = nrows;
    while (nl > 1) {
      const int npair = nl >> 1;
      for (int t = tid; t < npair * 2 * n2k; t += NTH) {
        const int pr = t / (2 * n2k), side = (t / n2k) & 1, pos = t - (2 * pr + side) * n2k;
        const float xv = sv[2 * pr + side][pos];
        const int xi = si[2 * pr + side][pos];
        const int o = 2 * pr + 1 - side;
        int lo = 0, hi = n2k;  // entries of list o better than x: a prefix of it
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (better(sv[o][mid], si[o][mid], xv, xi)) lo = mid + 1;
          else hi = mid;
        }
        const int slot = pos + lo;
        if (slot < n2k) {
          dv[pr][slot] = xv;
          di[pr][slot] = xi;
        }
      }
      if ((nl & 1) && tid < n2k) {  // an odd list out moves up unchanged
        dv[npair][tid] = sv[nl - 1][tid];
        di[npair][tid] = si[nl - 1][tid];
      }
      __syncthreads();
      float(*tv)[K2] = sv;
      int(*ti)[K2] = si;
      sv = dv;
      si = di;
      dv = tv;
      di = ti;
      nl = npair + (nl & 1);
    }
    if (tid < n2k) {
      S.cv[tid] = sv[0][tid];
      S.ci[tid] = si[0][tid];
    }
    __syncthreads();
  }
  stamp(5, (uint32_t)__builtin_amdgcn_s_memrealtime());

  // bookkeeping, one lane of wave 0 per ranked candidate c < 2k (the serial loops of
  // model.py:874-909 as ballots: a non-EOS candidate's slot is its rank among the non-EOS ones,
  // an EOS candidate's is (#non-EOS) + its rank among the EOS ones; slots >= k are dropped)
  if (wv == 0) {
    const int c = ln;
    const bool inr = c < n2k;
    int cc = inr ? S.ci[c] : 0;
    const bool bad = inr && (unsigned)cc >= (unsigned)(nrows * V);  // NaN rows leave empty slots
    if (bad) cc = 0;
    if (__ballot(bad) && ln == 0) atomicOr(a.err, CASR_DEV_BAD_CAND);
    const int beam = cc / V, tok = cc - beam * V;
    const bool f = inr && tok == eos;
    const float cs = inr ? S.cv[c] : 0.f;
    if (writer && c < k) {  // finished hypotheses among the first k candidates (model.py:874-889)
      const size_t ri = ((size_t)b * L + l) * k + c;
      a.rec_valid[ri] = f;
      if (f) {
        a.rec_score[ri] = cs;
        a.rec_src[ri] = beam;
      }
    }
    if (writer && ln == 0 && !a.topfin[b] && tok == eos) {  // model.py:897-901 (candidate 0)
      a.topfin[b] = 1;
      atomicAdd(&a.newdone[l], 1);
    }
    // active = first k non-EOS candidates in rank order, then EOS ones (model.py:904-909)
    const unsigned long long ne = __ballot(inr && !f), eo = __ballot(f);
    const unsigned long long below = (1ull << c) - 1ull;
    const int slot = f ? __popcll(ne) + __popcll(eo & below) : __popcll(ne & below);
    if (inr && slot < k) {
      const int row = b * k + slot;
      if (tok_l) {  // the fused caller's copy (attention.hip CELL 3, 4)
        tok_l[slot] = tok;
        src_l[slot] = b * k + beam;
      }
      if (writer) {
        a.tok_next[row] = tok;
        a.src_next[row] = b * k + beam;
        a.score_next[row] = cs;
        a.bp[(size_t)l * R + row] = beam;
        a.tk[(size_t)l * R + row] = tok;
      }
    }
    stamp(6, (uint32_t)__builtin_amdgcn_s_memrealtime());
  }
}


}  // namespace casr
