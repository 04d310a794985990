// Internal contracts between the casr host code (casr_capi.hip) and the kernel TUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "casr.h"

// the s16 arithmetic of this build (casr_common.h CASR_S16_ONE: the s16x1 build)
#ifndef CASR_S16_ONE
#define CASR_S16_ONE 0
#endif
constexpr int CASR_PREC_S16 = CASR_S16_ONE ? CASR_PREC_S16X1 : CASR_PREC_S16X3;

namespace casr {

// Dimensions of the deployed configuration (gpd.py), fixed at compile time so every
// tile loop unrolls.  casr_create rejects any other configuration (CASR_ERR_UNSUPPORTED).
constexpr int F = 80;     // n_mels
constexpr int D = 720;    // encoder input (3 ch x 3 frames x 80)
constexpr int H = 256;    // encoder hidden per direction
constexpr int C = 512;    // encoder output / context size (2H)
constexpr int HD = 512;   // decoder hidden
constexpr int E = 256;    // embedding
constexpr int A = 128;    // attention size
constexpr int KDEC = E + C + HD;  // 1280: decoder LSTM contraction [emb | ctx | h]
constexpr int KPROJ = C + HD;     // 1024: projection contraction [ctx | h]
constexpr int ST16 = C + HD + HD;  // offset of the s16 split words [ctx16 | h16] in a state row
constexpr int ST = ST16 + C + HD;  // 2560: per-row decoder state [ctx | h | c | ctx16 | h16]
constexpr int KMAX_BEAM = 16;

// Device guard bits: a data-dependent index (token id, predecessor row, back-pointer) out of
// range is clamped to a valid one and reported here instead of faulting the GPU.
constexpr int CASR_DEV_BAD_TOKEN = 1;    // decoder input token not in [0, V)
constexpr int CASR_DEV_BAD_SRC = 2;      // predecessor row not in [0, R)
constexpr int CASR_DEV_NAN_LOGITS = 4;   // no finite maximum in a logit row (greedy)
constexpr int CASR_DEV_BAD_CAND = 8;     // beam candidate index not in [0, k*V)
constexpr int CASR_DEV_BAD_BACKPTR = 16; // back-pointer walk left [0, k)
constexpr int CASR_DEV_REC_TIMEOUT = 32; // persistent recurrence: a bounded hand-off wait expired
constexpr int CASR_DEV_BAD_AUDIO = 64;   // front-end: n_samples < 513 (torch.stft raises) or > n_max
constexpr int CASR_DEV_F16_RANGE = 128;  // s16x3 path: a finite operand beyond the f16 range (>= 65520)

// MFMA-fragment-major weight block: a 16-row x 64-k tile stored as [q=0..3][lane][4] so
// lane l reads row (l&15), k = 16*(l>>4) + 4q + e with one coalesced 16 B load per q.
constexpr int FRAG = 16 * 64;

// Offsets (in floats) of every tensor inside the packed weight blob.
struct Layout {
  size_t enc_wih[CASR_MAX_LAYERS];   // [2*4H][Din]  row-major, gate-interleaved rows
  size_t enc_bias[CASR_MAX_LAYERS];  // [2*4H]       b_ih + b_hh, same row order
  size_t enc_whh[CASR_MAX_LAYERS];   // frag-major [2][H/16][4][H/64]
  size_t emb;                        // [V][E]
  size_t dec_w;                      // frag-major [HD/16][4][KDEC/64]
  size_t dec_b;                      // [4HD] gate-interleaved
  size_t proj_w;                     // frag-major [VP/64 * 4][KPROJ/64], k order [ctx | h]
  size_t proj_b;                     // [VP]
  size_t wencT;                      // [A][C]
  size_t wenc16;                     // [A][C/32][32 hi | 32 lo]: s16 row image of wencT (keys GEMM)
  size_t b_attn;                     // [A]
  size_t w_hidden;                   // [HD][A]
  size_t v;                          // [A]
  size_t info;                       // [64]: info[0] = 1 when the s16x3 images are valid
  // s16x3 images (casr_common.h split16) of the MFMA operands, same float count as the f32 ones
  size_t enc_wih16[CASR_MAX_LAYERS]; // [2*4H][Kp/32][32 hi | 32 lo], Kp = Din rounded up to 64
  size_t enc_whh16[CASR_MAX_LAYERS]; // s16 frag-major [2][H/16][4][H/64] (recurrence.hip)
  size_t emb16;                      // [V][E] split words (split16_word)
  size_t dec_w16;                    // s16 frag-major, same tiling / k order as dec_w
  size_t proj_w16;                   // s16 frag-major, same tiling / k order as proj_w
  size_t total;
  int layers, V, VP;
};

Layout make_layout(const casr_config& cfg);

// Tuning options of a handle (include/casr.h CASR_OPT_*): speed only, every value gives the same
// bits (CASR_OPT_ATTN_DIRECT: a numerics variant within the attention tolerance).
struct Tuning {
  int v[CASR_OPT_COUNT] = {1, 0, 1, -1, 2, 2, 2, 2, 0, 0, 1, 0, 0, 1, 1, 1, 1, 0, 0};
  int operator[](int i) const { return v[i]; }
};

// Packed row index of (gate g, unit u) for a gate-interleaved LSTM matrix with hidden
// size n_hidden: blocks of 16 units, each block = 4 gates x 16 units.
inline int packed_gate_row(int g, int u) { return (u / 16) * 64 + g * 16 + (u % 16); }
// Encoder input-projection column (Gin) of gate g of unit u within one direction: the four gates
// of a unit are adjacent (16-unit blocks of [unit][gate]), so a recurrence cell reads its gate
// pre-activations with one 16-B load instead of four 4-B loads (recurrence.hip, encoder.hip)
inline int enc_gate_col(int g, int u) { return (u / 16) * 64 + (u % 16) * 4 + g; }

// ---------------------------------------------------------------- launch timing
// Event pairs around launches of enabled kernel classes (casr_profile_enable).
// flush kernel of CASR_OPT_DIAG_COLD (fill.hip): reads n float4 of buf
hipError_t flush_caches(const void* buf, size_t bytes, hipStream_t s);

struct Profiler {
  uint32_t mask = 0;
  uint32_t cold_mask = 0;         // CASR_OPT_DIAG_COLD: classes launched after a cache flush
  const void* cold_buf = nullptr;  // the flush kernel's 1 GiB source
  size_t cold_bytes = 0;
  void cold(int cls, hipStream_t s) const {
    if (((cold_mask >> cls) & 1u) && cold_buf) (void)flush_caches(cold_buf, cold_bytes, s);
  }
  std::vector<hipEvent_t> ev[CASR_K_COUNT];
  std::vector<int> weight[CASR_K_COUNT];  // launches covered by each event pair
  size_t used[CASR_K_COUNT] = {};
  bool on(int cls) const { return (mask >> cls) & 1u; }
  // n > 1: the pair brackets a graph replay of n launches of this class (boundaries included)
  void mark(int cls, hipStream_t s, int n = 1) {
    if (!on(cls)) return;
    if (used[cls] == ev[cls].size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      ev[cls].push_back(e);
    }
    if ((used[cls] & 1) == 0) {
      if (weight[cls].size() <= used[cls] / 2) weight[cls].resize(used[cls] / 2 + 1);
      weight[cls][used[cls] / 2] = n;
    }
    (void)hipEventRecord(ev[cls][used[cls]++], s);
  }
  void reset() {
    for (int c = 0; c < CASR_K_COUNT; ++c) used[c] = 0;
  }
  ~Profiler() {
    for (auto& v : ev)
      for (hipEvent_t e : v) (void)hipEventDestroy(e);
  }
};

// RAII begin/end marker
struct ProfScope {
  Profiler* p;
  int cls;
  hipStream_t s;
  ProfScope(Profiler* p_, int c, hipStream_t s_, int n = 1) : p(p_), cls(c), s(s_) {
    if (p) {
      p->cold(cls, s);  // CASR_OPT_DIAG_COLD (measurement only): before the class's first event
      p->mark(cls, s, n);
    }
  }
  ~ProfScope() {
    if (p) p->mark(cls, s);
  }
};

// Instantiated hipGraphs keyed by everything a captured sequence bakes in (shapes, weight
// and workspace pointers, scalar arguments).  A key miss re-captures; a small LRU bound
// keeps stale entries (e.g. after a workspace grew) from piling up.
struct GraphCache {
  struct Entry {
    std::vector<uint64_t> key;
    hipGraphExec_t exec;
  };
  std::vector<Entry> entries;
  hipGraphExec_t find(const std::vector<uint64_t>& key) {
    for (size_t i = 0; i < entries.size(); ++i)
      if (entries[i].key == key) {
        if (i + 1 != entries.size()) std::swap(entries[i], entries.back());
        return entries.back().exec;
      }
    return nullptr;
  }
  void add(std::vector<uint64_t> key, hipGraphExec_t exec) {
    if (entries.size() >= 24) {
      (void)hipGraphExecDestroy(entries.front().exec);
      entries.erase(entries.begin());
    }
    entries.push_back(Entry{std::move(key), exec});
  }
  void clear() {
    for (auto& e : entries) (void)hipGraphExecDestroy(e.exec);
    entries.clear();
  }
  ~GraphCache() { clear(); }
};

// ---------------------------------------------------------------- kernel launchers
// fill.hip (graph-safe replacements for hipMemsetAsync)
hipError_t fill_u32(void* p, uint32_t v, size_t n_words, hipStream_t s);
hipError_t fill_u8(void* p, uint8_t v, size_t n_bytes, hipStream_t s);
// up to FILL_MAX_SEG fills (4-byte words or bytes) / device-to-device copies in one launch
constexpr int FILL_MAX_SEG = 8;
struct FillSeg {
  void* p;
  size_t count;    // elements
  uint32_t v;
  uint32_t bytes;  // element size: 4 or 1
};
struct FillList {
  FillSeg seg[FILL_MAX_SEG];
  int n = 0;
  void add32(void* p, uint32_t v, size_t n_words) { seg[n++] = FillSeg{p, n_words, v, 4}; }
  void add8(void* p, uint8_t v, size_t n_bytes) { seg[n++] = FillSeg{p, n_bytes, v, 1}; }
};
hipError_t fill_multi(const FillList& fl, hipStream_t s);
struct CopySeg {
  void* dst;
  const void* src;
  size_t bytes;
};
struct CopyList {
  CopySeg seg[FILL_MAX_SEG];
  int n = 0;
  void add(void* dst, const void* src, size_t bytes) { seg[n++] = CopySeg{dst, src, bytes}; }
};
hipError_t copy_multi(const CopyList& cl, hipStream_t s);

// frontend.hip: wav -> log-mel.  Constant tables live in one device struct per handle.
constexpr int FE_FBW = 20;  // widest mel filter kept (nonzero bins; the widest has 17)
struct FrontendConst {
  float fb[F][FE_FBW];          // filter m's nonzero weights, bins lo[m] .. hi[m] - 1
  int32_t lo[F], hi[F];         // nonzero bin range of each mel filter
  float win[400];               // periodic hann(400)
  float tw256r[256], tw256i[256];  // exp(-2 pi i k / 256), rounded once from double
  float tw512r[257], tw512i[257];  // exp(-2 pi i q / 512)
};
void mel_filterbank(int n_stft, float f_min, float f_max, int n_mels, float* fb);
void build_frontend_const(FrontendConst* c);
int frontend_frames(int n_samples);
// form: 1 = the 16-lane kernel (default), 0 = one wave per frame (round 4); the same bits
hipError_t launch_log_mel(const float* wav, const int32_t* nsamp, int B, int Nmax, int Tmax, float pre,
                          const FrontendConst* k, float* out, int32_t* frames, int32_t* err, hipStream_t s,
                          int form = 1);

// features.hip
// the layer-0 s16 row image straight from fbank (features_rows_kernel<true>, T <= 1024)
bool features_x16_supported(int T);
// stats: [B][2][D] floats of scratch (per-utterance mean and std + eps of the 720 dimensions)
hipError_t launch_features_x16(const float* fbank, const int32_t* frames, int B, int T, float eps,
                               int32_t* feat_len, float* stats, uint16_t* x16, int Kp, int32_t* err, hipStream_t s,
                               int km = 0);
hipError_t launch_features(const float* fbank, const int32_t* frames, int B, int T, float eps,
                           float* feat, int32_t* feat_len, float* stats, hipStream_t s);
hipError_t launch_gather_utts(const float* const* ptrs, const int32_t* lens, int B, int Tp,
                              float* feat, hipStream_t s);

// encoder.hip
hipError_t launch_input_proj(const float* X, int M, int Din, const float* W, const float* bias,
                             float* Gin, hipStream_t s);
// s16 images of an activation or weight matrix with rows R and Kp (multiple of 64) k per row, in one
// of two layouts (the same words): the row image [R][Kp / 32][32 hi | 32 lo] halves, or (km, round
// 5, CASR_OPT_X16_KM) 16-k-block major [Kp / 16][R][16 hi | 16 lo], in which 16 consecutive rows of
// one 16-k block are 1 KB contiguous (whole 128-B lines for the input GEMM's 16-deep stages).
// x16_km: whether one encode uses the 16-k-major layout (the ping-pong input GEMM, the balanced tail
// and the row-streaming keys form read it; the other forms take row images)
inline bool x16_km(const Tuning& t) {
  return t[CASR_OPT_X16_KM] && t[CASR_OPT_GEMM16_PERSIST] == 2 && t[CASR_OPT_GEMM16_TAIL] != 1 &&
         t[CASR_OPT_KEYS_ROWS];
}
// gemm16.hip: the s16x3 input projection on 256 x 256 tiles; X16 / W16 are s16 images with Kp
// (multiple of 64) k per row (km: both 16-k-block major, X16 with M rows).  K: the real input width
// (the images are zero from K to Kp); 0 = Kp.  persist / tail: CASR_OPT_GEMM16_PERSIST / _TAIL
hipError_t launch_input_proj_s16_big(const float* X16, int M, int Kp, const float* W16, const float* bias,
                                     float* Gin, hipStream_t s, int K, int persist, int tail, int km = 0,
                                     int lean = 0);
// a row-image weight matrix [R][Kp] -> its 16-k-block-major image (bind time)
hipError_t launch_relayout_km16(const float* rowimg, int R, int Kp, float* km, hipStream_t s);
hipError_t launch_split_rows(const float* X, int ldx, int M, int K, int Kp, uint16_t* out, int32_t* err,
                             hipStream_t s, int km = 0);
inline int s16_kpad(int K) { return (K + 63) / 64 * 64; }  // even number of 32-k tiles (gemm16.hip)
hipError_t launch_rec_step(const float* Whh_f, const float* Gin, const float* xin, float* out,
                           const float* hprev, float* hnext, float* cst, float* hfin,
                           const int32_t* lens, int B, int Tp, int step, int residual, int row0,
                           int row1, int s16, hipStream_t s);
// recurrence.hip: persistent per-layer recurrence (all Tp steps in one launch).  `layout` is the
// resolved workgroup shape rec_layout(B, opt) returns: 0 = 32 rows x 16 units, 1 = 16 x 32, 2 = 16 x 16
int rec_layout(int B, const Tuning& t);
size_t rec_layer_granule_bytes(int B, int layout);
int rec_layer_grid_blocks(int B, int layout);
int rec_layer_waves(int layout);      // waves per workgroup (trace layout)
int rec_layer_producers(int layout);  // workgroups per row group (trace layout)
bool rec_layer_fits(int B, int layout);  // the persistent grid for batch B is resident at once (one launch)
hipError_t reset_rec_layer(uint32_t* hx, int B, int layout, hipStream_t s);  // before EVERY launch_rec_layer
// x16 (s16 only, may be null): also write out's s16 row image [B*Tp][C/32][32 hi | 32 lo] (the
// next layer's input-GEMM operand, zeros past each length), replacing a split_rows pass.
// With t[CASR_OPT_REC_COOP] the launch is cooperative: a grid that cannot be co-resident returns
// an error (hipErrorCooperativeLaunchTooLarge) instead of spinning into the hand-off timeout.
hipError_t launch_rec_layer(const float* Whh_f, const float* Gin, const float* xin, float* out,
                            uint16_t* x16, uint32_t* hx, float* hfin, float* cst, const int32_t* lens, int B, int Tp,
                            int residual, int s16, int32_t* err, uint32_t* trace, int layout, const Tuning& t,
                            hipStream_t s, int km = 0);
// enc16: the encoder output's s16 image (km: 16-k-block major; rows = 1 only)
hipError_t launch_keys_s16(const float* enc16, int B, int Tp, const float* wenc16, const float* b_attn,
                           float* keysT, hipStream_t s, int rows = 1, int km = 0);
hipError_t launch_keys(const float* enc, int B, int Tp, const float* wencT, const float* b_attn,
                       float* keysT, hipStream_t s);

// decoder.hip
// projection column blocks (5 x 16 columns each) whose per-row partials the selects combine: V <= 5120
constexpr int GP_NB = 64;
struct GreedyPart {
  float* mx;    // [R][GP_NB] block maximum of the row's logits
  float* se;    // [R][GP_NB] sum exp(x - block maximum)
  int32_t* ix;  // [R][GP_NB] first column of the block maximum
  float* tmx;   // [R][GP_NT] maximum of each 16-column tile (beam at temperature 1), or nullptr
};
constexpr int GP_NT = 320;  // 16-column tiles per row (V <= 5120)

// a beam select's operands and outputs (beam_select.h; beam_select_kernel's argument, and the
// folded beam attention's prologue select, AttnCell::bs)
struct BeamSelArgs {
  const float* logits;
  int V, B, k, l, L, eos;
  float temperature;
  const float* score_cur;
  float* score_next;
  int32_t* tok_next;
  int32_t* src_next;
  uint8_t* topfin;
  int32_t* bp;
  int32_t* tk;
  float* rec_score;
  int32_t* rec_src;
  uint8_t* rec_valid;
  int32_t* newdone;
  int32_t* err;
  GreedyPart gp;
  int nbp;
};

// Greedy select of step lsel fused into a later kernel of step lsel + 1 (the LSTMCell GEMM's
// prologue, decoder.hip DecLstmA; or the folded step's attention kernel, attention.hip): the
// projection's per-block row partials of step lsel are reduced by the consumer itself and the
// bookkeeping of greedy_select_part_kernel (model.py:540-590) is done by one writer per row.
struct GreedySel {
  GreedyPart gp;
  int nbp, lsel, L, eos;
  uint8_t* fin;
  int32_t* out_len;
  float* accum;
  int32_t* tokens;
  int32_t* newdone;
};

#ifdef __HIPCC__
// the writer's bookkeeping of row r once its token t and log-probability lp are known (lane 0
// only): tokens, finished, lengths, score and the newly-finished counter, as model.py:554-578
__device__ __forceinline__ void greedy_book(const GreedySel& gs, int r, int t, float lp, uint8_t fin0, float acc0,
                                            int len0) {
  gs.tokens[(size_t)r * gs.L + gs.lsel] = t;
  const bool was = fin0 != 0;
  const bool cur = t == gs.eos;
  float acc = acc0;
  if (!was && cur) acc = acc + lp;  // model.py:567
  const bool now = was || cur;
  if (!now) {
    gs.out_len[r] = len0 + 1;  // model.py:573
    acc = acc + lp;            // model.py:576
  }
  gs.accum[r] = acc;
  if (now && !was) {
    gs.fin[r] = 1;
    atomicAdd(&gs.newdone[gs.lsel], 1);
  }
}
#endif

// Folded greedy decode (CASR_OPT_DEC_FOLD): per step l >= 1 two launches instead of three.
//   KA (attention.hip, attention_kernel<1, true>): select of step l-1 from the projection
//      partials, gates = gates_prev[r] + emb_gates[tok] (the per-token table: emb . W_emb^T +
//      b_ih + b_hh), the LSTM cell, q = h . W_hidden by f32 fma chains, then the attention.
//   KB (decoder.hip, dgemm_kernel<.., FoldEpi>): [ctx | h] . [W_p ; W_ch]^T on one fused
//      fragment image: the vocabulary tiles (greedy partials) and the LSTM gate tiles of the next
//      step (K = 1024: the ctx | h part of the LSTM contraction, decoder.py:104-114), one GEMM
//      over the same A rows.
constexpr int FOLD_GT = 4 * HD / 16;  // LSTM gate tiles (16 gate rows each) in the fused image
constexpr int FOLD_NT = 7;            // 16-column tiles per fused GEMM block (112 columns)
inline int fold_vtiles(int V) { return (V + 15) / 16; }
// (round 4) the gate tiles of the fused image start at the vocabulary tiles rounded up to a whole
// 7-tile wave column (zero tiles between): no wave column holds both vocabulary and gate tiles, so
// the fused GEMM's epilogue has no mixed column, the one that ended last
inline int fold_gtile0(int V) { return (fold_vtiles(V) + FOLD_NT - 1) / FOLD_NT * FOLD_NT; }
// bytes of one fused image (s16 or f32: the same tiling)
inline size_t fold_image_bytes(int V) { return (size_t)(fold_gtile0(V) + FOLD_GT) * (KPROJ / 64) * FRAG * sizeof(float); }
constexpr size_t FOLD_WQ16_FLOATS = (size_t)A * HD;  // the W_hidden fragment image (beam query)
struct FoldBufs {
  const float* wfold;      // fragment image (s16, or f32 under the exact-f32 arithmetic):
                           // [fold_gtile0(V) + FOLD_GT tiles][KPROJ / 64] FRAG blocks
  const float* emb_gates;  // [V][4 HD] packed gate-row order (packed_gate_row), biases included
  const float* wq16;       // s16 fragment image of W_hidden^T: [A / 16 tiles][HD / 64] FRAG blocks
  float* gates;            // [R][4 HD] the next step's [ctx | h] . W_ch^T, packed gate-row order
};
// build the fused images and the per-token gate table from a bound blob: wfold and wq16 from the s16
// images, wfold32 from the f32 fragment images (the folded greedy step under the exact-f32
// arithmetic), emb_gates from the embedding and the decoder LSTM weights; each nullptr is skipped
hipError_t build_fold(const float* W, const Layout& L, int V, float* wfold, float* emb_gates, float* wq16,
                      float* wfold32, hipStream_t s);

// the greedy folded GEMM's k split at R <= 32 (decoder.hip dgemm_kernel KS): DG_KS blocks per
// output block, at most DG_KS_GROUPS output blocks of 2 epilogue waves
constexpr int DG_KS = 4, DG_KS_GROUPS = 64, DG_KS_COUNTERS = 2 * DG_KS_GROUPS;
constexpr size_t DG_KS_PART_BYTES = (size_t)DG_KS_COUNTERS * DG_KS * FOLD_NT * 64 * 16;  // f32x4 per lane

struct DecodeBufs {
  float* st[2];          // [R][ST]
  float* logits;         // [R][V]
  GreedyPart part;       // per-block row partials of the projection (after the logits)
  float* qpart;          // [dec_q_slots(R)][R][A] attention query partials, one per LSTMCell column block
  int32_t* tok[2];       // [R]
  int32_t* src[2];       // [R]
  float* score[2];       // [R]
  int32_t* newdone;      // [max_len] rows/utterances newly finished at each step
  int32_t* err;          // [1] CASR_DEV_* guard bits set by kernels (casr_debug_flags)
  // greedy
  uint8_t* fin;          // [R]
  // beam
  uint8_t* topfin;       // [B]
  int32_t* bp;           // [L][R]
  int32_t* tk;           // [L][R]
  float* rec_score;      // [B][L][k]
  int32_t* rec_src;      // [B][L][k]
  uint8_t* rec_valid;    // [B][L][k]
  // greedy at R <= 32 with CASR_OPT_DEC_KSPLIT: the k-range sums and arrival counters (else nullptr)
  float* kspart;         // [groups][2 waves][DG_KS][FOLD_NT tiles][64 lanes] x 4 floats
  int32_t* kscnt;
  // greedy at R <= 64 with CASR_OPT_ATTN_SPLIT: the split attention's partials and counters (else nullptr)
  float* aspart;         // [R][AT_SPLIT_MAX][C + 4]
  int32_t* ascnt;        // [R]
  int asplit;            // splits asked for (8 at R <= 32, 4 at R <= 64)
};

struct DecodeArgs {
  const float* W;        // packed blob base
  Layout L;
  const float* enc;      // [B][Tp][C]
  const float* keysT;    // [B][A][Tp]
  const float* hfin;     // [2][B][H]
  const float* cfin;     // [2][B][H]
  const int32_t* lens;   // [B]
  int B, Tp, k, V, max_len, sos, eos;
  float temperature;
  int s16;               // decoder GEMMs on the s16x3 images (casr_set_precision)
  Profiler* prof;        // may be null
  int greedy_run;        // set by run_greedy: the projection writes per-block argmax partials
  int fuse_select;       // CASR_OPT_FUSE_SELECT
  int attn_kpb;          // CASR_OPT_ATTN_KPB (0 auto)
  int attn_direct;       // CASR_OPT_ATTN_DIRECT
  int proj_small;        // every |W_p| < 16 (blob info word 4): the one-accumulator s16x3 projection
  int fold;              // CASR_OPT_DEC_FOLD in effect (greedy, s16x3, tables built)
  FoldBufs fb;           // fold tables and the gates buffer (fold only)
};

// attention.hip: one decode step's additive attention for all R rows (writes ctx into st)
// decode rows at which the LSTMCell (128 x 128) and projection (256 x 160) blocks of decoder.hip
// fill the CUs in one round; below it the narrower blocks do
inline bool dec_wide(int R) { return R >= 2048; }
// attention query partials per decoder row: one per LSTMCell column block (decoder.hip
// launch_dec_lstm), 16 units each, 32 units at dec_wide(R)
inline int dec_q_slots(int R) { return dec_wide(R) ? HD / 32 : HD / 16; }
hipError_t launch_attention_step(const DecodeArgs& a, float* st, const float* qpart, float* align,
                                 int32_t* newdone, int l, int total, hipStream_t s);
// the folded step's attention (KA above): st_old supplies c, st receives h, c and ctx.  Greedy
// (k = 1): sel = the fused select of step gs.lsel (else tokens from tok).  Beam (k > 1, 4 or 8 rows
// per block): tokens and predecessor rows from the beam select (tok, src)
struct AttnCell {
  const float* st_old;
  const float* gates;
  const float* emb_gates;
  const float* w_hidden;  // [HD][A]
  const float* wq16;      // beam: FoldBufs::wq16
  const int32_t* tok;     // sel == 0 (beam: the select's tokens of the block's rows)
  const int32_t* src;     // beam: the predecessor row of each row (gates_prev and c are read there)
  int32_t* err;
  int sel;
  GreedySel gs;
  int bsel;        // beam, one block per utterance: the select of step l - 1 runs in the prologue (bs)
  BeamSelArgs bs;
  // greedy, CASR_OPT_ATTN_SPLIT (round 6): split > 1 blocks of tc steps per utterance, their
  // (max, sum, context) partials [B][AT_SPLIT_MAX][C + 4] and per-utterance arrival counters
  int split, tc;
  float* spart;
  int32_t* scnt;
};
constexpr int AT_SPLIT_MAX = 8;
hipError_t launch_attention_cell_step(const DecodeArgs& a, float* st, const AttnCell& cell, float* align,
                                      int32_t* newdone, int l, int total, hipStream_t s);
// fixed LDS of the attention launch; cell = 1: the folded greedy step's attention_kernel<1, 1>
// (its cell-phase area on top; CELL 2 keeps its cell data in the score scratch)
size_t attention_smem_bytes(int B, int k, int Tp, int opt, int cell = 0);
int attention_kpb(int B, int k, int opt);  // beam rows per attention block
void attn_trace_bind(uint32_t* buf);  // CASR_DG_TRACE diagnostics (attention.hip)

void dg_trace_init();  // decoder.hip, CASR_DG_TRACE diagnostics
void dg_trace_dump();
hipError_t run_greedy(const DecodeArgs& a, DecodeBufs& d, int32_t* tokens, int32_t* out_len,
                      uint8_t* finished, float* accum, float* align, hipStream_t s);
hipError_t run_beam(const DecodeArgs& a, DecodeBufs& d, float lm_weight, float length_weight,
                    int32_t* best_tokens, int32_t* best_len, float* best_score, int32_t* steps,
                    hipStream_t s);
hipError_t run_beam_records(const DecodeArgs& a, DecodeBufs& d, int32_t* rec_tokens,
                            float* rec_score, uint8_t* rec_valid, hipStream_t s);

}  // namespace casr
