// Host side of the casr C ABI (include/casr.h): weight packing into kernel layouts,
// per-handle device workspaces, and the encode / decode drivers.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "casr.h"
#include "casr_internal.h"

namespace casr {


// version word of the packed layout (bump whenever make_layout or a packer changes)
constexpr uint32_t LAYOUT_MAGIC = 0xCA5B0003u;

Layout make_layout(const casr_config& cfg) {
  Layout L{};
  size_t off = 0;
  auto take = [&](size_t n) {
    const size_t o = off;
    off += (n + 63) & ~size_t(63);  // 256 B alignment for every tensor
    return o;
  };
  L.layers = cfg.enc_layers;
  L.V = cfg.vocab;
  L.VP = (cfg.vocab + 63) / 64 * 64;
  for (int l = 0; l < cfg.enc_layers; ++l) {
    const int din = l == 0 ? D : C;
    L.enc_wih[l] = take((size_t)8 * H * din);
    L.enc_bias[l] = take((size_t)8 * H);
    L.enc_whh[l] = take((size_t)2 * 4 * H * H);
  }
  L.emb = take((size_t)cfg.vocab * E);
  L.dec_w = take((size_t)4 * HD * KDEC);
  L.dec_b = take((size_t)4 * HD);
  L.proj_w = take((size_t)L.VP * KPROJ);
  L.proj_b = take((size_t)L.VP);
  L.wencT = take((size_t)A * C);
  L.b_attn = take((size_t)A);
  L.w_hidden = take((size_t)HD * A);
  L.v = take((size_t)A);
  L.info = take(64);
  for (int l = 0; l < cfg.enc_layers; ++l) {
    const int din = l == 0 ? D : C;
    L.enc_wih16[l] = take((size_t)8 * H * s16_kpad(din));
    L.enc_whh16[l] = take((size_t)2 * 4 * H * H);
  }
  L.emb16 = take((size_t)cfg.vocab * E);
  L.dec_w16 = take((size_t)4 * HD * KDEC);
  L.proj_w16 = take((size_t)L.VP * KPROJ);
  L.wenc16 = take((size_t)A * C);
  L.total = off;
  return L;
}

// Write a [N][K] matrix (element accessor f(n, k), rows >= N zero) in MFMA-fragment-major
// order: 16-row x 64-k blocks, block (nt, kc) at (nt*NKC + kc)*FRAG, inside [q][lane][4]
// with lane row = lane&15, k = 16*(lane>>4) + 4q + e.
template <class Fn>
static void pack_frag(float* dst, int NT, int NKC, Fn f) {
  for (int nt = 0; nt < NT; ++nt)
    for (int kc = 0; kc < NKC; ++kc) {
      float* blk = dst + ((size_t)nt * NKC + kc) * FRAG;
      for (int q = 0; q < 4; ++q)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < 4; ++e) {
            const int n = nt * 16 + (lane & 15);
            const int k = kc * 64 + 16 * (lane >> 4) + 4 * q + e;
            blk[(q * 64 + lane) * 4 + e] = f(n, k);
          }
    }
}

// ---- s16x3 images (casr_common.h split16), host side: hi = f16_rn(x), lo = f16_rn((x - hi) 2^11)
static void split16_host(float x, uint16_t& hi, uint16_t& lo) {
  const _Float16 h = (_Float16)x;
  const float r = (x - (float)h) * 2048.0f;
  const _Float16 l = (r == r && std::fabs(r) < 65504.f) ? (_Float16)r : (_Float16)0.f;
  std::memcpy(&hi, &h, 2);
  std::memcpy(&lo, &l, 2);
}

// [N][K] (accessor f(n, k)) as s16 row images [N][Kp/32][32 hi | 32 lo], zeros past K
template <class Fn>
static void pack_rows16(float* dst, int N, int K, Fn f) {
  const int Kp = s16_kpad(K);
  uint16_t* o = reinterpret_cast<uint16_t*>(dst);
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < Kp; ++k) {
      uint16_t hi = 0, lo = 0;
      if (k < K) split16_host(f(n, k), hi, lo);
      uint16_t* t = o + (size_t)n * Kp * 2 + (k / 32) * 64 + (k % 32);
      t[0] = hi;
      t[32] = lo;
    }
}

// [N][K] in s16 fragment-major order: 16-row x 64-k blocks of FRAG floats, block (nt, kc) =
// [j = 0..1][hl = hi, lo][lane][8 halves] with lane row = lane & 15 and
// k = kc*64 + 16*(lane >> 4) + 8j + e: lane l's v_mfma_f32_16x16x32_f16 B operand for k-step j
// is one 16-B load, and its 16 k (both steps) are the 16 consecutive k of its f32 fragment row.
template <class Fn>
static void pack_frag16(float* dst, int NT, int NKC, Fn f) {
  uint16_t* o = reinterpret_cast<uint16_t*>(dst);
  for (int nt = 0; nt < NT; ++nt)
    for (int kc = 0; kc < NKC; ++kc) {
      uint16_t* blk = o + ((size_t)nt * NKC + kc) * FRAG * 2;
      for (int j = 0; j < 2; ++j)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < 8; ++e) {
            uint16_t hi, lo;
            split16_host(f(nt * 16 + (lane & 15), kc * 64 + 16 * (lane >> 4) + 8 * j + e), hi, lo);
            blk[((j * 2 + 0) * 64 + lane) * 8 + e] = hi;
            blk[((j * 2 + 1) * 64 + lane) * 8 + e] = lo;
          }
    }
}

}  // namespace casr

using namespace casr;

namespace {

thread_local std::string g_err;

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace

struct casr_handle {
  casr_config cfg{};
  Layout L{};
  int device = 0;
  const float* W = nullptr;
  std::string err;
  // encoder workspace
  DevBuf gin, out0, out1, hbuf, cst, hfin, keysT, lens;
  DevBuf feat;     // casr_encode_fbank outside the s16x3 image path: the f32 features
  DevBuf fstat;    // feature statistics scratch [B][2][D] (features.hip)
  DevBuf hx;       // persistent recurrence: tagged h words [3][2][Bp][H]
  // device guard bits, one word per source: [0] decode, [1] encoder + features, [2] front end.
  // Allocated and zeroed once; kernels OR bits in; casr_device_flags reads and clears them, so
  // they cover every call since the previous read (never reset inside a captured graph)
  DevBuf gflags;
  DevBuf fe_const; // FrontendConst (filterbank, window, twiddles), built on first casr_log_mel
  bool use_persistent = true;
  int precision = CASR_PREC_S16;  // requested (casr_set_precision)
  bool s16_valid = false;           // the bound blob's s16 images are usable (Layout::info)
  bool proj_small = false;          // every |W_p| < 16 (Layout::info + 4)
  bool dec_small = false;           // every decoder LSTM weight < 16 (Layout::info + 5)
  DevBuf x16;                       // s16 image of the current layer input [B*Tp][Kp] (or 16-k-block major)
  // the encoder layers' W_ih s16 images 16-k-block major (CASR_OPT_X16_KM), built at bind from an
  // s16-valid blob: layer l at wih16km_off[l]
  DevBuf wih16km;
  size_t wih16km_off[CASR_MAX_LAYERS] = {};
  // folded greedy decode (CASR_OPT_DEC_FOLD): fused projection | LSTM-gate fragment image and the
  // per-token gate table, built at bind from an s16-valid blob; the gates buffer [R][4 HD]
  DevBuf wfold, egates, fgates, wq16;
  bool fold_ready = false;
  // (round 4) the f32 fused image: the folded greedy step under the exact-f32 arithmetic
  DevBuf wfold32;
  DevBuf coldbuf;  // CASR_OPT_DIAG_COLD's flush source (measurement only)
  bool fold32_ready = false;
  bool s16() const { return precision == CASR_PREC_S16 && s16_valid; }
  int B = 0, Tp = 0;
  bool encoded = false;
  float* enc_out = nullptr;  // out0 or out1
  // decoder workspace
  DevBuf st, logits, small, bp, tk, rec, beam_small;
  DevBuf ksbuf;  // the greedy folded GEMM's k-split sums and counters (R <= 32, CASR_OPT_DEC_KSPLIT)
  DevBuf asbuf;  // the split greedy attention's partials and counters (R <= 64, CASR_OPT_ATTN_SPLIT)
  DecodeBufs d{};
  DevBuf gout;  // internal decode outputs written by captured graphs
  Profiler prof;
  int dec_k = 0;
  bool beam_done = false;
  // hipGraph replay of the launch-bound loops (per-layer recurrence, decode loop)
  // casr_set_graphs bits: 1 = the decode loop replays as a hipGraph, 2 = the per-step recurrence
  // fallback does.  Default 2: the decode loop launches eagerly (measured faster)
  int graph_mode = CASR_GRAPHS_RECURRENCE;
  hipStream_t cap = nullptr;      // capture stream
  hipStream_t xs[2] = {};         // replay streams, fenced to the caller's stream by events
  hipEvent_t ev_in = nullptr, ev_out[2] = {};
  GraphCache graphs;
  Tuning tune;  // casr_set_option
};

static int fail(casr_handle* h, int code, const char* fmt, ...);

// the handle's guard words (allocated and zeroed on first use; the caller has set the device)
static int32_t* guard_words(casr_handle* h) {
  if (!h->gflags.p) {
    if (h->gflags.ensure(64) != hipSuccess) return nullptr;
    if (hipMemset(h->gflags.p, 0, 64) != hipSuccess) {
      h->gflags.release();
      return nullptr;
    }
  }
  return h->gflags.as<int32_t>();
}
#define GUARD(h, i) (guard_words(h) + (i))

// Capture `body(stream)` once per key into a hipGraph on the handle's private capture stream,
// then replay it on the private replay stream, ordered after everything already enqueued on
// the caller's stream and before anything enqueued there afterwards (event fences both
// ways; the caller's stream may be the legacy null stream, which a graph is not launched on).
template <class Body>
static hipError_t get_graph(casr_handle* h, const std::vector<uint64_t>& key, Body&& body,
                            hipGraphExec_t* out) {
  hipError_t e;
  if (!h->cap) {
    e = hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipStreamCreateWithFlags(&h->xs[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&h->ev_out[i], hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  hipGraphExec_t exec = h->graphs.find(key);
  if (!exec) {
    e = hipStreamBeginCapture(h->cap, hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) return e;
    hipError_t eb = body(h->cap);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(h->cap, &g);
    if (eb != hipSuccess) e = eb;
    if (e == hipSuccess) e = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (e != hipSuccess) return e;
    h->graphs.add(key, exec);
  }
  *out = exec;
  return hipSuccess;
}

// Replay n (<= 2) graphs concurrently, graph i on replay stream i, all after the work already
// on `s` and before anything enqueued on `s` afterwards.
static hipError_t launch_graphs(casr_handle* h, const hipGraphExec_t* ex, int n, hipStream_t s) {
  hipError_t e = hipEventRecord(h->ev_in, s);
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    e = hipStreamWaitEvent(h->xs[i], h->ev_in, 0);
    if (e == hipSuccess) e = hipGraphLaunch(ex[i], h->xs[i]);
    if (e == hipSuccess) e = hipEventRecord(h->ev_out[i], h->xs[i]);
  }
  for (int i = 0; i < n && e == hipSuccess; ++i) e = hipStreamWaitEvent(s, h->ev_out[i], 0);
  return e;
}

template <class Body>
static hipError_t run_graph(casr_handle* h, const std::vector<uint64_t>& key, hipStream_t s, Body&& body) {
  hipGraphExec_t exec = nullptr;
  hipError_t e = get_graph(h, key, body, &exec);
  return e == hipSuccess ? launch_graphs(h, &exec, 1, s) : e;
}

static int fail(casr_handle* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  g_err = buf;
  return code;
}

#define HIP_OK(h, expr)                                                                \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail((h), CASR_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                  __FILE__, __LINE__);                                                 \
  } while (0)

static int check_config(const casr_config* c) {
  if (!c) return fail(nullptr, CASR_ERR_ARG, "config is NULL");
  if (c->n_mels != F || c->feat_dim != D || c->enc_hidden != H || c->dec_hidden != HD ||
      c->embed_dim != E || c->attn_size != A)
    return fail(nullptr, CASR_ERR_UNSUPPORTED,
                "this build implements n_mels=80 feat_dim=720 enc_hidden=256 dec_hidden=512 "
                "embed_dim=256 attn_size=128 (got %d %d %d %d %d %d)",
                c->n_mels, c->feat_dim, c->enc_hidden, c->dec_hidden, c->embed_dim, c->attn_size);
  if (c->enc_layers < 1 || c->enc_layers > CASR_MAX_LAYERS || c->vocab < 4 || c->max_len < 1 ||
      c->sos < 0 || c->sos >= c->vocab || c->eos < 0 || c->eos >= c->vocab || !(c->temperature > 0.f))
    return fail(nullptr, CASR_ERR_ARG, "invalid config (layers=%d vocab=%d max_len=%d)",
                c->enc_layers, c->vocab, c->max_len);
  return CASR_OK;
}

extern "C" {

int casr_api_version(void) { return CASR_API_VERSION; }

size_t casr_packed_weights_floats(const casr_config* cfg) {
  if (check_config(cfg) != CASR_OK) return 0;
  return make_layout(*cfg).total;
}

int casr_pack_weights(const casr_config* cfg, const casr_weights_host* w, float* out) {
  int rc = check_config(cfg);
  if (rc) return rc;
  if (!w || !out) return fail(nullptr, CASR_ERR_ARG, "weights/out is NULL");
  const Layout L = make_layout(*cfg);
  // the s16x3 images need every MFMA weight inside the f16 range with room to spare; blob word
  // L.info records whether they are usable (casr_bind_weights reads it)
  // (the input projection's images need |w| < 16: gemm16.hip scales w_hi by 2^11 in f16)
  auto in_range = [](const float* p, size_t n, float lim = 16384.f) {
    for (size_t i = 0; i < n; ++i)
      if (!(std::fabs(p[i]) < lim)) return false;
    return true;
  };
  bool s16_ok = true;
  for (int l = 0; l < cfg->enc_layers; ++l)
    for (int d = 0; d < 2; ++d)
      if (w->enc_w_ih[l][d] && w->enc_w_hh[l][d] &&
          (!in_range(w->enc_w_ih[l][d], (size_t)4 * H * (l == 0 ? D : C), 16.f) ||
           !in_range(w->enc_w_hh[l][d], (size_t)4 * H * H)))
        s16_ok = false;
  if (w->embedding && w->dec_w_ih && w->dec_w_hh && w->proj_w &&
      (!in_range(w->embedding, (size_t)cfg->vocab * E) || !in_range(w->dec_w_ih, (size_t)4 * HD * (E + C)) ||
       !in_range(w->dec_w_hh, (size_t)4 * HD * HD) || !in_range(w->proj_w, (size_t)cfg->vocab * KPROJ)))
    s16_ok = false;
  // keys GEMM (encoder.hip gemm_nt_kernel<KeysEpi, true>): two accumulators, no 2^11 scaling of
  // w_hi, so the f16 range limit of the other s16 images applies
  if (w->attn_w_enc && !in_range(w->attn_w_enc, (size_t)C * A)) s16_ok = false;
  std::memset(out, 0, L.total * sizeof(float));
  out[L.info] = s16_ok ? 1.f : 0.f;
  // info word 4: every projection weight below 16 in magnitude, so w_hi 2^11 is an f16 and the
  // beam projection can run its one-accumulator s16x3 form (decoder.hip dgemm_kernel ONE)
  out[L.info + 4] = (w->proj_w && in_range(w->proj_w, (size_t)cfg->vocab * KPROJ, 16.f)) ? 1.f : 0.f;
  // info word 5: every decoder LSTM weight below 16 in magnitude: with word 4 the folded beam step's
  // fused GEMM (projection | LSTM gates) can run the one-accumulator form (decoder.hip FoldEpi)
  out[L.info + 5] = (w->dec_w_ih && w->dec_w_hh && in_range(w->dec_w_ih, (size_t)4 * HD * (E + C), 16.f) &&
                     in_range(w->dec_w_hh, (size_t)4 * HD * HD, 16.f))
                        ? 1.f
                        : 0.f;
  // layout stamp: casr_bind_weights refuses a blob packed by a build with another layout
  const uint32_t stamp[3] = {LAYOUT_MAGIC, (uint32_t)(L.total & 0xFFFFFFFFu), (uint32_t)(L.total >> 32)};
  std::memcpy(out + L.info + 1, stamp, sizeof stamp);
  const int V = cfg->vocab;
  for (int l = 0; l < cfg->enc_layers; ++l) {
    const int din = l == 0 ? D : C;
    for (int d = 0; d < 2; ++d)
      if (!w->enc_w_ih[l][d] || !w->enc_w_hh[l][d] || !w->enc_b_ih[l][d] || !w->enc_b_hh[l][d])
        return fail(nullptr, CASR_ERR_ARG, "encoder layer %d dir %d: NULL tensor", l, d);
    // input projection rows: d*4H + packed(g, u) <- W_ih_d[g*H + u]
    for (int d = 0; d < 2; ++d)
      for (int g = 0; g < 4; ++g)
        for (int u = 0; u < H; ++u) {
          const int pr = d * 4 * H + enc_gate_col(g, u);
          const int orow = g * H + u;
          std::memcpy(out + L.enc_wih[l] + (size_t)pr * din, w->enc_w_ih[l][d] + (size_t)orow * din,
                      sizeof(float) * din);
          out[L.enc_bias[l] + pr] = w->enc_b_ih[l][d][orow] + w->enc_b_hh[l][d][orow];
        }
    // recurrent matrices, fragment-major per direction: n-tile (jb*4 + g) = gate g of units
    // jb*16 .. jb*16+15
    for (int d = 0; d < 2; ++d) {
      const float* Whh = w->enc_w_hh[l][d];
      auto whh = [&](int n, int k) {
        const int jb = n / 64, g = (n / 16) % 4, u = jb * 16 + (n % 16);
        return Whh[(size_t)(g * H + u) * H + k];
      };
      pack_frag(out + L.enc_whh[l] + (size_t)d * 4 * H * H, 4 * H / 16, H / 64, whh);
      pack_frag16(out + L.enc_whh16[l] + (size_t)d * 4 * H * H, 4 * H / 16, H / 64, whh);
    }
    const float* wih = out + L.enc_wih[l];
    pack_rows16(out + L.enc_wih16[l], 8 * H, din, [&](int n, int k) { return wih[(size_t)n * din + k]; });
  }
  if (!w->embedding || !w->dec_w_ih || !w->dec_w_hh || !w->dec_b_ih || !w->dec_b_hh || !w->proj_w ||
      !w->proj_b || !w->attn_w_enc || !w->attn_b || !w->attn_w_hidden || !w->attn_v)
    return fail(nullptr, CASR_ERR_ARG, "decoder/attention: NULL tensor");
  std::memcpy(out + L.emb, w->embedding, sizeof(float) * (size_t)V * E);
  {
    uint16_t* e16 = reinterpret_cast<uint16_t*>(out + L.emb16);
    for (size_t i = 0; i < (size_t)V * E; ++i) split16_host(w->embedding[i], e16[2 * i], e16[2 * i + 1]);
  }
  // decoder LSTM: K order [emb | ctx | h] = [W_ih | W_hh]
  auto decw = [&](int n, int k) {
    const int jb = n / 64, g = (n / 16) % 4, u = jb * 16 + (n % 16);
    const int orow = g * HD + u;
    return k < E + C ? w->dec_w_ih[(size_t)orow * (E + C) + k] : w->dec_w_hh[(size_t)orow * HD + (k - E - C)];
  };
  pack_frag(out + L.dec_w, 4 * HD / 16, KDEC / 64, decw);
  pack_frag16(out + L.dec_w16, 4 * HD / 16, KDEC / 64, decw);
  for (int g = 0; g < 4; ++g)
    for (int u = 0; u < HD; ++u)
      out[L.dec_b + packed_gate_row(g, u)] = w->dec_b_ih[g * HD + u] + w->dec_b_hh[g * HD + u];
  // projection: reference input is cat([h, ctx]) (decoder.py:131); packed K order [ctx | h]
  auto projw = [&](int n, int k) {
    if (n >= V) return 0.f;
    return k < C ? w->proj_w[(size_t)n * KPROJ + HD + k] : w->proj_w[(size_t)n * KPROJ + (k - C)];
  };
  pack_frag(out + L.proj_w, L.VP / 16, KPROJ / 64, projw);
  pack_frag16(out + L.proj_w16, L.VP / 16, KPROJ / 64, projw);
  for (int n = 0; n < V; ++n) out[L.proj_b + n] = w->proj_b[n];
  for (int a = 0; a < A; ++a)
    for (int c = 0; c < C; ++c) out[L.wencT + (size_t)a * C + c] = w->attn_w_enc[(size_t)c * A + a];
  pack_rows16(out + L.wenc16, A, C, [&](int n, int k) { return out[L.wencT + (size_t)n * C + k]; });
  std::memcpy(out + L.b_attn, w->attn_b, sizeof(float) * A);
  std::memcpy(out + L.w_hidden, w->attn_w_hidden, sizeof(float) * HD * A);
  std::memcpy(out + L.v, w->attn_v, sizeof(float) * A);
  return CASR_OK;
}

int casr_create(const casr_config* cfg, int device, casr_handle** out) {
  if (!out) return fail(nullptr, CASR_ERR_ARG, "out is NULL");
  *out = nullptr;
  int rc = check_config(cfg);
  if (rc) return rc;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return fail(nullptr, CASR_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n) return fail(nullptr, CASR_ERR_ARG, "device %d out of range", device);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(nullptr, CASR_ERR_UNSUPPORTED, "device %d is %s; this library is built for gfx950",
                device, prop.gcnArchName);
  auto* h = new casr_handle();
  h->cfg = *cfg;
  h->L = make_layout(*cfg);
  h->device = device;
  *out = h;
  return CASR_OK;
}

int casr_bind_weights(casr_handle* h, const float* packed_device) {
  if (!h || !packed_device) return fail(h, CASR_ERR_ARG, "handle/weights NULL");
  HIP_OK(h, hipSetDevice(h->device));
  float info[6] = {};
  HIP_OK(h, hipMemcpy(info, packed_device + h->L.info, sizeof info, hipMemcpyDeviceToHost));
  uint32_t stamp[3];
  std::memcpy(stamp, info + 1, sizeof stamp);
  if (stamp[0] != LAYOUT_MAGIC || stamp[1] != (uint32_t)(h->L.total & 0xFFFFFFFFu) ||
      stamp[2] != (uint32_t)(h->L.total >> 32))
    return fail(h, CASR_ERR_ARG,
                "casr_bind_weights: the blob was not packed by this build's layout (stamp %08x, %u floats; "
                "expected %08x, %zu floats)", stamp[0], stamp[1], LAYOUT_MAGIC, h->L.total);
  h->s16_valid = info[0] == 1.f;
  h->proj_small = info[4] == 1.f;
  h->dec_small = info[5] == 1.f;
  h->W = packed_device;
  h->graphs.clear();  // captured graphs bake in the precision and weight pointers
  // the folded step's tables (decoder.hip build_fold): derived from this blob, so rebuilt at every
  // bind; the gate table always, the s16 fused image and the s16 query image only from a blob with
  // valid s16 images.  The f32 fused image (29 MB, read only by the greedy fold under the exact-f32
  // arithmetic) is built by the first such decode (ensure_fold32)
  h->fold_ready = h->fold32_ready = false;
  {
    const int V = h->cfg.vocab;
    HIP_OK(h, h->egates.ensure((size_t)V * 4 * HD * sizeof(float)));
    if (h->s16_valid) {
      HIP_OK(h, h->wfold.ensure(fold_image_bytes(V)));
      HIP_OK(h, h->wq16.ensure(FOLD_WQ16_FLOATS * sizeof(float)));
    }
    HIP_OK(h, build_fold(h->W, h->L, V, h->s16_valid ? h->wfold.as<float>() : nullptr, h->egates.as<float>(),
                         h->s16_valid ? h->wq16.as<float>() : nullptr, nullptr, nullptr));
    HIP_OK(h, hipStreamSynchronize(nullptr));
    h->fold_ready = h->s16_valid;
  }
  if (h->s16_valid) {  // 16-k-block-major copies of the input-projection weight images
    size_t tot = 0;
    for (int l = 0; l < h->cfg.enc_layers; ++l) {
      h->wih16km_off[l] = tot;
      tot += (size_t)8 * H * s16_kpad(l == 0 ? D : C);
    }
    HIP_OK(h, h->wih16km.ensure(tot * sizeof(float)));
    for (int l = 0; l < h->cfg.enc_layers; ++l)
      HIP_OK(h, launch_relayout_km16(h->W + h->L.enc_wih16[l], 8 * H, s16_kpad(l == 0 ? D : C),
                                     h->wih16km.as<float>() + h->wih16km_off[l], nullptr));
    HIP_OK(h, hipStreamSynchronize(nullptr));
  }
  return CASR_OK;
}

// the f32 fused image of the folded greedy step under the exact-f32 arithmetic, built once per bind
// by the first decode that needs it (on the null stream, synchronised: a decode's captured graph
// never contains the build)
static int ensure_fold32(casr_handle* h) {
  if (h->fold32_ready) return CASR_OK;
  const int V = h->cfg.vocab;
  HIP_OK(h, h->wfold32.ensure(fold_image_bytes(V)));
  HIP_OK(h, build_fold(h->W, h->L, V, nullptr, nullptr, nullptr, h->wfold32.as<float>(), nullptr));
  HIP_OK(h, hipStreamSynchronize(nullptr));
  h->fold32_ready = true;
  return CASR_OK;
}

int casr_set_precision(casr_handle* h, int precision) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  if (precision != CASR_PREC_F32 && precision != CASR_PREC_S16X3 && precision != CASR_PREC_S16X1)
    return fail(h, CASR_ERR_ARG, "unknown precision %d", precision);
  if (precision != CASR_PREC_F32 && precision != CASR_PREC_S16)
    return fail(h, CASR_ERR_UNSUPPORTED, "this build computes %s; %s is the %s build", CASR_S16_ONE ? "s16x1" : "s16x3",
                CASR_S16_ONE ? "s16x3" : "s16x1", CASR_S16_ONE ? "libcasr_hip.so" : "libcasr_hip_s16x1.so");
  h->precision = precision;
  return CASR_OK;
}

int casr_get_precision(const casr_handle* h) {
  if (!h) return -1;
  return h->s16() ? CASR_PREC_S16 : CASR_PREC_F32;
}

void casr_destroy(casr_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  // work enqueued on any stream may still read the handle's buffers (a persistent recurrence
  // layer, a decode loop on the caller's stream, a graph replay on the private streams): drain
  // the device before graphs, streams and buffers go away
  (void)hipDeviceSynchronize();
  h->graphs.clear();
  if (h->cap) (void)hipStreamDestroy(h->cap);
  for (int i = 0; i < 2; ++i) {
    if (h->xs[i]) (void)hipStreamDestroy(h->xs[i]);
    if (h->ev_out[i]) (void)hipEventDestroy(h->ev_out[i]);
  }
  if (h->ev_in) (void)hipEventDestroy(h->ev_in);
  for (DevBuf* b : {&h->gin, &h->out0, &h->out1, &h->hbuf, &h->cst, &h->hfin, &h->keysT, &h->lens, &h->feat, &h->fstat, &h->hx, &h->x16, &h->gflags, &h->fe_const,
                    &h->st, &h->logits, &h->small, &h->bp, &h->tk, &h->rec, &h->beam_small, &h->gout, &h->wfold, &h->wfold32, &h->coldbuf,
                    &h->egates, &h->fgates, &h->wq16, &h->wih16km, &h->ksbuf, &h->asbuf})
    b->release();
  delete h;
}

int casr_set_graphs(casr_handle* h, int enable) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  if (enable < 0 || enable > 3) return fail(h, CASR_ERR_ARG, "casr_set_graphs: mode %d not in [0, 3]", enable);
  h->graph_mode = enable;
  return CASR_OK;
}

int casr_set_persistent(casr_handle* h, int enable) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  h->use_persistent = enable != 0;
  return CASR_OK;
}

int casr_recurrence_mode(const casr_handle* h, int B) {
  if (!h || B <= 0) return -1;
  if (!h->use_persistent) return 0;
  // the persistent recurrence needs every workgroup of its grid resident at once; the occupancy
  // query runs on the handle's device, and the caller's current device is restored
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return 0;
  if (cur != h->device && hipSetDevice(h->device) != hipSuccess) return 0;
  const int fits = rec_layer_fits(B, rec_layout(B, h->tune)) ? 1 : 0;
  if (cur != h->device) (void)hipSetDevice(cur);
  return fits;
}

int casr_set_option(casr_handle* h, int option, int value) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  if (option < 0 || option >= CASR_OPT_COUNT) return fail(h, CASR_ERR_ARG, "unknown option %d", option);
  static const int lo[CASR_OPT_COUNT] = {0, 0, 0, -1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  static const int hi[CASR_OPT_COUNT] = {1, 3, 1, 16, 8, 2, 2, 2, 8, 1, 1, CASR_MAX_LAYERS, (1 << CASR_K_COUNT) - 1, 1, 1, 1, 1, 1, AT_SPLIT_MAX};
  if (option == CASR_OPT_ATTN_KPB && value != 0 && value != 4 && value != 8)
    return fail(h, CASR_ERR_ARG, "CASR_OPT_ATTN_KPB: 0 (auto), 4 or 8");
  if (value < lo[option] || value > hi[option])
    return fail(h, CASR_ERR_ARG, "option %d: value %d not in [%d, %d]", option, value, lo[option], hi[option]);
  if (option == CASR_OPT_DIAG_COLD) {
    if (value) {
      HIP_OK(h, hipSetDevice(h->device));
      HIP_OK(h, h->coldbuf.ensure((size_t)1 << 30));
      HIP_OK(h, hipMemset(h->coldbuf.p, 0, (size_t)1 << 30));
    }
    h->prof.cold_buf = h->coldbuf.p;
    h->prof.cold_bytes = (size_t)1 << 30;
    h->prof.cold_mask = (uint32_t)value;
  }
  h->tune.v[option] = value;
  return CASR_OK;
}

int casr_get_option(const casr_handle* h, int option, int32_t* value) {
  if (!h || !value || option < 0 || option >= CASR_OPT_COUNT)
    return fail(nullptr, CASR_ERR_ARG, "casr_get_option: bad arguments");
  *value = h->tune[option];
  return CASR_OK;
}

const char* casr_last_error(const casr_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

int casr_features(casr_handle* h, const float* fbank, const int32_t* frames, int B, int T, float eps,
                  float* feat, int32_t* feat_len, void* stream) {
  if (!h || !fbank || !frames || !feat || !feat_len || B <= 0 || T < 3)
    return fail(h, CASR_ERR_ARG, "casr_features: bad arguments (B=%d T=%d)", B, T);
  HIP_OK(h, hipSetDevice(h->device));
  ProfScope ps(&h->prof, CASR_K_FEATURES, (hipStream_t)stream);
  HIP_OK(h, h->fstat.ensure((size_t)B * 2 * D * sizeof(float)));
  HIP_OK(h, launch_features(fbank, frames, B, T, eps, feat, feat_len, h->fstat.as<float>(), (hipStream_t)stream));
  return CASR_OK;
}

int casr_log_mel_frames(int n_samples) { return frontend_frames(n_samples); }

int casr_mel_filterbank(int n_stft, float f_min, float f_max, int n_mels, float* fb_host) {
  if (n_stft < 2 || n_mels < 1 || !fb_host || !(f_max > f_min))
    return fail(nullptr, CASR_ERR_ARG, "casr_mel_filterbank: bad arguments");
  mel_filterbank(n_stft, f_min, f_max, n_mels, fb_host);
  return CASR_OK;
}

int casr_log_mel(casr_handle* h, const float* wav, const int32_t* n_samples, int B, int n_max, int t_max,
                 float preemphasis, float* fbank, int32_t* frames, void* stream) {
  if (!h || !wav || !n_samples || !fbank || !frames || B <= 0 || n_max <= 0 || t_max <= 0)
    return fail(h, CASR_ERR_ARG, "casr_log_mel: bad arguments");
  if (t_max < frontend_frames(n_max))
    return fail(h, CASR_ERR_ARG, "casr_log_mel: t_max %d < %d frames of n_max %d samples", t_max,
                frontend_frames(n_max), n_max);
  if ((size_t)n_max * B > (size_t)1 << 40) return fail(h, CASR_ERR_ARG, "casr_log_mel: batch too large");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  if (!h->fe_const.p) {
    FrontendConst c;
    build_frontend_const(&c);
    HIP_OK(h, h->fe_const.ensure(sizeof(FrontendConst)));
    HIP_OK(h, hipMemcpy(h->fe_const.p, &c, sizeof c, hipMemcpyHostToDevice));
  }
  if (!guard_words(h)) return fail(h, CASR_ERR_HIP, "casr_log_mel: guard words not allocated");
  ProfScope ps(&h->prof, CASR_K_FEATURES, s);
  HIP_OK(h, launch_log_mel(wav, n_samples, B, n_max, t_max, preemphasis, h->fe_const.as<FrontendConst>(), fbank,
                           frames, GUARD(h, 2), s, h->tune[CASR_OPT_LOGMEL_Q16]));
  return CASR_OK;
}

int casr_gather_utterances(casr_handle* h, const float* const* utt_ptrs, const int32_t* lens, int B,
                           int Tp, float* feat, void* stream) {
  if (!h || !utt_ptrs || !lens || !feat || B <= 0 || Tp <= 0)
    return fail(h, CASR_ERR_ARG, "casr_gather_utterances: bad arguments");
  HIP_OK(h, hipSetDevice(h->device));
  HIP_OK(h, launch_gather_utts(utt_ptrs, lens, B, Tp, feat, (hipStream_t)stream));
  return CASR_OK;
}

// The encoder.  fb != nullptr (casr_encode_fbank): the inputs are fbank [B][T][n_mels] + frames
// and the features are computed here (s16x3: straight into the layer-0 row image); otherwise
// feat [B][Tp][feat_dim] + lens.
static int encode_impl(casr_handle* h, const float* feat, const int32_t* lens, int B, int Tp, hipStream_t s,
                       const float* fb = nullptr, const int32_t* frames = nullptr, int T = 0, float eps = 0.f) {
  const size_t rows = (size_t)B * Tp;
  HIP_OK(h, h->gin.ensure(rows * 8 * H * sizeof(float)));
  HIP_OK(h, h->out0.ensure(rows * C * sizeof(float)));
  HIP_OK(h, h->out1.ensure(rows * C * sizeof(float)));
  HIP_OK(h, h->hbuf.ensure((size_t)2 * 2 * B * H * sizeof(float)));
  HIP_OK(h, h->cst.ensure((size_t)2 * B * H * sizeof(float)));
  HIP_OK(h, h->hfin.ensure((size_t)2 * B * H * sizeof(float)));
  const int Tq = (Tp + 3) & ~3;  // keysT row stride (16 B aligned rows for the attention)
  HIP_OK(h, h->keysT.ensure(2 * (size_t)B * A * Tq * sizeof(float)));  // [keys | exp(2 keys)] (KeysEpi)
  HIP_OK(h, h->lens.ensure((size_t)B * sizeof(int32_t)));
  if (!fb) HIP_OK(h, hipMemcpyAsync(h->lens.p, lens, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s));
  const int layout = rec_layout(B, h->tune);
  bool persistent = casr_recurrence_mode(h, B) == 1;
  if (!persistent) {  // the persistent recurrence writes the padded frames itself
    HIP_OK(h, hipMemsetAsync(h->out0.p, 0, rows * C * sizeof(float), s));
    HIP_OK(h, hipMemsetAsync(h->out1.p, 0, rows * C * sizeof(float), s));
  }
  if (!guard_words(h)) return fail(h, CASR_ERR_HIP, "casr_encode: guard words not allocated");
  int32_t* eflag = GUARD(h, 1);
  {  // final h
    FillList fl;
    fl.add32(h->hfin.p, 0u, (size_t)2 * B * H);
    HIP_OK(h, fill_multi(fl, s));
  }
  const bool s16 = h->s16();
  // the layer-input images 16-k-block major (CASR_OPT_X16_KM and the GEMM / keys forms that read them)
  const int km = s16 && x16_km(h->tune) ? 1 : 0;
  if (s16) HIP_OK(h, h->x16.ensure(rows * s16_kpad(D) * sizeof(float)));
  if (persistent) HIP_OK(h, h->hx.ensure(rec_layer_granule_bytes(B, layout)));
  const int32_t* dl = h->lens.as<int32_t>();
  float* outs[2] = {h->out0.as<float>(), h->out1.as<float>()};
  bool x16_ready = false;
  if (fb) {
    ProfScope ps(&h->prof, CASR_K_FEATURES, s);
    HIP_OK(h, h->fstat.ensure((size_t)B * 2 * D * sizeof(float)));
    if (s16 && features_x16_supported(T)) {
      HIP_OK(h, launch_features_x16(fb, frames, B, T, eps, h->lens.as<int32_t>(), h->fstat.as<float>(),
                                    h->x16.as<uint16_t>(), s16_kpad(D),
                                    eflag, s, km));
      x16_ready = true;  // feat stays NULL: layer 0 reads only the image (no residual input)
    } else {
      HIP_OK(h, h->feat.ensure(rows * D * sizeof(float)));
      HIP_OK(h, launch_features(fb, frames, B, T, eps, h->feat.as<float>(), h->lens.as<int32_t>(), h->fstat.as<float>(), s));
      feat = h->feat.as<float>();
    }
  }
  const float* x = feat;
  float* hb = h->hbuf.as<float>();
  // s16: a persistent layer writes the next layer's input row image itself (no split pass)
  bool fell_back = false;  // a cooperative persistent launch was refused: per-step from here on
  for (int l = 0; l < h->cfg.enc_layers; ++l) {
    const int din = l == 0 ? D : C;
    float* out = outs[l & 1];
    {
    ProfScope ps(&h->prof, CASR_K_INPUT_PROJ, s);
    if (s16) {
      const int kp = s16_kpad(din);
      if (!x16_ready)
        HIP_OK(h, launch_split_rows(x, din, (int)rows, din, kp, h->x16.as<uint16_t>(), eflag, s, km));
      HIP_OK(h, launch_input_proj_s16_big(h->x16.as<float>(), (int)rows, kp,
                                          km ? h->wih16km.as<float>() + h->wih16km_off[l] : h->W + h->L.enc_wih16[l],
                                          h->W + h->L.enc_bias[l], h->gin.as<float>(), s, din,
                                          h->tune[CASR_OPT_GEMM16_PERSIST], h->tune[CASR_OPT_GEMM16_TAIL], km,
                                          h->tune[CASR_OPT_GEMM16_LEAN]));
    } else {
      HIP_OK(h, launch_input_proj(x, (int)rows, din, h->W + h->L.enc_wih[l], h->W + h->L.enc_bias[l],
                                  h->gin.as<float>(), s));
    }
    }
    const int residual = (h->cfg.residual && l > 0) ? 1 : 0;
    // layer 0 has no residual input: pass an internal pointer so a graph never bakes in the
    // caller's feature buffer
    const float* xin = residual ? x : out;
    const float* whh = h->W + (s16 ? h->L.enc_whh16[l] : h->L.enc_whh[l]);
    if (persistent) {
      // one launch runs all Tp steps; h and c start at zero inside (util.py:1236-1247)
      HIP_OK(h, reset_rec_layer(reinterpret_cast<uint32_t*>(h->hx.p), B, layout, s));
      // diagnostics only: CASR_REC_TRACE=<file> dumps per-wave phase timestamps of layer 0
      const char* trace_path = l == 0 ? std::getenv("CASR_REC_TRACE") : nullptr;
      DevBuf tbuf;
      const size_t tbytes = (size_t)rec_layer_grid_blocks(B, layout) * rec_layer_waves(layout) * Tp * 5 * sizeof(uint32_t);
      if (trace_path) {
        HIP_OK(h, tbuf.ensure(tbytes));
        HIP_OK(h, hipMemsetAsync(tbuf.p, 0, tbytes, s));
      }
      hipError_t er;
      if (h->tune[CASR_OPT_REC_COOP_REFUSE] == l + 1) {
        er = hipErrorCooperativeLaunchTooLarge;  // tests only: this layer's launch "refused"
      } else {
        ProfScope ps(&h->prof, CASR_K_REC_STEP, s);
        // the last layer's image feeds the keys GEMM
        uint16_t* x16o = s16 ? h->x16.as<uint16_t>() : nullptr;
        er = launch_rec_layer(whh, h->gin.as<float>(), xin, out, x16o, reinterpret_cast<uint32_t*>(h->hx.p),
                              h->hfin.as<float>(), h->cst.as<float>(), dl, B, Tp, residual, s16,
                              eflag, tbuf.as<uint32_t>(), layout, h->tune, s, km);
      }
      if (er == hipErrorCooperativeLaunchTooLarge) {
        // the device cannot hold the whole grid at once (e.g. CUs taken by other work): this layer
        // and the next ones run the per-step recurrence (same bits) instead of spinning
        (void)hipGetLastError();
        persistent = false;
        fell_back = true;
      } else {
        HIP_OK(h, er);
      }
      if (persistent && trace_path) {
        std::vector<uint32_t> hostv(tbytes / 4);
        HIP_OK(h, hipMemcpyAsync(hostv.data(), tbuf.p, tbytes, hipMemcpyDeviceToHost, s));
        HIP_OK(h, hipStreamSynchronize(s));
        tbuf.release();
        if (FILE* f = std::fopen(trace_path, "wb")) {
          const int32_t hdr[5] = {rec_layer_grid_blocks(B, layout), rec_layer_waves(layout), Tp, 5,
                                  rec_layer_producers(layout)};
          std::fwrite(hdr, sizeof hdr, 1, f);
          std::fwrite(hostv.data(), 4, hostv.size(), f);
          std::fclose(f);
        }
      }
      if (persistent) {
        x = out;
        x16_ready = s16;
        continue;
      }
    }
    x16_ready = false;
    // the persistent layers write their padded frames themselves; the per-step ones need zeros
    if (fell_back) HIP_OK(h, hipMemsetAsync(out, 0, rows * C * sizeof(float), s));
    // h (both ping-pong buffers) and c start at zero (RNN_RES state None, util.py:1236-1247)
    HIP_OK(h, fill_u32(hb, 0, (size_t)2 * 2 * B * H, s));
    HIP_OK(h, fill_u32(h->cst.p, 0, (size_t)2 * B * H, s));
    auto rec_loop = [&](hipStream_t st, Profiler* prof, int r0, int r1) -> hipError_t {
      hipError_t e = hipSuccess;
      for (int step = 0; step < Tp && e == hipSuccess; ++step) {
        const float* hprev = hb + (size_t)(step & 1) * 2 * B * H;
        float* hnext = hb + (size_t)((step + 1) & 1) * 2 * B * H;
        ProfScope ps(prof, CASR_K_REC_STEP, st);
        e = launch_rec_step(whh, h->gin.as<float>(), xin, out, hprev, hnext,
                            h->cst.as<float>(), h->hfin.as<float>(), dl, B, Tp, step, residual, r0, r1, s16, st);
      }
      return e;
    };
    if (h->graph_mode & CASR_GRAPHS_RECURRENCE) {
      // rows are independent: two row halves replay as two graphs on two streams, so one
      // half's load latency hides behind the other's MFMAs
      const int nsplit = B >= 64 ? 2 : 1;
      const int half = ((B / 2) + 15) / 16 * 16;
      hipGraphExec_t ex[2] = {};
      for (int p = 0; p < nsplit; ++p) {
        const int r0 = (nsplit == 1 || p == 0) ? 0 : half;
        const int r1 = (nsplit == 1 || p == 1) ? B : half;
        const std::vector<uint64_t> key = {1, (uint64_t)s16, (uint64_t)l, (uint64_t)B, (uint64_t)Tp, (uint64_t)residual,
                                           (uint64_t)r0, (uint64_t)r1, (uint64_t)h->W, (uint64_t)h->gin.p,
                                           (uint64_t)xin, (uint64_t)out, (uint64_t)hb, (uint64_t)h->cst.p,
                                           (uint64_t)h->hfin.p, (uint64_t)dl};
        HIP_OK(h, get_graph(h, key, [&](hipStream_t cs) { return rec_loop(cs, nullptr, r0, r1); }, &ex[p]));
      }
      ProfScope ps(&h->prof, CASR_K_REC_STEP, s, Tp);  // one pair per replay of Tp steps
      HIP_OK(h, launch_graphs(h, ex, nsplit, s));
    } else {
      HIP_OK(h, rec_loop(s, &h->prof, 0, B));
    }
    x = out;
  }
  h->enc_out = const_cast<float*>(x);
  {
  ProfScope ps(&h->prof, CASR_K_KEYS, s);
  // s16x3 keys on every s16 path (the per-step fallback splits the encoder output first), so both
  // recurrences give the same keys bits
  if (s16 && !x16_ready) {
    HIP_OK(h, launch_split_rows(h->enc_out, C, (int)rows, C, C, h->x16.as<uint16_t>(), eflag, s, km));
    x16_ready = true;
  }
  if (x16_ready)  // s16x3 keys from the image the last persistent layer wrote
    HIP_OK(h, launch_keys_s16(h->x16.as<float>(), B, Tp, h->W + h->L.wenc16, h->W + h->L.b_attn,
                              h->keysT.as<float>(), s, h->tune[CASR_OPT_KEYS_ROWS], km));
  else
    HIP_OK(h, launch_keys(h->enc_out, B, Tp, h->W + h->L.wencT, h->W + h->L.b_attn, h->keysT.as<float>(), s));
  }
  h->B = B;
  h->Tp = Tp;
  h->encoded = true;
  h->beam_done = false;
  return CASR_OK;
}

int casr_encode(casr_handle* h, const float* feat, const int32_t* lens, int B, int Tp, void* stream) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  if (!h->W) return fail(h, CASR_ERR_STATE, "casr_encode: no weights bound");
  if (!feat || !lens || B <= 0 || Tp <= 0) return fail(h, CASR_ERR_ARG, "casr_encode: bad arguments");
  HIP_OK(h, hipSetDevice(h->device));
  return encode_impl(h, feat, lens, B, Tp, (hipStream_t)stream);
}

int casr_encode_fbank(casr_handle* h, const float* fbank, const int32_t* frames, int B, int T, float eps,
                      int32_t* feat_len, void* stream) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  if (!h->W) return fail(h, CASR_ERR_STATE, "casr_encode_fbank: no weights bound");
  if (!fbank || !frames || B <= 0 || T < 3)
    return fail(h, CASR_ERR_ARG, "casr_encode_fbank: bad arguments (B=%d T=%d)", B, T);
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  const int rc = encode_impl(h, nullptr, nullptr, B, T / 3, s, fbank, frames, T, eps);
  if (rc == CASR_OK && feat_len)
    HIP_OK(h, hipMemcpyAsync(feat_len, h->lens.p, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s));
  return rc;
}

int casr_encoder_results(casr_handle* h, float* enc, float* h_final, float* c_final, float* keys,
                         void* stream) {
  if (!h || !h->encoded) return fail(h, CASR_ERR_STATE, "casr_encoder_results: nothing encoded");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  const int B = h->B, Tp = h->Tp;
  if (enc)
    HIP_OK(h, hipMemcpyAsync(enc, h->enc_out, (size_t)B * Tp * C * sizeof(float), hipMemcpyDeviceToDevice, s));
  // [2][B][H] -> [B][fw | bw]
  if (h_final)
    HIP_OK(h, hipMemcpy2DAsync(h_final, C * sizeof(float), h->hfin.p, H * sizeof(float), H * sizeof(float), B,
                               hipMemcpyDeviceToDevice, s));
  if (h_final)
    HIP_OK(h, hipMemcpy2DAsync(h_final + H, C * sizeof(float), h->hfin.as<float>() + (size_t)B * H,
                               H * sizeof(float), H * sizeof(float), B, hipMemcpyDeviceToDevice, s));
  if (c_final)
    HIP_OK(h, hipMemcpy2DAsync(c_final, C * sizeof(float), h->cst.p, H * sizeof(float), H * sizeof(float), B,
                               hipMemcpyDeviceToDevice, s));
  if (c_final)
    HIP_OK(h, hipMemcpy2DAsync(c_final + H, C * sizeof(float), h->cst.as<float>() + (size_t)B * H,
                               H * sizeof(float), H * sizeof(float), B, hipMemcpyDeviceToDevice, s));
  if (keys)
    HIP_OK(h, hipMemcpy2DAsync(keys, Tp * sizeof(float), h->keysT.p, ((Tp + 3) & ~3) * sizeof(float),
                               Tp * sizeof(float), (size_t)B * A, hipMemcpyDeviceToDevice, s));
  return CASR_OK;
}

// the decode loop replays as a graph unless a decode kernel class is being timed per launch
static bool decode_graph_ok(const casr_handle* h) {
  const uint32_t dec = (1u << CASR_K_DEC_LSTM) | (1u << CASR_K_ATTENTION) | (1u << CASR_K_PROJ) |
                       (1u << CASR_K_SELECT);
  return (h->graph_mode & CASR_GRAPHS_DECODE) && !(h->prof.mask & dec);
}

static int prepare_decode(casr_handle* h, int k, DecodeArgs& a, bool greedy) {
  if (!h->encoded) return fail(h, CASR_ERR_STATE, "decode before casr_encode");
  if (k < 1 || k > KMAX_BEAM) return fail(h, CASR_ERR_ARG, "beam width %d not in [1, %d]", k, KMAX_BEAM);
  const int B = h->B, Tp = h->Tp, L = h->cfg.max_len, V = h->cfg.vocab;
  const int R = B * k;
  const size_t smem = attention_smem_bytes(B, k, Tp, h->tune[CASR_OPT_ATTN_KPB]);
  if (smem > 160 * 1024)
    return fail(h, CASR_ERR_UNSUPPORTED, "attention needs %zu B of LDS (k=%d, Tp=%d) > 160 KiB", smem, k, Tp);
  HIP_OK(h, h->st.ensure(((size_t)2 * R * ST + (size_t)dec_q_slots(R) * R * A) * sizeof(float)));
  HIP_OK(h, h->logits.ensure(((size_t)R * V + (size_t)3 * R * GP_NB + (size_t)R * GP_NT) * sizeof(float)));
  HIP_OK(h, h->small.ensure((size_t)(6 * R + L + B + R + 1) * sizeof(int32_t) + 256));
  HIP_OK(h, h->bp.ensure((size_t)L * R * sizeof(int32_t)));
  HIP_OK(h, h->tk.ensure((size_t)L * R * sizeof(int32_t)));
  HIP_OK(h, h->rec.ensure((size_t)B * L * k * (sizeof(float) + sizeof(int32_t) + 1) + 256));
  DecodeBufs& d = h->d;
  d.st[0] = h->st.as<float>();
  d.st[1] = d.st[0] + (size_t)R * ST;
  d.qpart = d.st[1] + (size_t)R * ST;
  d.logits = h->logits.as<float>();
  d.part.mx = d.logits + (size_t)R * V;
  d.part.se = d.part.mx + (size_t)R * GP_NB;
  d.part.ix = reinterpret_cast<int32_t*>(d.part.se + (size_t)R * GP_NB);
  d.part.tmx = reinterpret_cast<float*>(d.part.ix + (size_t)R * GP_NB);
  int32_t* sp = h->small.as<int32_t>();
  d.tok[0] = sp;
  d.tok[1] = sp + R;
  d.src[0] = sp + 2 * R;
  d.src[1] = sp + 3 * R;
  d.score[0] = reinterpret_cast<float*>(sp + 4 * R);
  d.score[1] = reinterpret_cast<float*>(sp + 5 * R);
  d.newdone = sp + 6 * R;
  d.topfin = reinterpret_cast<uint8_t*>(sp + 6 * R + L);
  d.fin = reinterpret_cast<uint8_t*>(sp + 6 * R + L + B);
  if (!guard_words(h)) return fail(h, CASR_ERR_HIP, "decode: guard words not allocated");
  d.err = GUARD(h, 0);
  d.bp = h->bp.as<int32_t>();
  d.tk = h->tk.as<int32_t>();
  d.rec_score = h->rec.as<float>();
  d.rec_src = reinterpret_cast<int32_t*>(d.rec_score + (size_t)B * L * k);
  d.rec_valid = reinterpret_cast<uint8_t*>(d.rec_src + (size_t)B * L * k);
  d.aspart = nullptr;
  d.ascnt = nullptr;
  d.asplit = 0;
  if (greedy && R <= 64 && h->tune[CASR_OPT_ATTN_SPLIT]) {
    const size_t part = (size_t)R * AT_SPLIT_MAX * (C + 4) * sizeof(float);
    HIP_OK(h, h->asbuf.ensure(part + (size_t)R * sizeof(int32_t)));
    d.aspart = h->asbuf.as<float>();
    d.ascnt = reinterpret_cast<int32_t*>(h->asbuf.as<char>() + part);
    const int o = h->tune[CASR_OPT_ATTN_SPLIT];
    d.asplit = o == 1 ? (R <= 32 ? 8 : 4) : o;  // 1: by R; 2..AT_SPLIT_MAX: that many
  }
  d.kspart = nullptr;
  d.kscnt = nullptr;
  if (greedy && R <= 32 && h->tune[CASR_OPT_DEC_KSPLIT]) {
    HIP_OK(h, h->ksbuf.ensure(DG_KS_PART_BYTES + DG_KS_COUNTERS * sizeof(int32_t)));
    d.kspart = h->ksbuf.as<float>();
    d.kscnt = reinterpret_cast<int32_t*>(h->ksbuf.as<char>() + DG_KS_PART_BYTES);
  }
  a.W = h->W;
  a.L = h->L;
  a.enc = h->enc_out;
  a.keysT = h->keysT.as<float>();
  a.hfin = h->hfin.as<float>();
  a.cfin = h->cst.as<float>();
  a.lens = h->lens.as<int32_t>();
  a.B = B;
  a.Tp = Tp;
  a.k = k;
  a.V = V;
  a.max_len = L;
  a.sos = h->cfg.sos;
  a.eos = h->cfg.eos;
  a.temperature = h->cfg.temperature;
  a.s16 = h->s16() ? 1 : 0;
  a.prof = &h->prof;
  a.fuse_select = h->tune[CASR_OPT_FUSE_SELECT];
  a.attn_kpb = h->tune[CASR_OPT_ATTN_KPB];
  a.attn_direct = h->tune[CASR_OPT_ATTN_DIRECT];
  a.proj_small = h->proj_small;
  // the folded step: greedy (casr_greedy), or beam at R >= 1024 rows with 4 or 8 beam rows per
  // attention block and every projection / LSTM weight < 16 (the fused GEMM's one-accumulator
  // beam shapes, decoder.hip launch_fold_gemm).  casr_beam at k = 1 is a beam caller: it takes
  // the beam guards, never the greedy clause (its fused GEMM would pick the one-accumulator shapes)
  const bool fold_beam = !greedy && R >= 1024 && h->proj_small && h->dec_small &&
                         attention_kpb(B, k, h->tune[CASR_OPT_ATTN_KPB]) >= 4;
  // (a vocabulary beyond the 64 seven-tile partial blocks of the fused GEMM keeps the three-launch step)
  const bool fold_vocab = (fold_vtiles(V) + FOLD_NT - 1) / FOLD_NT <= GP_NB;
  // the folded greedy attention (attention_kernel<1, 1>) holds its cell-phase area on top of the
  // three-launch step's LDS: at Tp where only the latter fits, greedy keeps the three-launch step
  const bool fold_lds = !greedy || attention_smem_bytes(B, k, Tp, h->tune[CASR_OPT_ATTN_KPB], 1) <= 160 * 1024;
  // the folded greedy attention reads the early-exit counters of steps 0..max_len-1 one per lane
  const bool fold_len = !greedy || L <= 64;
  // greedy folds in either arithmetic (round 4: the exact-f32 MFMAs on the f32 fused image); the
  // beam fold's one-accumulator shapes and its s16 query need the s16 images
  if (!a.s16 && greedy && h->W && h->tune[CASR_OPT_DEC_FOLD] && fold_vocab && fold_lds && fold_len) {
    const int rc = ensure_fold32(h);
    if (rc) return rc;
  }
  const bool fold_arith = a.s16 ? h->fold_ready : (greedy && h->fold32_ready);
  a.fold = (greedy || fold_beam) && fold_vocab && fold_lds && fold_len && fold_arith && h->tune[CASR_OPT_DEC_FOLD] ? 1 : 0;
  if (a.fold) {
    HIP_OK(h, h->fgates.ensure((size_t)R * 4 * HD * sizeof(float)));
    a.fb = FoldBufs{a.s16 ? h->wfold.as<float>() : h->wfold32.as<float>(), h->egates.as<float>(), h->wq16.as<float>(),
                    h->fgates.as<float>()};
  }
  return CASR_OK;
}

int casr_greedy(casr_handle* h, int32_t* tokens, int32_t* out_len, uint8_t* finished, float* accum,
                float* align, void* stream) {
  if (!h || !tokens || !out_len || !finished || !accum) return fail(h, CASR_ERR_ARG, "casr_greedy: NULL output");
  HIP_OK(h, hipSetDevice(h->device));
  DecodeArgs a{};
  int rc = prepare_decode(h, 1, a, true);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (!decode_graph_ok(h)) {
    dg_trace_init();  // CASR_DG_TRACE diagnostics only
    HIP_OK(h, run_greedy(a, h->d, tokens, out_len, finished, accum, align, s));
    dg_trace_dump();
    return CASR_OK;
  }
  // graph replay into handle-owned outputs, then copies to the caller's buffers
  const int B = h->B, L = h->cfg.max_len;
  const size_t nal = align ? (size_t)L * h->Tp * B : 0;
  HIP_OK(h, h->gout.ensure(sizeof(int32_t) * ((size_t)B * L + B) + sizeof(float) * (B + nal) + B + 64));
  int32_t* itok = h->gout.as<int32_t>();
  int32_t* ilen = itok + (size_t)B * L;
  float* iacc = reinterpret_cast<float*>(ilen + B);
  float* ial = align ? iacc + B : nullptr;
  uint8_t* ifin = reinterpret_cast<uint8_t*>(iacc + B + nal);
  a.prof = nullptr;
  const std::vector<uint64_t> key = {2, (uint64_t)a.s16, (uint64_t)(h->d.kspart != nullptr), (uint64_t)h->d.asplit, (uint64_t)h->asbuf.p, (uint64_t)a.fuse_select, (uint64_t)a.attn_kpb, (uint64_t)a.attn_direct, (uint64_t)a.fold, (uint64_t)h->fgates.p, (uint64_t)a.fb.wfold, (uint64_t)B, (uint64_t)h->Tp, (uint64_t)h->W, (uint64_t)h->gout.p,
                                     (uint64_t)(align != nullptr), (uint64_t)h->st.p, (uint64_t)h->logits.p,
                                     (uint64_t)h->small.p, (uint64_t)h->enc_out, (uint64_t)h->keysT.p,
                                     (uint64_t)h->hfin.p, (uint64_t)h->cst.p, (uint64_t)h->lens.p};
  dg_trace_init();  // CASR_DG_TRACE diagnostics only (outside any capture)
  HIP_OK(h, run_graph(h, key, s, [&](hipStream_t cs) { return run_greedy(a, h->d, itok, ilen, ifin, iacc, ial, cs); }));
  dg_trace_dump();  // CASR_DG_TRACE diagnostics only (no-op otherwise)
  CopyList cl;  // the graph's outputs to the caller's buffers in one launch
  cl.add(tokens, itok, sizeof(int32_t) * B * L);
  cl.add(out_len, ilen, sizeof(int32_t) * B);
  cl.add(finished, ifin, B);
  cl.add(accum, iacc, sizeof(float) * B);
  if (align) cl.add(align, ial, sizeof(float) * nal);
  HIP_OK(h, copy_multi(cl, s));
  return CASR_OK;
}

int casr_beam(casr_handle* h, int k, float lm_weight, float length_weight, int32_t* best_tokens,
              int32_t* best_len, float* best_score, int32_t* steps, void* stream) {
  if (!h || !best_tokens || !best_len || !best_score || !steps)
    return fail(h, CASR_ERR_ARG, "casr_beam: NULL output");
  HIP_OK(h, hipSetDevice(h->device));
  DecodeArgs a{};
  int rc = prepare_decode(h, k, a, false);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  h->dec_k = k;
  h->beam_done = true;
  if (!decode_graph_ok(h)) {
    dg_trace_init();  // CASR_DG_TRACE diagnostics only
    HIP_OK(h, run_beam(a, h->d, lm_weight, length_weight, best_tokens, best_len, best_score, steps, s));
    dg_trace_dump();
    return CASR_OK;
  }
  const int B = h->B, L = h->cfg.max_len;
  HIP_OK(h, h->gout.ensure(sizeof(int32_t) * ((size_t)B * L + B + 1) + sizeof(float) * B + 64));
  int32_t* itok = h->gout.as<int32_t>();
  int32_t* ilen = itok + (size_t)B * L;
  int32_t* istp = ilen + B;
  float* isc = reinterpret_cast<float*>(istp + 1);
  a.prof = nullptr;
  uint32_t lmw, lw;
  std::memcpy(&lmw, &lm_weight, 4);
  std::memcpy(&lw, &length_weight, 4);
  const std::vector<uint64_t> key = {3, (uint64_t)a.s16, (uint64_t)a.attn_kpb, (uint64_t)a.attn_direct, (uint64_t)a.fold, (uint64_t)h->fgates.p, (uint64_t)B, (uint64_t)h->Tp, (uint64_t)k, lmw, lw, (uint64_t)h->W,
                                     (uint64_t)h->gout.p, (uint64_t)h->st.p, (uint64_t)h->logits.p,
                                     (uint64_t)h->small.p, (uint64_t)h->bp.p, (uint64_t)h->tk.p, (uint64_t)h->rec.p,
                                     (uint64_t)h->enc_out, (uint64_t)h->keysT.p, (uint64_t)h->hfin.p,
                                     (uint64_t)h->cst.p, (uint64_t)h->lens.p};
  dg_trace_init();  // CASR_DG_TRACE diagnostics only (outside any capture)
  HIP_OK(h, run_graph(h, key, s, [&](hipStream_t cs) {
    return run_beam(a, h->d, lm_weight, length_weight, itok, ilen, isc, istp, cs);
  }));
  dg_trace_dump();
  CopyList cl;  // the graph's outputs to the caller's buffers in one launch
  cl.add(best_tokens, itok, sizeof(int32_t) * B * L);
  cl.add(best_len, ilen, sizeof(int32_t) * B);
  cl.add(best_score, isc, sizeof(float) * B);
  cl.add(steps, istp, sizeof(int32_t));
  HIP_OK(h, copy_multi(cl, s));
  return CASR_OK;
}

int casr_beam_records(casr_handle* h, int32_t* rec_tokens, float* rec_score, uint8_t* rec_valid,
                      void* stream) {
  if (!h || !h->beam_done) return fail(h, CASR_ERR_STATE, "casr_beam_records before casr_beam");
  if (!rec_tokens || !rec_score || !rec_valid) return fail(h, CASR_ERR_ARG, "casr_beam_records: NULL output");
  HIP_OK(h, hipSetDevice(h->device));
  DecodeArgs a{};
  int rc = prepare_decode(h, h->dec_k, a, false);
  if (rc) return rc;
  HIP_OK(h, run_beam_records(a, h->d, rec_tokens, rec_score, rec_valid, (hipStream_t)stream));
  return CASR_OK;
}

int casr_device_flags(casr_handle* h, int32_t* flags, void* stream) {
  if (!h || !flags) return fail(h, CASR_ERR_ARG, "casr_device_flags: bad arguments");
  *flags = 0;
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  int32_t w[3] = {0, 0, 0};
  if (h->gflags.p) {
    HIP_OK(h, hipMemcpyAsync(w, h->gflags.p, sizeof w, hipMemcpyDeviceToHost, s));
    HIP_OK(h, hipStreamSynchronize(s));
    if (w[0] | w[1] | w[2]) HIP_OK(h, hipMemsetAsync(h->gflags.p, 0, sizeof w, s));  // read and clear
  }
  *flags = w[0] | w[1] | w[2];
  return CASR_OK;
}

int casr_profile_enable(casr_handle* h, uint32_t class_mask) {
  if (!h) return fail(h, CASR_ERR_ARG, "handle NULL");
  h->prof.mask = class_mask;
  h->prof.reset();
  return CASR_OK;
}

int casr_profile_read(casr_handle* h, int cls, int32_t* launches, double* total_ms) {
  if (!h || cls < 0 || cls >= CASR_K_COUNT || !launches || !total_ms)
    return fail(h, CASR_ERR_ARG, "casr_profile_read: bad arguments");
  Profiler& p = h->prof;
  const size_t n = p.used[cls] / 2;
  double ms = 0.0;
  int32_t nl = 0;
  if (n) HIP_OK(h, hipEventSynchronize(p.ev[cls][2 * n - 1]));
  for (size_t i = 0; i < n; ++i) {
    float t = 0.f;
    HIP_OK(h, hipEventElapsedTime(&t, p.ev[cls][2 * i], p.ev[cls][2 * i + 1]));
    ms += t;
    nl += p.weight[cls][i];
  }
  *launches = nl;
  *total_ms = ms;
  return CASR_OK;
}

}  // extern "C"
