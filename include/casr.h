/*
 * casr.h — C ABI of the MI355X (gfx950) inference path for the shawnthu/chinese-asr
 * attention seq2seq model: fbank features -> 4-layer BiLSTM encoder -> Bahdanau
 * attention -> LSTM decoder -> greedy / beam-search decode loop.
 *
 * The reference has no FFI: its boundary is the Python method surface of `Model`
 * (model.py:18-987) and `main.py` (main.py:27-102).  Each entry point below names the
 * reference function it replaces; the Python host layer (chinese-asr_amd/model.py,
 * main.py, data.py) binds them with ctypes and keeps the reference signatures.
 *
 * Conventions
 *   - every function returns CASR_OK (0) or an error code; casr_last_error() explains;
 *   - all tensor arguments are DEVICE pointers owned by the caller, float32 / int32,
 *     C-contiguous, unless a comment says "host";
 *   - `stream` is a hipStream_t passed as void*; no call synchronises the host except
 *     where noted (the beam/greedy calls return after enqueueing);
 *   - one handle per device; a handle is not thread-safe; workspaces are owned by the
 *     handle and grow on demand (first call at a new size allocates).
 */
#ifndef CASR_H
#define CASR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CASR_API_VERSION 3
#define CASR_MAX_LAYERS 8

enum {
  CASR_OK = 0,
  CASR_ERR_ARG = 1,         /* bad argument / shape */
  CASR_ERR_HIP = 2,         /* HIP runtime error */
  CASR_ERR_STATE = 3,       /* call order (e.g. decode before encode, no weights) */
  CASR_ERR_UNSUPPORTED = 4  /* configuration this build does not implement */
};

typedef struct casr_handle casr_handle;

/* Frozen `gpd` values (gpd.py:13-125), bound at import time in the reference
 * (encoder.py:17-24, decoder.py:11-16, attention.py:21). */
typedef struct casr_config {
  int32_t n_mels;      /* 80   gpd['n_mels'] */
  int32_t feat_dim;    /* 720  encoder.py:19 (n_mels * 3 * 3) */
  int32_t enc_hidden;  /* 256  gpd['encoder_hidden_size'] */
  int32_t enc_layers;  /* 4    gpd['encoder_num_layers'] */
  int32_t residual;    /* 1    gpd['residual'] (util.py:1284) */
  int32_t dec_hidden;  /* 512  gpd['decoder_hidden_size'] (must be 2*enc_hidden) */
  int32_t embed_dim;   /* 256  gpd['embed_dim'] */
  int32_t attn_size;   /* 128  gpd['attn_size'] */
  int32_t vocab;       /* 5004 decoder.py:12 real_vcb_sz */
  int32_t max_len;     /* 40   gpd['max_len'] */
  int32_t sos;         /* 1 */
  int32_t eos;         /* 2 */
  float temperature;   /* gpd['temperature'], model.py:834 (beam only) */
} casr_config;

/* HOST pointers to the reference state-dict tensors, in their reference layouts
 * (Model.save, model.py:347-355).  [l][0] = forward, [l][1] = `_reverse`. */
typedef struct casr_weights_host {
  const float* enc_w_ih[CASR_MAX_LAYERS][2]; /* rnn.rnn.{l}.weight_ih_l0{,_reverse} [4H][Din] */
  const float* enc_w_hh[CASR_MAX_LAYERS][2]; /* rnn.rnn.{l}.weight_hh_l0{,_reverse} [4H][H]   */
  const float* enc_b_ih[CASR_MAX_LAYERS][2]; /* rnn.rnn.{l}.bias_ih_l0{,_reverse}   [4H]      */
  const float* enc_b_hh[CASR_MAX_LAYERS][2]; /* rnn.rnn.{l}.bias_hh_l0{,_reverse}   [4H]      */
  const float* embedding;      /* embedding.weight       [V][E]           decoder.py:30 */
  const float* dec_w_ih;       /* cell.cell.0.weight_ih  [4Hd][E+C]       util.py:1629  */
  const float* dec_w_hh;       /* cell.cell.0.weight_hh  [4Hd][Hd]                      */
  const float* dec_b_ih;       /* cell.cell.0.bias_ih    [4Hd]                          */
  const float* dec_b_hh;       /* cell.cell.0.bias_hh    [4Hd]                          */
  const float* proj_w;         /* proj_linear.weight     [V][Hd+C]        decoder.py:50 */
  const float* proj_b;         /* proj_linear.bias       [V]                            */
  const float* attn_w_enc;     /* attn_mechanism.W_enc   [C][A]           attention.py:28 */
  const float* attn_b;         /* attn_mechanism.b_attn  [A]                            */
  const float* attn_w_hidden;  /* attn_mechanism.W_hidden [Hd][A]                       */
  const float* attn_v;         /* attn_mechanism.v       [A]                            */
} casr_weights_host;

int casr_api_version(void);

/* Packed weight blob (kernel layouts: gate-interleaved LSTM rows, MFMA-fragment-major
 * decoder matrices, transposed attention key matrix).  Replaces Model.load's
 * load_state_dict (model.py:357-370): pack once on the host, upload / broadcast the
 * blob (RCCL over xGMI for multi-GPU), then bind it on each device. */
size_t casr_packed_weights_floats(const casr_config* cfg);
int casr_pack_weights(const casr_config* cfg, const casr_weights_host* w, float* packed_host);

int casr_create(const casr_config* cfg, int device, casr_handle** out);
/* Bind a device copy of the packed blob (not copied; must outlive its use).  The blob must hold
 * casr_packed_weights_floats(cfg) floats: the library checks the layout stamp casr_pack_weights
 * writes (magic + size) and refuses (CASR_ERR_ARG) a blob packed by another layout. */
int casr_bind_weights(casr_handle* h, const float* packed_device);
void casr_destroy(casr_handle* h);
const char* casr_last_error(const casr_handle* h); /* h may be NULL: last global error */

/* Feature post-processing of a batch of log-mel / fbank frames (data.py:226-249 +
 * main.py:37 CMVN): 9-tap delta / delta-delta (add_delta_deltas, data.py:129-164),
 * 3-frame stacking to feat_dim, per-utterance per-dimension (x-mean)/(std_unbiased+eps).
 *   fbank    [B][T][n_mels]    frames [B] (valid frames per utterance, <= T)
 *   feat     [B][Tp][feat_dim] with Tp = T/3; rows past frames[b]/3 are zero
 *   feat_len [B] = frames[b]/3
 * eps < 0 skips CMVN (the stacked features get_log_mel itself returns). */
int casr_features(casr_handle* h, const float* fbank, const int32_t* frames, int B, int T,
                  float eps, float* feat, int32_t* feat_len, void* stream);

/* wav -> log-mel (get_log_mel data.py:167-224, inference: no dither / augmentation):
 * pre-emphasis (data.py:201-202), |STFT|^2 with n_fft 512, hop 160, periodic hann(400)
 * centred, center=False (data.py:205-221), mel filterbank (MelScale, create_fb_matrix
 * data.py:21-106, incl. the linspace(80, 7600, 257) bin quirk), eps floor and log
 * (data.py:223-224).
 *   wav       [B][n_max] float32 samples (soundfile float32 scale), n_samples [B] int32
 *   fbank     [B][t_max][80] log-mel, rows past frames[b] zero
 *   frames    [B] = 1 + (n_samples[b] - 1 - 512) / 160  (0 and device flag 64 when
 *             n_samples[b] < 513, where torch.stft raises, data.py:204)
 * t_max must be >= casr_log_mel_frames(n_max). */
int casr_log_mel(casr_handle* h, const float* wav, const int32_t* n_samples, int B, int n_max, int t_max,
                 float preemphasis, float* fbank, int32_t* frames, void* stream);

/* Frames casr_log_mel produces for an utterance of n samples (0 if n < 513).  Host only. */
int casr_log_mel_frames(int n_samples);

/* The mel filterbank [n_stft][n_mels] casr_log_mel uses (create_fb_matrix, data.py:21-57,
 * float32).  Host only, no device needed. */
int casr_mel_filterbank(int n_stft, float f_min, float f_max, int n_mels, float* fb_host);

/* The list-of-tensors boundary of Model.eval_one_batch_* (model.py:514-516): gather B
 * device rows [lens[b]][feat_dim] (utt_ptrs is a DEVICE array of B device pointers) into
 * the padded batch-major [B][Tp][feat_dim] layout. */
int casr_gather_utterances(casr_handle* h, const float* const* utt_ptrs, const int32_t* lens,
                           int B, int Tp, float* feat, void* stream);

/* RNNEncoder.forward (encoder.py:36-81, RNN_RES util.py:1223-1324) + BauAttn
 * .compute_key_value (attention.py:67-78).  feat [B][Tp][feat_dim], lens [B] (<= Tp).
 * Results stay in the handle for the following casr_greedy / casr_beam. */
int casr_encode(casr_handle* h, const float* feat, const int32_t* lens, int B, int Tp, void* stream);

/* casr_features + casr_encode in one call, from fbank [B][T][n_mels] (frames [B]): the parse()
 * chain main.py:36-53 (stacking, deltas, CMVN with eps, then RNNEncoder.forward).  The features
 * stay inside the handle: in s16x3 arithmetic the feature kernel writes the encoder's layer-0
 * split-f16 row image directly, so the f32 features never reach HBM (results equal the two-call
 * sequence bit for bit).  feat_len [B] = frames[b]/3 is also written when not NULL. */
int casr_encode_fbank(casr_handle* h, const float* fbank, const int32_t* frames, int B, int T, float eps,
                      int32_t* feat_len, void* stream);

/* Copy of the encoder results (tests / EncoderOutput): enc [B][Tp][2H] (zeros past len),
 * h_final / c_final [B][2H] (last layer [fw || bw]), keys [B][A][Tp] (any may be NULL). */
int casr_encoder_results(casr_handle* h, float* enc, float* h_final, float* c_final, float* keys,
                         void* stream);

/* Model.eval_one_batch_with_greedy decode loop (model.py:527-580) on the last encode.
 *   tokens   [B][max_len] argmax token of every executed step
 *   out_len  [B] final_lens (tokens before the first EOS, model.py:573)
 *   finished [B] 0/1, accum [B] accumulated logp (model.py:567-576)
 *   align    NULL or [max_len][Tp][B] attention weights per step (model.py:553)
 * Score = accum / (out_len + finished) is formed by the host (model.py:593). */
int casr_greedy(casr_handle* h, int32_t* tokens, int32_t* out_len, uint8_t* finished, float* accum,
                float* align, void* stream);

/* Model.eval_one_batch_with_beam search loop (model.py:660-931) + first-max finalize
 * (model.py:765 / :961-972) for bmsz = k (1..16) on the last encode.
 *   best_tokens [B][max_len], best_len [B], best_score [B], steps [1] loop steps executed.
 * With length_weight the unfinished fallback adds length_weight*(l+1) (model.py:964). */
int casr_beam(casr_handle* h, int k, float lm_weight, float length_weight, int32_t* best_tokens,
              int32_t* best_len, float* best_score, int32_t* steps, void* stream);

/* Every finished hypothesis of the last casr_beam, for second-pass rescoring on the host
 * (parse_finished_tensors, model.py:708-765):
 *   rec_tokens [B][max_len][k][max_len] (record at step l has l tokens), rec_score
 *   [B][max_len][k], rec_valid [B][max_len][k] (0/1); order = (step, candidate rank). */
int casr_beam_records(casr_handle* h, int32_t* rec_tokens, float* rec_score, uint8_t* rec_valid,
                      void* stream);

/* Guard bits raised by the device since the previous casr_device_flags call (read and clear;
 * they accumulate over every encode / decode / log-mel call in between, so one read after a
 * series of calls vouches for all of them; 0 = clean): a data-dependent index out of range (1 token, 2 predecessor row, 4 NaN logit
 * row, 8 beam candidate, 16 back-pointer) is clamped and reported here instead of faulting
 * the device; 32 = a bounded hand-off wait of the persistent recurrence expired (results of
 * that casr_encode are invalid); 64 = casr_log_mel got an utterance shorter than 513
 * samples or longer than n_max; 128 = s16x3 arithmetic met a finite activation beyond the f16
 * range (|x| >= 65520: a layer input split by the encoder), so the split images and every
 * result after them are wrong: re-run the batch with casr_set_precision(CASR_PREC_F32) (the
 * Python Model does this itself, chinese-asr_amd/casr/engine.py run_checked).
 * Synchronises `stream`. */
int casr_device_flags(casr_handle* h, int32_t* flags_host, void* stream);

/* Encoder recurrence strategy.  Default (enable = 1): one persistent launch per layer runs all
 * Tp steps, workgroups keep W_hh and c in registers and exchange h through tagged
 * write-through granules; used when its grid (16 x ceil(B/32) x 2 workgroups of 512 threads)
 * fits the device's resident capacity, else the per-step launches below.  0 = per-step
 * launches always.  Both give bitwise identical results. */
int casr_set_persistent(casr_handle* h, int enable);

/* Arithmetic of the MFMA contractions (encoder input projection and recurrence; decoder LSTM
 * cell and projection).  Both compute in f32 on f32 data and keep f32 accumulators:
 *   CASR_PREC_F32    v_mfma_f32_16x16x4_f32, exact f32 products in k order;
 *   CASR_PREC_S16X3  every f32 operand split as hi + 2^-11 lo (two f16), three f16 MFMAs per
 *                    product (hi.hi + 2^-11 (hi.lo + lo.hi)) on the 16x-faster f16 pipes; 22
 *                    significant operand bits, measured error no larger than the f32 path's.
 *   CASR_PREC_S16X1  (round 6, an opt-in perf arithmetic, never the headline: BASELINE config 2's
 *                    "bf16 perf mode") the hi.hi MFMA of every split product only:
 *                    one f16 MFMA instead of three, 11 significant operand bits (bf16 keeps 8),
 *                    f32 accumulators.  Token ids are NOT identical to the reference's; bench.py
 *                    reports its token agreement.  It is a separate build of this library,
 *                    libcasr_hip_s16x1.so (casr/build.py variant "s16x1", -DCASR_S16_ONE=1), whose
 *                    s16 mode is S16X1: each build accepts F32 and its own s16 mode, and answers
 *                    the other s16 mode with CASR_ERR_UNSUPPORTED.
 * Default: the build's s16 mode.  A blob whose MFMA weights do not fit the split (non-finite,
 * |w| >= 2^14, or an encoder W_ih entry >= 16) runs F32 whatever is set; casr_get_precision
 * reports the effective mode. */
enum { CASR_PREC_F32 = 0, CASR_PREC_S16X3 = 1, CASR_PREC_S16X1 = 2 };
int casr_set_precision(casr_handle* h, int precision);
int casr_get_precision(const casr_handle* h); /* effective mode, -1 on a NULL handle */

/* Which recurrence casr_encode would use for batch B: 1 persistent, 0 per-step, -1 bad args.
 * Does not change the calling thread's current HIP device. */
int casr_recurrence_mode(const casr_handle* h, int B);

/* Tuning options of one handle.  The defaults are the measured fastest variants;
 * every value of every option gives the same results bit for bit (tests/test_gpu_parity.py sweeps
 * them), so an option only ever changes speed.  Options are read at each call and are part of the
 * keys of the captured hipGraphs, so changing one between calls takes effect at the next call.
 *   CASR_OPT_FUSE_SELECT     1 (default): the select of step l runs inside a kernel of step l + 1:
 *                            greedy, the LSTMCell (three-launch step) or the attention (folded
 *                            step); beam 4 or 8 with one attention block per utterance, or beam 8
 *                            with two (4 rows per block: both run the select, the first writes the
 *                            bookkeeping) (folded step), the attention.  0: every select a launch
 *                            of its own
 *   CASR_OPT_REC_LAYOUT      persistent recurrence workgroup shape: 0 auto (default: 16 rows x 16
 *                            units when that grid fits one workgroup per CU, else 32 x 16), 1 32x16,
 *                            2 16x32, 3 16x16
 *   CASR_OPT_REC_STORE_PLAIN 1: hand-off words stored L2-kept when the workgroup's whole hand-off
 *                            group runs on its XCD (checked per launch; default); 0: write-through
 *   CASR_OPT_REC_SLEEP       pacing of the recurrence's first poll per step, x 64 clocks; -1
 *                            (default, round 6): 0 for grids of 64 workgroups or more, 1 below
 *                            (B <= 16); measured: 0 is 2-3 % faster at B = 32 and 128, 1 is 1.6 %
 *                            faster at B = 1
 *   CASR_OPT_REC_POLL_GAP    second poll of a pass issued this many x 64 clocks after the first
 *                            (1..8, default 2)
 *   CASR_OPT_REC_COOP        2 (default, round 6): the persistent recurrence is an ordinary launch
 *                            after the occupancy check, ordered after the previous persistent launch
 *                            of this process on the same device (a process-wide event per device), so
 *                            two persistent grids of batches in flight never share the chip; 1: a
 *                            cooperative launch, so a grid that cannot be co-resident fails at launch
 *                            (the encode then falls back to the per-step recurrence) instead of
 *                            spinning into the hand-off timeout (about 25 us more per launch);
 *                            0: ordinary launch, unordered
 *   CASR_OPT_GEMM16_PERSIST  s16x3 input-projection kernel: 2 persistent ping-pong form (default: two
 *                            wave groups one barrier apart, 16-deep stages on a ring of four); 1
 *                            persistent, 32-deep stages on two buffers; 0 one workgroup per tile
 *   CASR_OPT_GEMM16_TAIL     2 (default): the persistent kernel takes whole rounds of tiles and the
 *                            rows after them go to one round of (32 RT) x 128 tiles; 1: to one
 *                            launch of 128 x 256 half tiles; 0: partial last round
 *   CASR_OPT_LOGMEL_Q16      1: casr_log_mel runs 16 lanes per frame, 16 FFT points per lane, one
 *                            stage exchange per frame (default, round 5); 0: one wave per frame, three
 *                            stage exchanges (round 4).  The same butterflies in the same order
 *   CASR_OPT_ATTN_KPB        beam rows per attention block at k > 2: 0 auto (8 at B >= 256 and
 *                            k >= 8, else 4), 4 or 8
 *   CASR_OPT_KEYS_ROWS       1: the s16x3 keys GEMM keeps W_enc in registers and streams 16-row
 *                            items of the encoder output through LDS, one workgroup per CU (default,
 *                            round 5); 0: 128 x 128 tiles (gemm_nt_kernel).  The same MFMAs in the
 *                            same order
 *   CASR_OPT_X16_KM          1: the s16 images of the encoder's layer inputs (and of W_ih) are laid
 *                            out 16-k-block major, so the input GEMM's 16-deep stages read whole
 *                            cache lines (default, round 5; in effect with GEMM16_PERSIST = 2,
 *                            GEMM16_TAIL != 1 and KEYS_ROWS = 1, the forms that read it); 0: row
 *                            images.  The same words in another order: the same bits
 *   CASR_OPT_GEMM16_LEAN     1: the ping-pong input projection (GEMM16_PERSIST = 2 on 16-k-major
 *                            images) advances its DMA sources by a stride per stage and waits on
 *                            constant vmcnt counts in its steady state (round 6); 0: 64-bit stage
 *                            addresses and the runtime wait ladder.  The same MFMAs in the same order
 * Three options select numerics variants instead (the same token ids, floating-point results within
 * the stated tolerances, not bit for bit; tests/test_gpu_parity.py compares each pair):
 *   CASR_OPT_DEC_KSPLIT      1: the greedy folded GEMM at R <= 32 decode rows (BASELINE config 2)
 *                            splits its k range over 4 workgroups per 32 x 112 output block (252
 *                            workgroups instead of 63; the 4 sums added in a fixed order by the last
 *                            to arrive) (default, round 5); 0: one workgroup per output block.  The
 *                            same products summed in another fixed order: tokens identical, scores
 *                            within 1e-4 of the unsplit form (test_greedy_ksplit_small_batch)
 *   CASR_OPT_ATTN_DIRECT     0: attention scores in the split exponential form 1 - 2 / (1 + e^{2k}
 *                            e^{2q}) (default; one transcendental per term); 1: the
 *                            direct tanh(k + q) form the split form falls back to per block
 *   CASR_OPT_DEC_FOLD        1: greedy decode in two launches per step (default; under f32 the
 *                            fused GEMM runs the exact-f32 MFMAs on an f32 fused image): the
 *                            projection GEMM also computes the next step's LSTM gate
 *                            pre-activations from the same [ctx | h] rows, the embedding part of
 *                            the gates is a per-token table built at bind, and the LSTM cell and
 *                            the attention query run inside the attention kernel;
 *                            0: three launches per step (LSTMCell GEMM, attention, projection).
 *                            Replaces decoder.py:104-114 + attention.py:92 + decoder.py:129-135 per
 *                            step with the same arithmetic regrouped (gates = [ctx | h] W_ch^T +
 *                            (emb W_emb^T + b), q by f32 fma chains).  It is also the default beam
 *                            step at R = B k >= 1024 decode rows when the attention takes 4 or 8 beam
 *                            rows per block and every projection and decoder LSTM weight is below 16
 *                            in magnitude (blob info words 4 and 5): there the fused GEMM runs the
 *                            one-accumulator s16x3 form (the whole sum scaled by 2^11) and the beam
 *                            attention kernel applies the cell (CELL 2).  Same token ids as the
 *                            three-launch step; scores within 2e-3, alignments within 1e-5
 *                            (tests/test_gpu_parity.py test_decode_fold_vs_three_launches,
 *                            test_beam_fold_vs_three_launches).  Not used by casr_beam at k = 1.
 * Two numerics choices are compile-time, not options (both on in the shipped build; the oracle
 * tests pin the tokens with them, both arithmetics):
 *   CASR_FAST_PART_EXP       (decoder.hip) the projection epilogue's per-block Σexp(x - max) partials
 *                            use v_exp_f32 of (x - max) log2(e) instead of libm expf: each row's
 *                            log-sum-exp, so the greedy accum and every beam score, moves in the
 *                            last bits (within the 2e-3 score tolerance), and at a near tie of two
 *                            beam candidates their rank can differ from an expf build's
 *   CASR_LOGITS_NT           (decoder.hip) beam logits stored with the non-temporal hint: speed only
 *   CASR_OPT_ATTN_SPLIT      0 (default): one attention block per utterance.  1 (round 6, measured and
 *                            not adopted): the folded greedy attention at R <= 64
 *                            decode rows (BASELINE config 2) splits each utterance's time steps over 8
 *                            (R <= 32) or 4 blocks, whose softmax maxima, sums and unnormalised
 *                            contexts the last block merges in split order (the same token ids; scores
 *                            within 1e-4 of the unsplit form, test_greedy_split_attention_small_batch);
 *                            2..8: that many ranges at every R <= 64.  Not with an alignment output
 *                            (it needs the whole row)
 * One option exists for tests only:
 *   CASR_OPT_REC_COOP_REFUSE 0 (default): off; n in 1..8: casr_encode treats the cooperative launch
 *                            of encoder layer n - 1 as refused (hipErrorCooperativeLaunchTooLarge,
 *                            without launching), so the mid-encode fallback to the per-step
 *                            recurrence (that layer and every later one) can be checked bit for bit
 *                            against all-persistent and all-per-step encodes
 * And one for measurement only (speed, never bits):
 *   CASR_OPT_DIAG_COLD       0 (default): off; a mask of kernel classes (bit CASR_K_*): before every
 *                            launch of such a class, a flush kernel reads a 1 GiB handle-owned buffer
 *                            (evicting every L2 and the 256 MiB Infinity Cache), outside the class's
 *                            timing events, so the class's time is that of cold operands: warm minus
 *                            cold shows how much of its traffic the Infinity Cache serves
 *                            (the GPU exposes no Infinity-Cache counter) */
enum {
  CASR_OPT_FUSE_SELECT = 0,
  CASR_OPT_REC_LAYOUT = 1,
  CASR_OPT_REC_STORE_PLAIN = 2,
  CASR_OPT_REC_SLEEP = 3,
  CASR_OPT_REC_POLL_GAP = 4,
  CASR_OPT_REC_COOP = 5,
  CASR_OPT_GEMM16_PERSIST = 6,
  CASR_OPT_GEMM16_TAIL = 7,
  CASR_OPT_ATTN_KPB = 8,
  CASR_OPT_ATTN_DIRECT = 9,
  CASR_OPT_DEC_FOLD = 10,
  CASR_OPT_REC_COOP_REFUSE = 11,
  CASR_OPT_DIAG_COLD = 12,
  CASR_OPT_LOGMEL_Q16 = 13,
  CASR_OPT_KEYS_ROWS = 14,
  CASR_OPT_X16_KM = 15,
  CASR_OPT_DEC_KSPLIT = 16,
  CASR_OPT_GEMM16_LEAN = 17,
  CASR_OPT_ATTN_SPLIT = 18,
  CASR_OPT_COUNT = 19
};
int casr_set_option(casr_handle* h, int option, int value);
int casr_get_option(const casr_handle* h, int option, int32_t* value_host);

/* hipGraph replay of the launch-bound loops: bit CASR_GRAPHS_DECODE = the whole decode loop,
 * bit CASR_GRAPHS_RECURRENCE = each layer's Tp steps of the per-step recurrence fallback; each
 * loop is captured once per shape on a private stream and replayed on `stream`, else its kernels
 * launch eagerly on `stream` (same results, bit for bit).  Default CASR_GRAPHS_RECURRENCE: the
 * decode loop launches eagerly, measured 0.1 ms faster per greedy batch and 0.17 ms per beam
 * batch than its replay (round 3; the host enqueues ~160 launches well ahead of the device). */
enum { CASR_GRAPHS_DECODE = 1, CASR_GRAPHS_RECURRENCE = 2 };
int casr_set_graphs(casr_handle* h, int mode);

/* Launch timing per kernel class with HIP event pairs recorded on the launch stream around
 * every launch of the enabled classes (bench.py's roofline figures).  Enabling resets
 * the counters; reading synchronises on the recorded events. */
enum {
  CASR_K_FEATURES = 0,   /* stack + CMVN */
  CASR_K_INPUT_PROJ = 1, /* encoder input-projection GEMM (per layer) */
  CASR_K_REC_STEP = 2,   /* one BiLSTM time step (both directions) */
  CASR_K_KEYS = 3,       /* attention key GEMM */
  CASR_K_DEC_LSTM = 4,   /* decoder LSTM cell GEMM */
  CASR_K_ATTENTION = 5,  /* additive attention + context */
  CASR_K_PROJ = 6,       /* output projection GEMM */
  CASR_K_SELECT = 7,     /* greedy argmax / beam top-2k + bookkeeping */
  CASR_K_COUNT = 8
};
int casr_profile_enable(casr_handle* h, uint32_t class_mask);
int casr_profile_read(casr_handle* h, int kernel_class, int32_t* launches, double* total_ms);

#ifdef __cplusplus
}
#endif
#endif /* CASR_H */
