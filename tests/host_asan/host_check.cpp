// Host-side sanitizer driver for the C-ABI library (tests/test_host_sanitizer.py builds it with
// clang AddressSanitizer + UndefinedBehaviorSanitizer on the host half of casr_capi.hip; no GPU).
//
//   host_check <tensors.bin> <packed.bin> <fbank.bin>
//
// tensors.bin: casr_config (12 int32 + 1 float), then int64 count, then per tensor int64 n +
// n float32, in casr_weights_host order (encoder l, d: w_ih, w_hh, b_ih, b_hh; then the eleven
// decoder / attention tensors).  Every tensor gets its own exact-size heap buffer, so a read past
// any tensor's end in casr_pack_weights is an ASan report; the packed blob goes to an exact-size
// buffer too (casr_packed_weights_floats).  Writes the blob and the default mel filterbank for the
// test to compare with the product library, and checks the host error paths.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "casr.h"

#define EXPECT(c)                                                       \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "host_check: %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(3);                                                     \
    }                                                                   \
  } while (0)

static float* read_tensor(FILE* f) {
  long long n = 0;
  EXPECT(std::fread(&n, sizeof n, 1, f) == 1 && n > 0);
  float* p = static_cast<float*>(std::malloc(sizeof(float) * (size_t)n));
  EXPECT(p && std::fread(p, sizeof(float), (size_t)n, f) == (size_t)n);
  return p;
}

static void write_all(const char* path, const float* p, size_t n) {
  FILE* f = std::fopen(path, "wb");
  EXPECT(f && std::fwrite(p, sizeof(float), n, f) == n);
  std::fclose(f);
}

static bool has_message() {
  const char* m = casr_last_error(nullptr);
  return m && std::strlen(m) > 0;
}

int main(int argc, char** argv) {
  EXPECT(argc == 4);
  EXPECT(casr_api_version() == CASR_API_VERSION);
  FILE* f = std::fopen(argv[1], "rb");
  EXPECT(f);
  casr_config cfg;
  EXPECT(std::fread(&cfg, sizeof cfg, 1, f) == 1);
  long long count = 0;
  EXPECT(std::fread(&count, sizeof count, 1, f) == 1);
  EXPECT(count == 4LL * 2 * cfg.enc_layers + 11);
  casr_weights_host w;
  std::memset(&w, 0, sizeof w);
  std::vector<float*> owned;
  for (int l = 0; l < cfg.enc_layers; ++l)
    for (int d = 0; d < 2; ++d) {
      float* t[4];
      for (auto& x : t) owned.push_back(x = read_tensor(f));
      w.enc_w_ih[l][d] = t[0];
      w.enc_w_hh[l][d] = t[1];
      w.enc_b_ih[l][d] = t[2];
      w.enc_b_hh[l][d] = t[3];
    }
  const float** dec[11] = {&w.embedding, &w.dec_w_ih, &w.dec_w_hh, &w.dec_b_ih, &w.dec_b_hh, &w.proj_w,
                           &w.proj_b, &w.attn_w_enc, &w.attn_b, &w.attn_w_hidden, &w.attn_v};
  for (auto p : dec) {
    owned.push_back(read_tensor(f));
    *p = owned.back();
  }
  std::fclose(f);

  const size_t n = casr_packed_weights_floats(&cfg);
  EXPECT(n > 0);
  float* packed = static_cast<float*>(std::malloc(sizeof(float) * n));
  EXPECT(packed);
  EXPECT(casr_pack_weights(&cfg, &w, packed) == CASR_OK);
  write_all(argv[2], packed, n);

  // error paths: every one returns its code and leaves a message
  EXPECT(casr_pack_weights(nullptr, &w, packed) == CASR_ERR_ARG && has_message());
  EXPECT(casr_pack_weights(&cfg, nullptr, packed) == CASR_ERR_ARG && has_message());
  EXPECT(casr_pack_weights(&cfg, &w, nullptr) == CASR_ERR_ARG && has_message());
  {
    casr_weights_host w2 = w;
    w2.attn_v = nullptr;
    EXPECT(casr_pack_weights(&cfg, &w2, packed) == CASR_ERR_ARG && has_message());
    w2 = w;
    w2.enc_b_hh[cfg.enc_layers - 1][1] = nullptr;
    EXPECT(casr_pack_weights(&cfg, &w2, packed) == CASR_ERR_ARG && has_message());
  }
  {
    casr_config bad = cfg;
    bad.enc_hidden = 128;
    EXPECT(casr_packed_weights_floats(&bad) == 0);
    EXPECT(casr_pack_weights(&bad, &w, packed) == CASR_ERR_UNSUPPORTED && has_message());
    bad = cfg;
    bad.vocab = 3;
    EXPECT(casr_pack_weights(&bad, &w, packed) == CASR_ERR_ARG);
    bad = cfg;
    bad.eos = cfg.vocab;
    EXPECT(casr_pack_weights(&bad, &w, packed) == CASR_ERR_ARG);
    bad = cfg;
    bad.temperature = 0.f;
    EXPECT(casr_pack_weights(&bad, &w, packed) == CASR_ERR_ARG);
    bad = cfg;
    bad.enc_layers = CASR_MAX_LAYERS + 1;
    EXPECT(casr_pack_weights(&bad, &w, packed) == CASR_ERR_ARG);
  }
  EXPECT(casr_set_option(nullptr, 0, 1) == CASR_ERR_ARG);
  {
    int32_t v = 0;
    EXPECT(casr_get_option(nullptr, 0, &v) == CASR_ERR_ARG);
  }
  EXPECT(casr_set_precision(nullptr, 0) == CASR_ERR_ARG);
  EXPECT(casr_get_precision(nullptr) == -1);
  EXPECT(casr_set_graphs(nullptr, 1) == CASR_ERR_ARG);
  EXPECT(casr_create(&cfg, 0, nullptr) == CASR_ERR_ARG);
  casr_destroy(nullptr);

  // front end host helpers
  EXPECT(casr_log_mel_frames(0) == 0);
  EXPECT(casr_log_mel_frames(-5) == 0);
  EXPECT(casr_log_mel_frames(16000) > 0);
  const int n_stft = 257, n_mels = 80;
  float* fb = static_cast<float*>(std::malloc(sizeof(float) * n_stft * n_mels));
  EXPECT(fb);
  EXPECT(casr_mel_filterbank(n_stft, 80.f, 7600.f, n_mels, fb) == CASR_OK);
  write_all(argv[3], fb, (size_t)n_stft * n_mels);
  EXPECT(casr_mel_filterbank(0, 80.f, 7600.f, n_mels, fb) == CASR_ERR_ARG);
  EXPECT(casr_mel_filterbank(n_stft, 80.f, 7600.f, n_mels, nullptr) == CASR_ERR_ARG);

  std::free(fb);
  std::free(packed);
  for (float* p : owned) std::free(p);
  std::puts("host_check ok");
  return 0;
}
