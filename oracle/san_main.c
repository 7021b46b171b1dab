/* san_main.c -- TEST INFRASTRUCTURE: drives every entry point of the CPU restatement (the oracle C files)
 * in one native process built with AddressSanitizer + UndefinedBehaviorSanitizer
 * (`make -C oracle SAN=1 san_check`). The ctypes checker cannot run an
 * ASan-instrumented library inside an uninstrumented Python, so this executable is the sanitized
 * form of what tests/ call through oracle.py. Usage:
 *   san_check MODEL_BLOB CODEC_DIMS CODEC_WEIGHTS
 * MODEL_BLOB: a rwkvtts weight blob (tests write W.synth_blob(W.DIMS_TINY)); CODEC_DIMS: the raw
 * bytes of a rwkvtts_codec_dims; CODEC_WEIGHTS: its f32 weight blob. Exit 0 = every check passed
 * and no sanitizer fired (the sanitizers abort with a report otherwise). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static void* slurp(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc((size_t)len > 0 ? (size_t)len : 1);
  if (len > 0 && fread(p, 1, (size_t)len, f) != (size_t)len) {
    fprintf(stderr, "short read %s\n", path);
    exit(2);
  }
  fclose(f);
  *n = (size_t)len;
  return p;
}

static uint64_t lcg = 0x9E3779B97F4A7C15ull;
static float frand(void) { /* [-1, 1) */
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((lcg >> 40) & 0xFFFFFF) / 8388608.0f - 1.0f;
}

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "check failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                     \
    }                                                               \
  } while (0)

static int rng_checks(void) {
  uint32_t out[16];
  const uint32_t key[8] = {0};
  oracle_chacha_block(key, 0, 0, 20, out);
  CHECK(out[0] == 0xade0b876u); /* all-zero ChaCha20 known answer */
  for (uint64_t s = 0; s < 64; ++s) {
    oracle_rng r;
    oracle_rng_seed_from_u64(s, &r);
    for (int i = 0; i < 100; ++i) {
      const float f = oracle_rng_gen_f32(&r);
      CHECK(f >= 0.0f && f < 1.0f);
    }
  }
  return 0;
}

static int sampler_checks(void) {
  const int ns[] = {1, 2, 7, 64, 4096, 8193, 77923};
  const int ks[] = {0, 1, 20, 80, 300};
  const float ps[] = {0.0f, 0.85f, 0.95f, 1.0f};
  float* row = (float*)malloc(sizeof(float) * 77923);
  for (size_t a = 0; a < sizeof(ns) / sizeof(ns[0]); ++a) {
    const int n = ns[a];
    for (int shape = 0; shape < 4; ++shape) {
      for (int i = 0; i < n; ++i) {
        float v = frand() * 3.0f;
        if (shape == 1) v = (i % 7 == 0) ? 1.0f : 1.0f + 1e-7f * (float)(i % 3); /* near-ties */
        if (shape == 2) v = (i == n / 2) ? 30.0f : -INFINITY;                  /* one-hot */
        if (shape == 3 && i % 5 == 0) v = -INFINITY;                            /* masked columns */
        row[i] = v;
      }
      if (shape == 3) row[0] = 0.5f;
      for (size_t b = 0; b < sizeof(ks) / sizeof(ks[0]); ++b)
        for (size_t c = 0; c < sizeof(ps) / sizeof(ps[0]); ++c) {
          oracle_rng r;
          oracle_rng_seed_from_u64(1000 + a * 97 + b * 13 + c, &r);
          float sum = 0.f, draw = 0.f;
          const int t = oracle_sample_dbg(row, n, 1.0f, ps[c], ks[b], -1, &r, &sum, &draw);
          CHECK(t >= 0 && t < n);
          const int t2 = oracle_sample(row, n, 0.7f, ps[c], ks[b], n > 1 ? 0 : -1, NULL);
          CHECK(t2 >= 0 && t2 < n);
        }
    }
  }
  free(row);
  return 0;
}

static int model_checks(const void* blob, size_t bytes) {
  oracle_set_threads(2);
  oracle_model* m = oracle_model_load(blob, bytes);
  CHECK(m != NULL);
  const int64_t nf = oracle_state_floats(m);
  CHECK(nf > 0);
  float* st = (float*)calloc((size_t)nf, sizeof(float));
  float* logits = (float*)malloc(sizeof(float) * 8193);
  for (int i = 0; i < 24; ++i) {
    oracle_forward_token(m, st, (uint32_t)(12293 + 37 * i), logits, i % 2 ? 8193 : 0);
    if (i % 2) CHECK(isfinite(logits[0]) && isfinite(logits[8192]));
  }
  int32_t text[12], props[6] = {77823, 77838, 77869, 77845, 77830, 77826};
  for (int i = 0; i < 12; ++i) text[i] = 12293 + 101 * i;
  int32_t rg[32], rs[20];
  for (int i = 0; i < 32; ++i) rg[i] = (i * 131) % 4096;
  for (int i = 0; i < 20; ++i) rs[i] = (i * 313) % 8192;
  oracle_result* res = (oracle_result*)malloc(sizeof(oracle_result));
  for (int mode = 0; mode < 3; ++mode) {
    rwkvtts_request q;
    memset(&q, 0, sizeof(q));
    q.text_tokens = text;
    q.n_text = 12;
    q.has_seed = 1;
    q.seed = 7 + mode;
    q.max_tokens = 24;
    if (mode == 0) { /* normal mode, sampled until EOS or the limit */
      q.property_tokens = props;
      q.n_property = 6;
    } else if (mode == 1) { /* fixed-length benchmark mode */
      q.property_tokens = props;
      q.n_property = 6;
      q.fixed_semantic = 6;
    } else { /* zero-shot with reference tokens */
      q.ref_global = rg;
      q.n_ref_global = 32;
      q.ref_semantic = rs;
      q.n_ref_semantic = 20;
    }
    memset(res, 0, sizeof(*res));
    CHECK(oracle_generate(m, &q, res) == 0);
    CHECK(res->n_semantic >= 0 && res->n_semantic <= RWKVTTS_SEMANTIC_LIMIT);
    if (mode == 1) CHECK(res->n_semantic == 6 && res->n_global == 32);
  }
  CHECK(oracle_model_quantize(m, 1, 1) == 0); /* Int8 layer 0 */
  oracle_forward_token(m, st, 12345, logits, 8193);
  CHECK(isfinite(logits[100]));
  free(res);
  free(logits);
  free(st);
  oracle_model_free(m);
  return 0;
}

static int mel_checks(void) {
  const int lens[] = {0, 1, 399, 400, 16000, 20801};
  for (size_t a = 0; a < sizeof(lens) / sizeof(lens[0]); ++a) {
    const int n = lens[a];
    float* wav = (float*)malloc(sizeof(float) * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) wav[i] = 0.3f * frand();
    const int frames = n / 320 + 1; /* (n + 2 * 512 - 1024) / 320 + 1, or 1 (mel.c) */
    float* mel = (float*)malloc(sizeof(float) * 128 * (size_t)frames);
    int f2 = 0;
    CHECK(oracle_mel(n ? wav : NULL, n, mel, &f2) == 0);
    CHECK(f2 == frames);
    for (int i = 0; i < 128 * f2; ++i) CHECK(isfinite(mel[i]));
    free(mel);
    free(wav);
  }
  return 0;
}

static int codec_checks(const rwkvtts_codec_dims* d, const float* w) {
  const int T = 16;
  int64_t sem[16], glob[64];
  for (int i = 0; i < T; ++i) sem[i] = (i * 977) % d->codebook_size;
  for (int i = 0; i < d->n_global && i < 64; ++i) glob[i] = (i * 59) % 4096;
  const int per_frame = 320;
  float* pcm = (float*)malloc(sizeof(float) * (size_t)T * per_frame * 2);
  CHECK(oracle_codec_decode(d, w, sem, T, glob, pcm) == 0);
  for (int i = 0; i < T * per_frame; ++i) CHECK(isfinite(pcm[i]));
  free(pcm);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: san_check MODEL_BLOB CODEC_DIMS CODEC_WEIGHTS\n");
    return 2;
  }
  size_t nb = 0, nd = 0, nw = 0;
  void* blob = slurp(argv[1], &nb);
  void* dims = slurp(argv[2], &nd);
  void* cw = slurp(argv[3], &nw);
  if (nd != sizeof(rwkvtts_codec_dims)) {
    fprintf(stderr, "codec dims: %zu bytes, expected %zu\n", nd, sizeof(rwkvtts_codec_dims));
    return 2;
  }
  int rc = rng_checks();
  if (!rc) rc = sampler_checks();
  if (!rc) rc = model_checks(blob, nb);
  if (!rc) rc = mel_checks();
  if (!rc) rc = codec_checks((const rwkvtts_codec_dims*)dims, (const float*)cw);
  free(blob);
  free(dims);
  free(cw);
  if (!rc) printf("san_check: ok\n");
  return rc;
}
