/*
 * oracle.h -- CPU restatement of the liuzl/rwkv-tts-rs hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
 * product library (rwkv-tts-rs_amd/) never links, calls or falls back to it.
 *
 * What each part restates (reference root = /root/reference, Cargo.lock pins):
 *   rng.c        rand 0.8.5 StdRng = rand_chacha 0.3.1 ChaCha12Rng, rand_core 0.6.4
 *                seed_from_u64 (PCG32 fill), Standard f32 = (u32 >> 8) * 2^-24
 *                (third-party crates, absent from the tree; used at src/normal_mode_inference.rs:138-174).
 *                Pinned by the RFC 8439 / ChaCha known-answer vectors (tests/test_oracle_rng.py).
 *   sampler.c    src/rwkv_sampler.rs:55-211 sample_logits_with_top_p_k, f32 throughout, glibc expf
 *                (what Rust f32::exp calls on Linux), stable descending sort.
 *   rwkv7.c      RWKV-7 "x070" forward as executed by web-rwkv 0.10.16 v7::Bundle<f32>
 *                (external crate, not vendored): f32 activations/state, matrices
 *                read from the 2-byte blob.  PARITY UNPINNED against web-rwkv itself (no source,
 *                weights or GPU runtime here); pinned only by restatement.
 *   controller.c src/normal_mode_inference.rs:37-391, src/zero_shot_inference.rs:47-364.
 *   codec.c      BiCodec decoder restatement (SparkTTS arch, assumed; ONNX graph absent:
 *                parity unpinned against ORT; IO contract from lightweight_tts_pipeline.rs:706-730).
 *   mel.c        src/tts_pipeline_fixes.rs:12-159.
 */
#ifndef RWKVTTS_ORACLE_H
#define RWKVTTS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/rwkvtts.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- rng.c ---------------- */
typedef struct {
  uint32_t key[8];
  uint64_t index; /* next u32 draw index (block = index / 16) */
} oracle_rng;
void oracle_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds,
                         uint32_t out[16]);
void oracle_chacha_block_raw(const uint32_t in[16], int rounds, uint32_t out[16]);
void oracle_rng_seed_from_u64(uint64_t seed, oracle_rng* r);
uint32_t oracle_rng_next_u32(oracle_rng* r);
float oracle_rng_gen_f32(oracle_rng* r);

/* ---------------- sampler.c ---------------- */
/* rng == NULL mirrors `rng: &mut None` (fresh StdRng::seed_from_u64(42)). forbid < 0 = None. */
int oracle_sample(const float* logits, int n, float temperature, float top_p, int top_k,
                  int forbid, oracle_rng* rng);
/* Debug variant: also returns the softmax denominator and the draw. */
int oracle_sample_dbg(const float* logits, int n, float temperature, float top_p, int top_k,
                      int forbid, oracle_rng* rng, float* sum_out, float* r_out);
float oracle_expf(float x); /* = glibc expf */

/* ---------------- rwkv7.c ---------------- */
typedef struct oracle_model oracle_model;
oracle_model* oracle_model_load(const void* blob, size_t bytes);
void oracle_model_free(oracle_model* m);
/* web-rwkv Quant restated (rwkv7.c): layers [0, quant_layers) use dequantised r / k / v / o / FFN
 * matrices; quant_type 1 Int8, 2 NF4 (0: none). 0 ok, -1 invalid. */
int oracle_model_quantize(oracle_model* m, int quant_layers, int quant_type);
int64_t oracle_state_floats(const oracle_model* m);
/* one token; state updated in place; logits (head_rows, may be NULL) of this token */
void oracle_forward_token(const oracle_model* m, float* state, uint32_t token, float* logits,
                          int head_rows);
void oracle_set_threads(int n);

/* ---------------- controller.c ---------------- */
typedef struct {
  int32_t n_global, n_semantic;
  int32_t global_tokens[RWKVTTS_N_GLOBAL];
  int32_t semantic_tokens[RWKVTTS_SEMANTIC_LIMIT];
  int32_t n_forward; /* tokens pushed through the model */
} oracle_result;
/* Same request struct as the product ABI; runs the reference's serial phase logic. If
 * trace_logits != NULL it receives the masked row each sample was drawn from
 * (n_samples x 8193, see controller.c). */
int oracle_generate(const oracle_model* m, const rwkvtts_request* req, oracle_result* out);

/* ---------------- mel.c ---------------- */
int oracle_mel(const float* wav, int n, float* mel, int* n_frames);

/* ---------------- codec.c ---------------- */
int oracle_codec_decode(const rwkvtts_codec_dims* d, const float* weights, const int64_t* semantic,
                        int T, const int64_t* global, float* pcm);

#ifdef __cplusplus
}
#endif
#endif
