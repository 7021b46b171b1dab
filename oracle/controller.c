/* controller.c -- TEST INFRASTRUCTURE (see oracle.h).
 * Serial phase controllers, one request at a time on a fresh state (the uncontended reference,
 * SURVEY Appendix B1):
 *  - normal mode: src/normal_mode_inference.rs:37-391
 *      prompt = property ⧺ [TAG_2] ⧺ text ⧺ [TAG_0] (:37-41); prefill until logits (:74-80);
 *      32 global samples from logits[0:4096) (k20 p.95 T1, StdRng(seed+1000)), each fed back
 *      as g+8196 (:222-287); push TAG_1 and infer (:303-313); semantic loop i < min(max_tokens,
 *      2048) (:316): logits with j > 8192 and tags masked, k80 p.95 T1, StdRng(seed+2000),
 *      EOS -> stop, else feed raw id (:319-391). The last pushed token is never inferred.
 *  - zero-shot: src/zero_shot_inference.rs:47-364
 *      prompt = property ⧺ [TAG_2] ⧺ text ⧺ [TAG_0] ⧺ (clamp(g,0,4095)+8196)... ⧺ [TAG_1]
 *      (:47,76-85); EOS masked while i < hard_min (:128-142,256-261); window rule (12, 0.7) with
 *      re-draw (:219-309). Seed: the reference ignores it (B5); this build seeds the semantic
 *      stream with seed + semantic_seed_offset when a seed is given, as normal mode does
 *      (StdRng(0) when use_independent_seeds is off, as the reference).
 *  - benchmark extensions: fixed_semantic > 0 masks EOS and emits exactly that
 *      many semantic tokens; greedy forces top_k = 1 in both phases.
 * Sampling always sees the prefix rows that can be drawn (global: 4096; semantic: 8193);
 * masked rows contribute exp(-inf) = 0 to every sum, so this is bit-identical to sampling the
 * full-length masked vector. */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define SEM_ROWS (RWKVTTS_EOS_TOKEN + 1)

typedef struct {
  const oracle_model* m;
  float* state;
  float* logits;
  int head_rows;
  int n_forward;
} runner;

static void feed(runner* rn, uint32_t tok, int want_logits) {
  oracle_forward_token(rn->m, rn->state, tok, want_logits ? rn->logits : NULL, rn->head_rows);
  rn->n_forward++;
}

int oracle_generate(const oracle_model* m, const rwkvtts_request* req, oracle_result* out) {
  memset(out, 0, sizeof(*out));
  runner rn;
  rn.m = m;
  rn.head_rows = SEM_ROWS;
  rn.n_forward = 0;
  const int64_t sf = oracle_state_floats(m);
  rn.state = (float*)calloc((size_t)sf, sizeof(float));
  rn.logits = (float*)malloc(sizeof(float) * SEM_ROWS);
  float* row = (float*)malloc(sizeof(float) * SEM_ROWS);

  const int zero_shot = req->ref_global != NULL && req->ref_semantic != NULL;
  const uint64_t seed = req->has_seed ? req->seed : 0; /* no seed: caller must pass one */
  /* LayeredRandomnessConfig (rwkv_sampler.rs:251-275): normal_mode_inference.rs:138-174 */
  const int indep = req->layered_set ? req->use_independent_seeds != 0 : 1;
  const uint64_t goff = req->layered_set ? req->global_seed_offset : 1000;
  const uint64_t soff = req->layered_set ? req->semantic_seed_offset : 2000;
  const uint64_t gseed = indep ? seed + goff : seed + 100;
  /* zero-shot without independent seeds: the StdRng::seed_from_u64(0) of
   * dynamic_batch_manager.rs:491-494 (zero_shot_inference.rs:204-216) */
  const uint64_t sseed = indep ? seed + soff : (zero_shot ? 0 : seed + 200);

  /* ---- prompt ---- */
  int n_prompt = req->n_property + 1 + req->n_text + 1 + (zero_shot ? req->n_ref_global + 1 : 0);
  uint32_t* prompt = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n_prompt);
  int p = 0;
  for (int i = 0; i < req->n_property; ++i) prompt[p++] = (uint32_t)req->property_tokens[i];
  prompt[p++] = RWKVTTS_TAG_2;
  for (int i = 0; i < req->n_text; ++i) prompt[p++] = (uint32_t)req->text_tokens[i];
  prompt[p++] = RWKVTTS_TAG_0;
  if (zero_shot) {
    for (int i = 0; i < req->n_ref_global; ++i) {
      int g = req->ref_global[i];
      g = g < 0 ? 0 : (g > 4095 ? 4095 : g);
      prompt[p++] = (uint32_t)(g + RWKVTTS_GLOBAL_TOKEN_OFFSET);
    }
    prompt[p++] = RWKVTTS_TAG_1;
  }
  for (int i = 0; i < n_prompt; ++i) feed(&rn, prompt[i], i == n_prompt - 1);
  free(prompt);

  const int kg = req->greedy ? 1 : 20, ks = req->greedy ? 1 : 80;
  /* usize::min(max_tokens, 2048) (normal_mode_inference.rs:316): 0 -> no semantic tokens */
  int limit = req->max_tokens > 0 ? req->max_tokens : 0;
  if (limit > RWKVTTS_SEMANTIC_LIMIT) limit = RWKVTTS_SEMANTIC_LIMIT;
  if (req->fixed_semantic > 0) limit = req->fixed_semantic < RWKVTTS_SEMANTIC_LIMIT ? req->fixed_semantic : RWKVTTS_SEMANTIC_LIMIT;

  if (!zero_shot) {
    oracle_rng rg, rs;
    oracle_rng_seed_from_u64(gseed, &rg);
    oracle_rng_seed_from_u64(sseed, &rs);
    for (int i = 0; i < RWKVTTS_N_GLOBAL; ++i) {
      if (i > 0) feed(&rn, (uint32_t)(out->global_tokens[i - 1] + RWKVTTS_GLOBAL_TOKEN_OFFSET), 1);
      int id = oracle_sample(rn.logits, 4096, 1.0f, 0.95f, kg, -1, &rg);
      out->global_tokens[out->n_global++] = id;
    }
    feed(&rn, (uint32_t)(out->global_tokens[RWKVTTS_N_GLOBAL - 1] + RWKVTTS_GLOBAL_TOKEN_OFFSET), 0);
    feed(&rn, RWKVTTS_TAG_1, 1);
    for (int i = 0; i < limit; ++i) {
      if (i > 0) feed(&rn, (uint32_t)out->semantic_tokens[i - 1], 1);
      memcpy(row, rn.logits, sizeof(float) * SEM_ROWS);
      if (req->fixed_semantic > 0) row[RWKVTTS_EOS_TOKEN] = -INFINITY;
      int id = oracle_sample(row, SEM_ROWS, 1.0f, 0.95f, ks, -1, &rs);
      if (id == RWKVTTS_EOS_TOKEN) break;
      out->semantic_tokens[out->n_semantic++] = id;
    }
  } else {
    for (int i = 0; i < req->n_ref_global && i < RWKVTTS_N_GLOBAL; ++i) {
      int g = req->ref_global[i];
      out->global_tokens[out->n_global++] = g < 0 ? 0 : (g > 4095 ? 4095 : g);
    }
    oracle_rng rs;
    oracle_rng_seed_from_u64(sseed, &rs);
    const int tlen = req->n_text;
    int min_sem = tlen / 4;
    min_sem = min_sem < 8 ? 8 : (min_sem > 64 ? 64 : min_sem);
    int est = (int)ceilf((float)tlen * 1.8f);
    int upper = (int)floorf((float)RWKVTTS_SEMANTIC_LIMIT * 0.9f);
    int hard_min = est > min_sem ? est : min_sem;
    if (hard_min > upper) hard_min = upper;
    int zlimit = RWKVTTS_SEMANTIC_LIMIT;
    if (req->fixed_semantic > 0) zlimit = limit;
    int window[12], wlen = 0;
    for (int i = 0; i < zlimit; ++i) {
      if (i > 0) feed(&rn, (uint32_t)out->semantic_tokens[i - 1], 1);
      memcpy(row, rn.logits, sizeof(float) * SEM_ROWS);
      if (i < hard_min || req->fixed_semantic > 0) row[RWKVTTS_EOS_TOKEN] = -INFINITY;
      int id = oracle_sample(row, SEM_ROWS, 1.0f, 0.95f, ks, -1, &rs);
      if (id == RWKVTTS_EOS_TOKEN) {
        int non_eos = 0;
        for (int j = 0; j < wlen; ++j) non_eos += window[j];
        float ratio = wlen > 0 ? (float)non_eos / (float)wlen : 0.0f;
        if (wlen >= 12 && ratio >= 0.7f) break;
        row[RWKVTTS_EOS_TOKEN] = -INFINITY;
        id = oracle_sample(row, SEM_ROWS, 1.0f, 0.95f, ks, -1, &rs);
      }
      if (id > RWKVTTS_EOS_TOKEN) break;
      int is_non_eos = id != RWKVTTS_EOS_TOKEN;
      if (wlen == 12) {
        memmove(window, window + 1, sizeof(int) * 11);
        wlen = 11;
      }
      window[wlen++] = is_non_eos;
      out->semantic_tokens[out->n_semantic++] = id;
    }
  }
  out->n_forward = rn.n_forward;
  free(rn.state);
  free(rn.logits);
  free(row);
  return 0;
}
