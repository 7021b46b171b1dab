/* sampler.c -- TEST INFRASTRUCTURE (see oracle.h).
 * Line-by-line restatement of src/rwkv_sampler.rs:55-211 (sample_logits_with_top_p_k).
 * All arithmetic f32 in the reference's order. f32::exp on Linux is glibc expf; f32::powf is
 * glibc powf. sort_by(b.partial_cmp(a)) is a stable descending sort: equal probabilities keep
 * ascending index order, which is what the (p desc, index asc) comparator below reproduces for
 * NaN-free inputs. */
#include <math.h>
#include <stdlib.h>
#include "oracle.h"

float oracle_expf(float x) { return expf(x); }

typedef struct {
  float p;
  int i;
} pi_t;

static int cmp_desc_stable(const void* a, const void* b) {
  const pi_t* x = (const pi_t*)a;
  const pi_t* y = (const pi_t*)b;
  if (x->p > y->p) return -1;
  if (x->p < y->p) return 1;
  return (x->i < y->i) ? -1 : (x->i > y->i);
}

int oracle_sample_dbg(const float* logits, int n, float temperature, float top_p, int top_k,
                      int forbid, oracle_rng* rng, float* sum_out, float* r_out) {
  if (n == 0) return 0; /* :64-66 */
  float* probs = (float*)malloc(sizeof(float) * (size_t)n);
  for (int i = 0; i < n; ++i) probs[i] = logits[i];
  if (forbid >= 0 && forbid < n) probs[forbid] = -INFINITY; /* :72-76 */

  /* softmax :79-92 -- max fold from -inf, exp(l - max), sequential f32 sum, divide */
  float mx = -INFINITY;
  for (int i = 0; i < n; ++i) mx = fmaxf(mx, probs[i]); /* f32::max ignores NaN like fmaxf */
  for (int i = 0; i < n; ++i) probs[i] = expf(probs[i] - mx);
  float sum = 0.0f;
  for (int i = 0; i < n; ++i) sum += probs[i];
  if (sum > 0.0f)
    for (int i = 0; i < n; ++i) probs[i] /= sum;
  if (sum_out) *sum_out = sum;

  pi_t* ip = (pi_t*)malloc(sizeof(pi_t) * (size_t)n);
  /* top-k :95-105 */
  if (top_k > 0 && top_k < n) {
    for (int i = 0; i < n; ++i) { ip[i].p = probs[i]; ip[i].i = i; }
    qsort(ip, (size_t)n, sizeof(pi_t), cmp_desc_stable);
    for (int r = top_k; r < n; ++r) probs[ip[r].i] = 0.0f;
  }
  /* top-p :108-153 */
  if (top_p < 1.0f) {
    for (int i = 0; i < n; ++i) { ip[i].p = probs[i]; ip[i].i = i; }
    qsort(ip, (size_t)n, sizeof(pi_t), cmp_desc_stable);
    float cum = 0.0f, cutoff = 0.0f;
    int found = 0;
    for (int r = 0; r < n; ++r) {
      cum += ip[r].p;
      if (cum >= top_p) { found = 1; cutoff = ip[r].p; break; }
    }
    if (found) {
      for (int i = 0; i < n; ++i)
        if (probs[i] < cutoff) probs[i] = 0.0f;
      if (top_p > 0.0f) {
        float cur = 0.0f;
        for (int i = 0; i < n; ++i) cur += probs[i];
        if (cur < top_p) {
          float remaining = top_p - cur;
          int cnt = 0;
          for (int i = 0; i < n; ++i) cnt += (probs[i] == cutoff);
          if (cnt > 0) {
            float adj = remaining / (float)cnt;
            for (int i = 0; i < n; ++i)
              if (probs[i] == cutoff) probs[i] = cutoff + adj;
          }
        }
      }
    }
  }
  free(ip);
  /* temperature :156-171 (skipped for T == 1: no renormalisation after top-k/top-p) */
  if (temperature != 1.0f && temperature > 0.0f) {
    float tinv = 1.0f / temperature;
    for (int i = 0; i < n; ++i)
      if (probs[i] > 0.0f) probs[i] = powf(probs[i], tinv);
    float s2 = 0.0f;
    for (int i = 0; i < n; ++i) s2 += probs[i];
    if (s2 > 0.0f)
      for (int i = 0; i < n; ++i) probs[i] /= s2;
  }
  /* multinomial :174-207 */
  oracle_rng tmp;
  if (!rng) { oracle_rng_seed_from_u64(42, &tmp); rng = &tmp; }
  float r = oracle_rng_gen_f32(rng);
  if (r_out) *r_out = r;
  int ret = -1;
  float cum = 0.0f;
  for (int i = 0; i < n; ++i) {
    cum += probs[i];
    if (r <= cum) { ret = i; break; }
  }
  if (ret < 0) {
    for (int i = n - 1; i >= 0; --i)
      if (probs[i] > 0.0f) { ret = i; break; }
  }
  if (ret < 0) ret = 0; /* :209-210 */
  free(probs);
  return ret;
}

int oracle_sample(const float* logits, int n, float temperature, float top_p, int top_k,
                  int forbid, oracle_rng* rng) {
  return oracle_sample_dbg(logits, n, temperature, top_p, top_k, forbid, rng, NULL, NULL);
}
