/*
 * codec.c -- TEST INFRASTRUCTURE (see oracle.h). f32 CPU restatement of the BiCodec decoder
 * (BiCodecDetokenize.onnx, run by the reference through ORT at
 * src/lightweight_tts_pipeline.rs:706-730; IO contract semantic [1,T] i64 + global [1,1,32] i64
 * -> wav f32 [T*320]).  The graph itself is not in the reference tree: the structure below is
 * upstream SparkTTS BiCodec.detokenize as described in SURVEY §8a-7 -- PARITY UNPINNED against
 * ORT; the GPU path is checked against this restatement on synthetic weights.
 *
 *   z      = out_proj(codebook[semantic])                          [T][latent]
 *   d      = spk_proj(flatten_{c,t}(fsq_proj(fsq_codes(global))))   [spk]
 *   x      = linear_pre(z); x = AdaLN0(embed_conv7(x), d)
 *   x      = x + gamma * pw2(gelu(pw1(AdaLN(dwconv7(x), d))))     (x prenet_layers)
 *   x      = linear(LN(x)) + d
 *   x      = conv7(x); per up block: snake -> convT(k,s) -> 3 x [x + conv1(snake(conv7_dil(snake(x))))]
 *   wav    = tanh(conv7(snake(x)))
 * Activations are channel-last [t][c]; weights are read from the layout of
 * include/rwkvtts_codec_layout.h.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "../include/rwkvtts_codec_layout.h"

#define W(g, i, t) (w + rwkvtts_codec_offset(d, (g), (i), (t)))

/* y[t][co] = b[co] + sum_{k,ci} W[co][k][ci] * act(x[t + k*dil - pad][ci])  (stride 1, zero pad) */
static void conv1d(const float* x, int T, int Ci, const float* wt, const float* b, int Co, int K,
                   int dil, int pad, const float* alpha, float* y) {
  float* xs = NULL;
  if (alpha) { /* Snake1d: x + 1/(alpha + 1e-9) * sin(alpha * x)^2 (applied before zero padding) */
    xs = (float*)malloc(sizeof(float) * (size_t)T * Ci);
    for (int64_t i = 0; i < (int64_t)T * Ci; ++i) {
      const float a = alpha[i % Ci], v = x[i], s = sinf(a * v);
      xs[i] = v + (1.0f / (a + 1e-9f)) * (s * s);
    }
    x = xs;
  }
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T; ++t)
    for (int co = 0; co < Co; ++co) {
      float acc = 0.0f;
      for (int k = 0; k < K; ++k) {
        const int p = t + k * dil - pad;
        if (p < 0 || p >= T) continue;
        const float* wr = wt + ((int64_t)co * K + k) * Ci;
        const float* xr = x + (int64_t)p * Ci;
        for (int ci = 0; ci < Ci; ++ci) acc += wr[ci] * xr[ci];
      }
      y[(int64_t)t * Co + co] = acc + b[co];
    }
  free(xs);
}

/* ConvTranspose1d(stride s, padding p = (K - s) / 2): out length T*s;
 * y[to][co] = b[co] + sum_{ti,k: to = ti*s + k - p} W[co][k][ci] * act(x[ti][ci]) */
static void conv_transpose1d(const float* x, int T, int Ci, const float* wt, const float* b, int Co,
                             int K, int s, const float* alpha, float* y) {
  const int p = (K - s) / 2, To = T * s;
  float* xs = (float*)malloc(sizeof(float) * (size_t)T * Ci);
  for (int64_t i = 0; i < (int64_t)T * Ci; ++i) {
    const float a = alpha[i % Ci], v = x[i], sn = sinf(a * v);
    xs[i] = v + (1.0f / (a + 1e-9f)) * (sn * sn);
  }
#pragma omp parallel for schedule(static)
  for (int to = 0; to < To; ++to)
    for (int co = 0; co < Co; ++co) {
      float acc = 0.0f;
      for (int k = 0; k < K; ++k) {
        const int num = to + p - k;
        if (num < 0 || num % s) continue;
        const int ti = num / s;
        if (ti >= T) continue;
        const float* wr = wt + ((int64_t)co * K + k) * Ci;
        const float* xr = xs + (int64_t)ti * Ci;
        for (int ci = 0; ci < Ci; ++ci) acc += wr[ci] * xr[ci];
      }
      y[(int64_t)to * Co + co] = acc + b[co];
    }
  free(xs);
}

/* y = LayerNorm(x) (eps 1e-6, no affine) * scale + shift over the last dim */
static void layer_norm_rows(float* x, int T, int C, const float* scale, const float* shift) {
  for (int t = 0; t < T; ++t) {
    float* r = x + (int64_t)t * C;
    float mean = 0.0f, var = 0.0f;
    for (int c = 0; c < C; ++c) mean += r[c];
    mean /= (float)C;
    for (int c = 0; c < C; ++c) var += (r[c] - mean) * (r[c] - mean);
    var /= (float)C;
    const float inv = 1.0f / sqrtf(var + 1e-6f);
    for (int c = 0; c < C; ++c) r[c] = (r[c] - mean) * inv * scale[c] + shift[c];
  }
}

/* o[r] = b[r] + sum_i W[r][i] * v[i] */
static void gemv(const float* wt, const float* b, const float* v, int rows, int cols, float* o) {
  for (int r = 0; r < rows; ++r) {
    float acc = 0.0f;
    for (int i = 0; i < cols; ++i) acc += wt[(int64_t)r * cols + i] * v[i];
    o[r] = acc + b[r];
  }
}

int oracle_codec_decode(const rwkvtts_codec_dims* d, const float* w, const int64_t* semantic, int T,
                        const int64_t* global, float* pcm) {
  if (!d || !w || !semantic || !global || !pcm || T <= 0) return -1;
  const int L = d->latent_dim, P = d->prenet_dim, I = d->prenet_inter, S = d->spk_dim;
  const int Q = RWKVTTS_CODEC_SPK_LATENT, G = d->n_global, CD = d->codebook_dim;
  for (int t = 0; t < T; ++t)
    if (semantic[t] < 0 || semantic[t] >= d->codebook_size) return -1;
  int n_codes = 1;
  for (int i = 0; i < d->fsq_dims; ++i) n_codes *= d->fsq_levels;
  for (int t = 0; t < G; ++t)
    if (global[t] < 0 || global[t] >= n_codes) return -1;

  /* speaker d-vector: FSQ indices -> codes (level - L/2) / (L/2) -> project_out -> flatten(c, t) */
  float* h = (float*)malloc(sizeof(float) * (size_t)Q * G);
  float* dvec = (float*)malloc(sizeof(float) * S);
  for (int t = 0; t < G; ++t) {
    float code[16];
    int64_t idx = global[t];
    const int half = d->fsq_levels / 2;
    for (int k = 0; k < d->fsq_dims; ++k) {
      code[k] = (float)((int)(idx % d->fsq_levels) - half) / (float)half;
      idx /= d->fsq_levels;
    }
    for (int c = 0; c < Q; ++c) {
      float acc = 0.0f;
      for (int k = 0; k < d->fsq_dims; ++k) acc += W(0, 0, CD_FSQ_W)[c * d->fsq_dims + k] * code[k];
      h[c * G + t] = acc + W(0, 0, CD_FSQ_B)[c];
    }
  }
  gemv(W(0, 0, CD_SPK_W), W(0, 0, CD_SPK_B), h, S, Q * G, dvec);
  free(h);

  /* semantic FVQ: codebook lookup -> 1x1 out_proj */
  float* z = (float*)malloc(sizeof(float) * (size_t)T * L);
  for (int t = 0; t < T; ++t) {
    const float* e = W(0, 0, CD_CODEBOOK) + semantic[t] * CD;
    for (int c = 0; c < L; ++c) {
      float acc = 0.0f;
      for (int k = 0; k < CD; ++k) acc += W(0, 0, CD_OUTP_W)[c * CD + k] * e[k];
      z[(int64_t)t * L + c] = acc + W(0, 0, CD_OUTP_B)[c];
    }
  }

  /* prenet (Vocos backbone, AdaLN on d) */
  float* x = (float*)malloc(sizeof(float) * (size_t)T * P);
  float* u = (float*)malloc(sizeof(float) * (size_t)T * P);
  float* hid = (float*)malloc(sizeof(float) * (size_t)T * I);
  float* sc = (float*)malloc(sizeof(float) * P);
  float* sh = (float*)malloc(sizeof(float) * P);
  conv1d(z, T, L, W(0, 0, CD_PRE_W), W(0, 0, CD_PRE_B), P, 1, 1, 0, NULL, u);
  conv1d(u, T, P, W(0, 0, CD_EMB_W), W(0, 0, CD_EMB_B), P, 7, 1, 3, NULL, x);
  gemv(W(0, 0, CD_N0_SW), W(0, 0, CD_N0_SB), dvec, P, S, sc);
  gemv(W(0, 0, CD_N0_HW), W(0, 0, CD_N0_HB), dvec, P, S, sh);
  layer_norm_rows(x, T, P, sc, sh);
  for (int l = 0; l < d->prenet_layers; ++l) {
    const float* dw = W(1, l, CB_DW_W);
    const float* db = W(1, l, CB_DW_B);
    for (int t = 0; t < T; ++t) /* depthwise conv k7 pad 3 */
      for (int c = 0; c < P; ++c) {
        float acc = 0.0f;
        for (int k = 0; k < 7; ++k) {
          const int p = t + k - 3;
          if (p >= 0 && p < T) acc += dw[c * 7 + k] * x[(int64_t)p * P + c];
        }
        u[(int64_t)t * P + c] = acc + db[c];
      }
    gemv(W(1, l, CB_SW), W(1, l, CB_SB), dvec, P, S, sc);
    gemv(W(1, l, CB_HW), W(1, l, CB_HB), dvec, P, S, sh);
    layer_norm_rows(u, T, P, sc, sh);
    conv1d(u, T, P, W(1, l, CB_PW1_W), W(1, l, CB_PW1_B), I, 1, 1, 0, NULL, hid);
    for (int64_t i = 0; i < (int64_t)T * I; ++i) /* exact GELU */
      hid[i] = 0.5f * hid[i] * (1.0f + erff(hid[i] * 0.70710678118654752f));
    conv1d(hid, T, I, W(1, l, CB_PW2_W), W(1, l, CB_PW2_B), P, 1, 1, 0, NULL, u);
    const float* gm = W(1, l, CB_GAMMA);
    for (int64_t i = 0; i < (int64_t)T * P; ++i) x[i] += gm[i % P] * u[i];
  }
  layer_norm_rows(x, T, P, W(0, 0, CD_FLN_W), W(0, 0, CD_FLN_B));
  float* y = (float*)malloc(sizeof(float) * (size_t)T * L);
  conv1d(x, T, P, W(0, 0, CD_LIN_W), W(0, 0, CD_LIN_B), L, 1, 1, 0, NULL, y);
  for (int64_t i = 0; i < (int64_t)T * L; ++i) y[i] += dvec[i % L]; /* x + d_vector (L == S) */
  free(x); free(u); free(hid); free(sc); free(sh); free(z); free(dvec);

  /* WaveGenerator */
  int C = d->dec_channels, Tc = T;
  float* a = (float*)malloc(sizeof(float) * (size_t)Tc * C);
  conv1d(y, Tc, L, W(0, 0, CD_CIN_W), W(0, 0, CD_CIN_B), C, 7, 1, 3, NULL, a);
  free(y);
  for (int ub = 0; ub < d->n_up; ++ub) {
    const int Co = C / 2, s = d->up_rates[ub], K = d->up_kernels[ub], To = Tc * s;
    float* b = (float*)malloc(sizeof(float) * (size_t)To * Co);
    conv_transpose1d(a, Tc, C, W(2, ub, CU_T_W), W(2, ub, CU_T_B), Co, K, s, W(2, ub, CU_SNAKE), b);
    free(a);
    float* r1 = (float*)malloc(sizeof(float) * (size_t)To * Co);
    float* r2 = (float*)malloc(sizeof(float) * (size_t)To * Co);
    static const int dils[3] = {1, 3, 9};
    for (int r = 0; r < 3; ++r) {
      const int o = r * (CU_R1_A1 - CU_R0_A1);
      conv1d(b, To, Co, W(2, ub, CU_R0_W7 + o), W(2, ub, CU_R0_B7 + o), Co, 7, dils[r], 3 * dils[r],
             W(2, ub, CU_R0_A1 + o), r1);
      conv1d(r1, To, Co, W(2, ub, CU_R0_W1 + o), W(2, ub, CU_R0_B1 + o), Co, 1, 1, 0,
             W(2, ub, CU_R0_A2 + o), r2);
      for (int64_t i = 0; i < (int64_t)To * Co; ++i) b[i] += r2[i];
    }
    free(r1); free(r2);
    a = b; C = Co; Tc = To;
  }
  float* outp = (float*)malloc(sizeof(float) * (size_t)Tc);
  conv1d(a, Tc, C, W(0, 0, CD_COUT_W), W(0, 0, CD_COUT_B), 1, 7, 1, 3, W(0, 0, CD_SOUT_A), outp);
  for (int t = 0; t < Tc; ++t) pcm[t] = tanhf(outp[t]);
  free(outp); free(a);
  return 0;
}
