/* rwkv7.c -- TEST INFRASTRUCTURE (see oracle.h).
 * RWKV-7 "x070" single-token forward, f32 activations and state, matrices from the packed
 * 2-byte blob (include/rwkvtts.h layout). This is the arithmetic web-rwkv 0.10.16's
 * v7::Bundle<f32> runs for every Runtime<Rnn>::infer token (call sites
 * src/normal_mode_inference.rs:75,228,308,324; src/zero_shot_inference.rs:113,228),
 * restated from the published RWKV-7 formulation:
 *   x = LN0(emb[tok]);  per layer:
 *   xx = LN1(x); d = shift - xx; x_* = xx + d*mu_*; shift = xx
 *   r = Wr x_r; k = Wk x_k; v = Wv x_v
 *   w = exp(-e^{-1/2} sigmoid(w0 + W2 tanh(W1 x_w)));  a = sigmoid(a0 + A2 A1 x_a)
 *   g = G2 sigmoid(G1 x_g);  kk = normalize_head(k*k_k);  k = k*(1 + (a-1)*k_a)
 *   v = layer0 ? (v_first = v) : v + (v_first - v)*sigmoid(v0 + V2 V1 x_v)
 *   S = S diag(w) - (S kk)(kk*a)^T + v k^T;  y = S r        (S[i=value][j=key])
 *   y = GroupNorm_H(y, eps 64e-5) + (sum_head r*k*r_k) v;  x += Wo (y*g)
 *   xx = LN2(x); kx = xx + (shift' - xx)*mu_k; shift' = xx;  x += Wv relu(Wk kx)^2
 *   logits = Head LN_out(x)
 * Matrix-vector products accumulate in f32 in natural index order. */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle.h"

struct oracle_model {
  rwkvtts_dims d;
  int dtype;
  uint8_t* blob;
  size_t bytes;
  float** qf; /* [n_layer][6] dequantised r, k, v, o, ffn key, ffn value (NULL: 16-bit) */
};

static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline float f16_to_f32(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023, u;
  if (e == 0) {
    if (m == 0) u = s;
    else { /* subnormal */
      int sh = 0;
      while (!(m & 1024)) { m <<= 1; ++sh; }
      m &= 1023;
      u = s | ((uint32_t)(127 - 15 - sh + 1) << 23) | (m << 13);
    }
  } else if (e == 31) u = s | 0x7f800000u | (m << 13);
  else u = s | ((e + 112) << 23) | (m << 13);
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static const void* T(const oracle_model* m, int layer, int t) {
  return m->blob + rwkvtts_tensor_offset(&m->d, layer, t);
}
static const float* V(const oracle_model* m, int layer, int t) {
  return (const float*)T(m, layer, t);
}
static inline float mat_at(const oracle_model* m, const uint16_t* w, int64_t i) {
  return m->dtype == RWKVTTS_DTYPE_BF16 ? bf16_to_f32(w[i]) : f16_to_f32(w[i]);
}

static int g_threads = 0;
void oracle_set_threads(int n) { g_threads = n; }

/* ---- quantised matrices: web-rwkv 0.10.16 Quant::{Int8, NF4} (ModelBuilder::quant, set from the
 * server's --quant-layers / --quant-type, bin/server.rs:1029-1071). The crate is not vendored,
 * so this restates its published block quantisers (parity unpinned):
 *   Int8: blocks of 128 consecutive elements of a row (along K); mn = f16(min), mx = f16(max);
 *     q = floor(fma(clamp((x - mn) / (mx - mn), 0, 1), 255, 0.5)) (0 when mx == mn);
 *     w = fma(q, (mx - mn) / 255, mn)               (min + unpack4x8unorm(q) * (max - min))
 *   NF4: blocks of 64; s = f16(max |x|); q = #{i < 15 : x / s > (t[i] + t[i+1]) / 2}
 *     (7 when s == 0); w = t[q] * s, t = the NormalFloat-4 table.
 * f16(.) is round-to-nearest-even. */
static uint16_t f32_to_f16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(sign | (a > 0x7f800000u ? 0x7e00u : 0x7c00u));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520: inf */
  if (a < 0x38800000u) {                                     /* f16 subnormal or zero */
    const int e = (int)(a >> 23);
    if (e < 102) return (uint16_t)sign;
    const uint32_t m = (a & 0x7fffffu) | 0x800000u;
    const int sh = 126 - e; /* value = m * 2^(e - 150); f16 unit 2^-24 */
    uint32_t q = m >> sh, r = m & ((1u << sh) - 1u), half = 1u << (sh - 1);
    if (r > half || (r == half && (q & 1u))) ++q;
    return (uint16_t)(sign | q);
  }
  uint32_t q = ((a >> 13) - (112u << 10)), r = a & 0x1fffu;
  if (r > 0x1000u || (r == 0x1000u && (q & 1u))) ++q;
  return (uint16_t)(sign | q);
}
static const float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
    -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
    0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

/* dequantised copy of a [N][K] matrix (2-byte blob storage) */
static float* quant_matrix(const oracle_model* m, const uint16_t* W, int N, int K, int qt) {
  float* out = (float*)malloc((size_t)N * K * sizeof(float));
  const int BS = qt == 1 ? 128 : 64;
  for (int n = 0; n < N; ++n)
    for (int k0 = 0; k0 < K; k0 += BS) {
      const uint16_t* src = W + (size_t)n * K + k0;
      float* dst = out + (size_t)n * K + k0;
      if (qt == 1) {
        float lo = mat_at(m, src, 0), hi = lo;
        for (int i = 1; i < BS; ++i) {
          const float x = mat_at(m, src, i);
          lo = fminf(lo, x);
          hi = fmaxf(hi, x);
        }
        const float mn = f16_to_f32(f32_to_f16_rne(lo)), mx = f16_to_f32(f32_to_f16_rne(hi)), d = mx - mn;
        for (int i = 0; i < BS; ++i) {
          unsigned q = 0;
          if (mx != mn) {
            float v = (mat_at(m, src, i) - mn) / d;
            v = fminf(fmaxf(v, 0.0f), 1.0f);
            q = (unsigned)floorf(fmaf(v, 255.0f, 0.5f));
          }
          dst[i] = fmaf((float)q, d / 255.0f, mn);
        }
      } else {
        float am = 0.0f;
        for (int i = 0; i < BS; ++i) am = fmaxf(am, fabsf(mat_at(m, src, i)));
        const float sc = f16_to_f32(f32_to_f16_rne(am));
        for (int i = 0; i < BS; ++i) {
          unsigned q = 7;
          if (sc != 0.0f) {
            const float v = mat_at(m, src, i) / sc;
            q = 0;
            for (int t = 0; t < 15; ++t) q += v > 0.5f * (kNF4[t] + kNF4[t + 1]) ? 1u : 0u;
          }
          dst[i] = kNF4[q] * sc;
        }
      }
    }
  return out;
}

static const int kQuantT[6] = {RWKVTTS_L_WR, RWKVTTS_L_WK, RWKVTTS_L_WV, RWKVTTS_L_WO, RWKVTTS_L_FFN_K,
                               RWKVTTS_L_FFN_V};

int oracle_model_quantize(oracle_model* m, int quant_layers, int quant_type) {
  if (quant_type < 0 || quant_type > 2 || quant_layers < 0) return -1;
  if (quant_type == 0 || quant_layers == 0) return 0;
  const int L = m->d.n_layer, C = m->d.n_embd, F = m->d.n_ffn;
  if (C % 128 || F % 128) return -1;
  if (!m->qf) m->qf = (float**)calloc((size_t)L * 6, sizeof(float*));
  for (int l = 0; l < L && l < quant_layers; ++l)
    for (int j = 0; j < 6; ++j) {
      const int N = j == 4 ? F : C, K = j == 5 ? F : C;
      free(m->qf[l * 6 + j]);
      m->qf[l * 6 + j] = quant_matrix(m, (const uint16_t*)T(m, l, kQuantT[j]), N, K, quant_type);
    }
  return 0;
}

/* y[rows] = W[rows][cols] x[cols] */
static void matvec(const oracle_model* m, const void* W, int rows, int cols, const float* x,
                   float* y) {
  const uint16_t* w = (const uint16_t*)W;
#ifdef _OPENMP
  int nt = g_threads > 0 ? g_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt) if ((int64_t)rows * cols >= (1 << 18))
#endif
  for (int r = 0; r < rows; ++r) {
    const uint16_t* row = w + (int64_t)r * cols;
    float acc = 0.0f;
    if (m->dtype == RWKVTTS_DTYPE_BF16)
      for (int c = 0; c < cols; ++c) acc += bf16_to_f32(row[c]) * x[c];
    else
      for (int c = 0; c < cols; ++c) acc += f16_to_f32(row[c]) * x[c];
    y[r] = acc;
  }
}

/* matrix t of layer l: the dequantised copy when the layer is quantised */
static void matvec_l(const oracle_model* m, int l, int t, int rows, int cols, const float* x, float* y) {
  const float* q = NULL;
  if (m->qf)
    for (int j = 0; j < 6; ++j)
      if (kQuantT[j] == t) q = m->qf[l * 6 + j];
  if (!q) {
    matvec(m, T(m, l, t), rows, cols, x, y);
    return;
  }
#ifdef _OPENMP
  int nt = g_threads > 0 ? g_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt) if ((int64_t)rows * cols >= (1 << 18))
#endif
  for (int r = 0; r < rows; ++r) {
    const float* row = q + (int64_t)r * cols;
    float acc = 0.0f;
    for (int c = 0; c < cols; ++c) acc += row[c] * x[c];
    y[r] = acc;
  }
}

static void layer_norm(const float* x, int n, const float* w, const float* b, float eps,
                       float* out) {
  float mean = 0.0f;
  for (int i = 0; i < n; ++i) mean += x[i];
  mean /= (float)n;
  float var = 0.0f;
  for (int i = 0; i < n; ++i) {
    float dv = x[i] - mean;
    var += dv * dv;
  }
  var /= (float)n;
  float rstd = 1.0f / sqrtf(var + eps);
  for (int i = 0; i < n; ++i) out[i] = (x[i] - mean) * rstd * w[i] + b[i];
}

static inline float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

oracle_model* oracle_model_load(const void* blob, size_t bytes) {
  const rwkvtts_blob_header* h = (const rwkvtts_blob_header*)blob;
  if (bytes < 256 || h->magic != RWKVTTS_BLOB_MAGIC) return NULL;
  if ((size_t)rwkvtts_blob_bytes(&h->dims) > bytes) return NULL;
  oracle_model* m = (oracle_model*)calloc(1, sizeof(*m));
  m->d = h->dims;
  m->dtype = h->dtype;
  m->bytes = bytes;
  m->blob = (uint8_t*)malloc(bytes);
  memcpy(m->blob, blob, bytes);
  return m;
}

void oracle_model_free(oracle_model* m) {
  if (!m) return;
  if (m->qf) {
    for (int i = 0; i < m->d.n_layer * 6; ++i) free(m->qf[i]);
    free(m->qf);
  }
  free(m->blob);
  free(m);
}

int64_t oracle_state_floats(const oracle_model* m) {
  const int64_t C = m->d.n_embd, N = m->d.head_size, H = C / N;
  return (int64_t)m->d.n_layer * (2 * C + H * N * N);
}

void oracle_forward_token(const oracle_model* m, float* state, uint32_t token, float* logits,
                          int head_rows) {
  const rwkvtts_dims* d = &m->d;
  const int C = d->n_embd, N = d->head_size, H = C / N, F = d->n_ffn;
  const int Dw = d->d_decay, Da = d->d_aaa, Dv = d->d_mv, Dg = d->d_gate;
  const int64_t per_layer = 2 * (int64_t)C + (int64_t)H * N * N;
  const float decay_scale = 0.60653066f; /* e^{-1/2} */

  float* x = (float*)malloc(sizeof(float) * C);
  float* xx = (float*)malloc(sizeof(float) * C);
  float* mix[6];
  for (int i = 0; i < 6; ++i) mix[i] = (float*)malloc(sizeof(float) * C);
  float *r = malloc(sizeof(float) * C), *k = malloc(sizeof(float) * C),
        *v = malloc(sizeof(float) * C), *w = malloc(sizeof(float) * C),
        *a = malloc(sizeof(float) * C), *g = malloc(sizeof(float) * C),
        *kk = malloc(sizeof(float) * C), *y = malloc(sizeof(float) * C),
        *tmp = malloc(sizeof(float) * C), *vfirst = malloc(sizeof(float) * C);
  float* hid = (float*)malloc(sizeof(float) * 512);
  float* hid2 = (float*)malloc(sizeof(float) * 512);
  float* kf = (float*)malloc(sizeof(float) * F);

  /* embedding + ln0 */
  {
    const uint16_t* emb = (const uint16_t*)T(m, -1, RWKVTTS_T_EMB);
    for (int c = 0; c < C; ++c) tmp[c] = mat_at(m, emb, (int64_t)token * C + c);
    layer_norm(tmp, C, V(m, -1, RWKVTTS_T_LN0_W), V(m, -1, RWKVTTS_T_LN0_B), 1e-5f, x);
  }

  for (int l = 0; l < d->n_layer; ++l) {
    float* st = state + (int64_t)l * per_layer;
    float* att_shift = st;
    float* S = st + C;
    float* ffn_shift = st + C + (int64_t)H * N * N;

    /* ---- time mix ---- */
    layer_norm(x, C, V(m, l, RWKVTTS_L_LN1_W), V(m, l, RWKVTTS_L_LN1_B), 1e-5f, xx);
    static const int mu_idx[6] = {RWKVTTS_L_XR, RWKVTTS_L_XW, RWKVTTS_L_XK,
                                  RWKVTTS_L_XV, RWKVTTS_L_XA, RWKVTTS_L_XG};
    for (int i = 0; i < 6; ++i) {
      const float* mu = V(m, l, mu_idx[i]);
      for (int c = 0; c < C; ++c) mix[i][c] = xx[c] + (att_shift[c] - xx[c]) * mu[c];
    }
    memcpy(att_shift, xx, sizeof(float) * C);
    float *xr = mix[0], *xw = mix[1], *xk = mix[2], *xv = mix[3], *xa = mix[4], *xg = mix[5];

    matvec_l(m, l, RWKVTTS_L_WR, C, C, xr, r);
    matvec_l(m, l, RWKVTTS_L_WK, C, C, xk, k);
    matvec_l(m, l, RWKVTTS_L_WV, C, C, xv, v);

    /* w = exp(-e^-0.5 * sigmoid(w0 + W2 tanh(W1 xw))) */
    matvec(m, T(m, l, RWKVTTS_L_W1T), Dw, C, xw, hid);
    for (int i = 0; i < Dw; ++i) hid[i] = tanhf(hid[i]);
    matvec(m, T(m, l, RWKVTTS_L_W2T), C, Dw, hid, w);
    {
      const float* w0 = V(m, l, RWKVTTS_L_W0);
      for (int c = 0; c < C; ++c) w[c] = expf(-decay_scale * sigmoidf_(w0[c] + w[c]));
    }
    /* a = sigmoid(a0 + A2 A1 xa) */
    matvec(m, T(m, l, RWKVTTS_L_A1T), Da, C, xa, hid);
    matvec(m, T(m, l, RWKVTTS_L_A2T), C, Da, hid, a);
    {
      const float* a0 = V(m, l, RWKVTTS_L_A0);
      for (int c = 0; c < C; ++c) a[c] = sigmoidf_(a0[c] + a[c]);
    }
    /* g = G2 sigmoid(G1 xg) */
    matvec(m, T(m, l, RWKVTTS_L_G1T), Dg, C, xg, hid);
    for (int i = 0; i < Dg; ++i) hid[i] = sigmoidf_(hid[i]);
    matvec(m, T(m, l, RWKVTTS_L_G2T), C, Dg, hid, g);

    /* kk = normalize_head(k * k_k); k = k * (1 + (a - 1) * k_a) */
    {
      const float* k_k = V(m, l, RWKVTTS_L_KK);
      const float* k_a = V(m, l, RWKVTTS_L_KA);
      for (int c = 0; c < C; ++c) kk[c] = k[c] * k_k[c];
      for (int h = 0; h < H; ++h) {
        float ss = 0.0f;
        for (int j = 0; j < N; ++j) ss += kk[h * N + j] * kk[h * N + j];
        float nrm = sqrtf(ss);
        if (nrm < 1e-12f) nrm = 1e-12f;
        for (int j = 0; j < N; ++j) kk[h * N + j] /= nrm;
      }
      for (int c = 0; c < C; ++c) k[c] = k[c] * (1.0f + (a[c] - 1.0f) * k_a[c]);
    }
    /* value residual */
    if (l == 0) {
      memcpy(vfirst, v, sizeof(float) * C);
    } else {
      matvec(m, T(m, l, RWKVTTS_L_V1T), Dv, C, xv, hid);
      matvec(m, T(m, l, RWKVTTS_L_V2T), C, Dv, hid, tmp);
      const float* v0 = V(m, l, RWKVTTS_L_V0);
      for (int c = 0; c < C; ++c) {
        float gate = sigmoidf_(v0[c] + tmp[c]);
        v[c] = v[c] + (vfirst[c] - v[c]) * gate;
      }
    }
    /* WKV-7 state update per head */
    for (int h = 0; h < H; ++h) {
      float* Sh = S + (int64_t)h * N * N;
      const float *kkh = kk + h * N, *ah = a + h * N, *wh = w + h * N, *kh = k + h * N,
                  *vh = v + h * N, *rh = r + h * N;
      for (int i = 0; i < N; ++i) {
        float* Si = Sh + (int64_t)i * N;
        float sa = 0.0f;
        for (int j = 0; j < N; ++j) sa += Si[j] * kkh[j];
        float yi = 0.0f;
        for (int j = 0; j < N; ++j) {
          float sn = Si[j] * wh[j] - sa * (kkh[j] * ah[j]) + vh[i] * kh[j];
          Si[j] = sn;
          yi += sn * rh[j];
        }
        y[h * N + i] = yi;
      }
    }
    /* GroupNorm(H groups, eps 64e-5) + bonus, gate */
    {
      const float* lw = V(m, l, RWKVTTS_L_LNX_W);
      const float* lb = V(m, l, RWKVTTS_L_LNX_B);
      const float* rk = V(m, l, RWKVTTS_L_RK);
      for (int h = 0; h < H; ++h) {
        float* yh = y + h * N;
        float mean = 0.0f;
        for (int j = 0; j < N; ++j) mean += yh[j];
        mean /= (float)N;
        float var = 0.0f;
        for (int j = 0; j < N; ++j) {
          float dv = yh[j] - mean;
          var += dv * dv;
        }
        var /= (float)N;
        float rstd = 1.0f / sqrtf(var + 64e-5f);
        float bonus = 0.0f;
        for (int j = 0; j < N; ++j) bonus += r[h * N + j] * k[h * N + j] * rk[h * N + j];
        for (int j = 0; j < N; ++j) {
          int c = h * N + j;
          float gn = (yh[j] - mean) * rstd * lw[c] + lb[c];
          tmp[c] = (gn + bonus * v[c]) * g[c];
        }
      }
    }
    matvec_l(m, l, RWKVTTS_L_WO, C, C, tmp, y);
    for (int c = 0; c < C; ++c) x[c] += y[c];

    /* ---- channel mix ---- */
    layer_norm(x, C, V(m, l, RWKVTTS_L_LN2_W), V(m, l, RWKVTTS_L_LN2_B), 1e-5f, xx);
    {
      const float* mu = V(m, l, RWKVTTS_L_FFN_XK);
      for (int c = 0; c < C; ++c) tmp[c] = xx[c] + (ffn_shift[c] - xx[c]) * mu[c];
    }
    memcpy(ffn_shift, xx, sizeof(float) * C);
    matvec_l(m, l, RWKVTTS_L_FFN_K, F, C, tmp, kf);
    for (int i = 0; i < F; ++i) {
      float t = kf[i] > 0.0f ? kf[i] : 0.0f;
      kf[i] = t * t;
    }
    matvec_l(m, l, RWKVTTS_L_FFN_V, C, F, kf, y);
    for (int c = 0; c < C; ++c) x[c] += y[c];
  }

  if (logits && head_rows > 0) {
    layer_norm(x, C, V(m, -1, RWKVTTS_T_LNOUT_W), V(m, -1, RWKVTTS_T_LNOUT_B), 1e-5f, xx);
    matvec(m, T(m, -1, RWKVTTS_T_HEAD), head_rows, C, xx, logits);
  }

  free(x); free(xx);
  for (int i = 0; i < 6; ++i) free(mix[i]);
  free(r); free(k); free(v); free(w); free(a); free(g); free(kk); free(y); free(tmp);
  free(vfirst); free(hid); free(hid2); free(kf);
}
