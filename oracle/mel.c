/* mel.c -- TEST INFRASTRUCTURE (see oracle.h). f32 restatement, in the reference's operation
 * order, of TtsPipelineFixes::extract_mel_spectrogram_consistent (src/tts_pipeline_fixes.rs:12-159):
 * center zero padding, Hann window (2*pi*i/(n_fft-1)), naive DFT magnitude (per bin, angle
 * -2*pi*k*n/n_fft in f32, sequential f32 sums), Slaney-normalised triangular mel filterbank with
 * the HTK-style mel scale 2595*log10(1 + hz/700), no log. f32::cos/sin/log10/powf on Linux are
 * glibc cosf/sinf/log10f/powf, so this file calls exactly those. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define N_MELS 128
#define N_FFT 1024
#define HOP 320
#define N_FREQ (N_FFT / 2 + 1)

/* :114-158 */
static void mel_filterbank(float* fb /* [N_MELS][N_FREQ] */) {
  const float sample_rate = 16000.0f, fmin = 10.0f, fmax = 8000.0f;
  memset(fb, 0, sizeof(float) * N_MELS * N_FREQ);
  const float mel_min = 2595.0f * log10f(1.0f + fmin / 700.0f);
  const float mel_max = 2595.0f * log10f(1.0f + fmax / 700.0f);
  float hz[N_MELS + 2], bin[N_MELS + 2];
  for (int i = 0; i <= N_MELS + 1; ++i) {
    const float mel = mel_min + (float)i * (mel_max - mel_min) / (float)(N_MELS + 1);
    hz[i] = 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f);
    bin[i] = hz[i] * (float)N_FFT / sample_rate;
  }
  for (int m = 1; m <= N_MELS; ++m) {
    const float left = bin[m - 1], center = bin[m], right = bin[m + 1];
    float* row = fb + (m - 1) * N_FREQ;
    for (int k = 0; k < N_FREQ; ++k) {
      const float kf = (float)k;
      if (kf >= left && kf <= right) {
        if (kf <= center) {
          if (center > left) row[k] = (kf - left) / (center - left);
        } else if (right > center) {
          row[k] = (right - kf) / (right - center);
        }
      }
    }
    const float norm = 2.0f / (hz[m + 1] - hz[m - 1]);
    for (int k = 0; k < N_FREQ; ++k) row[k] *= norm;
  }
}

int oracle_mel(const float* wav, int n, float* mel, int* n_frames_out) {
  if (n < 0 || (!wav && n > 0) || !mel || !n_frames_out) return -1;
  const int pad = N_FFT / 2, len = n + 2 * pad;
  float* padded = (float*)calloc((size_t)len, sizeof(float));
  for (int i = 0; i < n; ++i) padded[pad + i] = wav[i];
  const int n_frames = len <= N_FFT ? 1 : (len - N_FFT) / HOP + 1;
  float window[N_FFT];
  for (int i = 0; i < N_FFT; ++i) {
    const float angle = 2.0f * 3.14159265358979323846f * (float)i / (float)(N_FFT - 1);
    window[i] = 0.5f * (1.0f - cosf(angle));
  }
  float* fb = (float*)malloc(sizeof(float) * N_MELS * N_FREQ);
  mel_filterbank(fb);
  /* twiddles of :84-104, computed once (same f32 angle expression, same libm) */
  float* tc = (float*)malloc(sizeof(float) * N_FREQ * N_FFT);
  float* ts = (float*)malloc(sizeof(float) * N_FREQ * N_FFT);
  for (int k = 0; k < N_FREQ; ++k)
    for (int t = 0; t < N_FFT; ++t) {
      const float angle = -2.0f * 3.14159265358979323846f * (float)k * (float)t / (float)N_FFT;
      tc[k * N_FFT + t] = cosf(angle);
      ts[k * N_FFT + t] = sinf(angle);
    }
#pragma omp parallel for schedule(static)
  for (int f = 0; f < n_frames; ++f) {
    float frame[N_FFT], spec[N_FREQ];
    const int start = f * HOP, end = start + N_FFT < len ? start + N_FFT : len;
    for (int i = 0; i < N_FFT; ++i) frame[i] = i < end - start ? padded[start + i] * window[i] : 0.0f;
    for (int k = 0; k < N_FREQ; ++k) {
      float re = 0.0f, im = 0.0f;
      for (int t = 0; t < N_FFT; ++t) {
        re += frame[t] * tc[k * N_FFT + t];
        im += frame[t] * ts[k * N_FFT + t];
      }
      spec[k] = sqrtf(re * re + im * im);
    }
    for (int m = 0; m < N_MELS; ++m) {
      float e = 0.0f;
      for (int k = 0; k < N_FREQ; ++k) e += spec[k] * fb[m * N_FREQ + k];
      mel[(size_t)m * n_frames + f] = e;
    }
  }
  *n_frames_out = n_frames;
  free(padded); free(fb); free(tc); free(ts);
  return 0;
}
