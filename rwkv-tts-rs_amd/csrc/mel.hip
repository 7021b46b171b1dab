// mel.hip -- zero-shot reference-audio mel spectrogram on the MI355X, replacing
// TtsPipelineFixes::extract_mel_spectrogram_consistent (src/tts_pipeline_fixes.rs:12-159).
//
// The reference computes, in f32: center zero padding (n_fft/2 each side), a Hann window with
// angle 2*pi*i/(n_fft-1), a *naive* DFT per bin k (twiddle angle -2*pi*k*n/n_fft evaluated in
// f32, then f32::cos/sin = glibc cosf/sinf) with sequential f32 sums, the magnitude
// sqrt(re^2 + im^2), and a Slaney-normalised triangular mel filterbank (128 x 513), no log.
// Bit-exact reproduction: the window, twiddle table and filterbank are computed once on the host
// with the same glibc calls and the same f32 expression order, and the device sums every
// product in the reference's order with non-contracted multiply/add (__fmul_rn/__fadd_rn).
// Work: one thread per (bin k, frame) runs the 1024-term dot products against the twiddle
// column (coalesced across k); 16 frames of windowed samples are staged in LDS per workgroup.
#include <math.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "common.h"

namespace rwkvtts {

constexpr int kMels = 128, kFft = 1024, kHop = 320, kFreq = kFft / 2 + 1, kFrameTile = 16;

// frames: [n_frames][kFft] windowed; tw: [kFft][2*kFreq] (cos, sin interleaved per n row)
__global__ __launch_bounds__(128) void k_dft_mag(const float* wav, int n, const float* window, const float2* tw,
                                                 int n_frames, float* mag /* [n_frames][kFreq] */) {
  __shared__ float s_fr[kFrameTile][kFft];
  const int f0 = blockIdx.y * kFrameTile, k = blockIdx.x * 128 + threadIdx.x;
  const int pad = kFft / 2, len = n + 2 * pad;
  for (int i = threadIdx.x; i < kFrameTile * kFft; i += 128) {
    const int fi = i / kFft, t = i % kFft, f = f0 + fi;
    float v = 0.0f;
    if (f < n_frames) {
      const int p = f * kHop + t;                  // index into the padded signal
      const int src = p - pad;                     // zero outside [0, n)
      const float x = (p < len && src >= 0 && src < n) ? wav[src] : 0.0f;
      v = __fmul_rn(x, window[t]);
    }
    s_fr[fi][t] = v;
  }
  __syncthreads();
  if (k >= kFreq) return;
  float re[kFrameTile], im[kFrameTile];
#pragma unroll
  for (int j = 0; j < kFrameTile; ++j) re[j] = im[j] = 0.0f;
  for (int t = 0; t < kFft; ++t) {
    const float2 cs = tw[(int64_t)t * kFreq + k];
#pragma unroll
    for (int j = 0; j < kFrameTile; ++j) {
      re[j] = __fadd_rn(re[j], __fmul_rn(s_fr[j][t], cs.x));
      im[j] = __fadd_rn(im[j], __fmul_rn(s_fr[j][t], cs.y));
    }
  }
#pragma unroll
  for (int j = 0; j < kFrameTile; ++j)
    if (f0 + j < n_frames)
      // correctly rounded f32 sqrt (v_sqrt_f32 alone is not): via the correctly rounded double
      // sqrt, whose rounding to f32 is exact-safe (53 >= 2*24 + 2)
      mag[(int64_t)(f0 + j) * kFreq + k] =
          (float)__dsqrt_rn((double)__fadd_rn(__fmul_rn(re[j], re[j]), __fmul_rn(im[j], im[j])));
}

// mel[m][f] = sum_k mag[f][k] * fb[m][k], k in order
__global__ __launch_bounds__(128) void k_mel_apply(const float* mag, const float* fb, int n_frames, float* mel) {
  const int m = threadIdx.x, f = blockIdx.x;
  if (m >= kMels || f >= n_frames) return;
  const float* sp = mag + (int64_t)f * kFreq;
  const float* w = fb + m * kFreq;
  float e = 0.0f;
  for (int k = 0; k < kFreq; ++k) e = __fadd_rn(e, __fmul_rn(sp[k], w[k]));
  mel[(int64_t)m * n_frames + f] = e;
}

// Host tables, built once per device with the reference's f32 expressions and glibc calls.
struct MelTables {
  float* window = nullptr;
  float2* tw = nullptr;
  float* fb = nullptr;
};

static void host_tables(std::vector<float>& win, std::vector<float2>& tw, std::vector<float>& fb) {
  const float pi = 3.14159265358979323846f;  // std::f32::consts::PI
  win.resize(kFft);
  for (int i = 0; i < kFft; ++i) {
    const float angle = 2.0f * pi * (float)i / (float)(kFft - 1);
    win[i] = 0.5f * (1.0f - cosf(angle));
  }
  tw.resize((size_t)kFft * kFreq);
  for (int k = 0; k < kFreq; ++k)
    for (int t = 0; t < kFft; ++t) {
      const float angle = -2.0f * pi * (float)k * (float)t / (float)kFft;
      tw[(size_t)t * kFreq + k] = make_float2(cosf(angle), sinf(angle));
    }
  fb.assign((size_t)kMels * kFreq, 0.0f);
  const float sr = 16000.0f, fmin = 10.0f, fmax = 8000.0f;
  const float mel_min = 2595.0f * log10f(1.0f + fmin / 700.0f);
  const float mel_max = 2595.0f * log10f(1.0f + fmax / 700.0f);
  float hz[kMels + 2], bin[kMels + 2];
  for (int i = 0; i <= kMels + 1; ++i) {
    const float mel = mel_min + (float)i * (mel_max - mel_min) / (float)(kMels + 1);
    hz[i] = 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f);
    bin[i] = hz[i] * (float)kFft / sr;
  }
  for (int m = 1; m <= kMels; ++m) {
    const float left = bin[m - 1], center = bin[m], right = bin[m + 1];
    float* row = fb.data() + (size_t)(m - 1) * kFreq;
    for (int k = 0; k < kFreq; ++k) {
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
    for (int k = 0; k < kFreq; ++k) row[k] *= norm;
  }
}

static int get_tables(int device, MelTables** out) {
  static std::mutex mu;
  static std::vector<MelTables> per_dev;
  std::lock_guard<std::mutex> lock(mu);
  if ((int)per_dev.size() <= device) per_dev.resize(device + 1);
  MelTables& t = per_dev[device];
  if (!t.window) {
    std::vector<float> win, fb;
    std::vector<float2> tw;
    host_tables(win, tw, fb);
    RT_HIP(hipMalloc(&t.window, win.size() * sizeof(float)));
    RT_HIP(hipMalloc(&t.tw, tw.size() * sizeof(float2)));
    RT_HIP(hipMalloc(&t.fb, fb.size() * sizeof(float)));
    RT_HIP(hipMemcpy(t.window, win.data(), win.size() * sizeof(float), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(t.tw, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice));
    RT_HIP(hipMemcpy(t.fb, fb.data(), fb.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  *out = &t;
  return RWKVTTS_OK;
}

}  // namespace rwkvtts

using namespace rwkvtts;

extern "C" int rwkvtts_mel(int device, const float* wav, int n, float* mel, int* n_frames) {
  RT_CHECK(n >= 0 && (wav || n == 0) && mel && n_frames, RWKVTTS_EINVAL, "mel: bad arguments");
  RT_HIP(hipSetDevice(device));
  MelTables* t = nullptr;
  int rc = get_tables(device, &t);
  if (rc) return rc;
  const int len = n + kFft;
  const int nf = len <= kFft ? 1 : (len - kFft) / kHop + 1;
  float *d_wav = nullptr, *d_mag = nullptr, *d_mel = nullptr;
  RT_HIP(hipMalloc(&d_wav, (size_t)std::max(n, 1) * sizeof(float)));
  RT_HIP(hipMalloc(&d_mag, (size_t)nf * kFreq * sizeof(float)));
  RT_HIP(hipMalloc(&d_mel, (size_t)nf * kMels * sizeof(float)));
  if (n > 0) RT_HIP(hipMemcpy(d_wav, wav, (size_t)n * sizeof(float), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_dft_mag, dim3((kFreq + 127) / 128, (nf + kFrameTile - 1) / kFrameTile), dim3(128), 0, 0,
                     d_wav, n, t->window, t->tw, nf, d_mag);
  hipLaunchKernelGGL(k_mel_apply, dim3(nf), dim3(128), 0, 0, d_mag, t->fb, nf, d_mel);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(mel, d_mel, (size_t)nf * kMels * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(d_wav);
  (void)hipFree(d_mag);
  (void)hipFree(d_mel);
  RT_HIP(e);
  *n_frames = nf;
  return RWKVTTS_OK;
}
