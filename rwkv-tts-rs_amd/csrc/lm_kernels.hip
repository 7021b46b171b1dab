// lm_kernels.hip -- RWKV-7 x070 forward kernels for gfx950 (CDNA4).
//
// One forward step processes R "rows" (tokens) drawn from any number of state slots
// (ragged batch: decode rows are 1 per slot, prefill rows are consecutive per slot). Every
// kernel's per-row result depends only on that row's inputs, the slot's state and fixed
// reduction orders, so a request's outputs are bit-identical whatever else shares the step
// (batch-invariant), and chunking a prompt does not change the arithmetic.
//
// Kernels (per layer): ln_mix(att) -> gemm(r,k,v,LoRA-down) -> wkv -> gemm(Wo) ->
// ln_mix(ffn, + Wo residual) -> gemm(ffn key, relu^2) -> gemm(ffn value) -> [next layer's
// ln_mix adds the ffn residual]. Activations that feed an MFMA are split x = hi + lo into two
// bf16 planes (|lo| <= 2^-9 |x|), so each projection is W(bf16) . x at ~16-bit activation
// precision with f32 accumulation; weights are read exactly once per step.
#include "lm_kernels.h"

namespace rwkvtts {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// deterministic block (256 threads) sum; every thread gets the result
__device__ inline float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__device__ inline void split_store(float x, bf16_t* hi, bf16_t* lo, int64_t idx) {
  const uint16_t h = f32_to_bf16(x);
  const float r = x - bf16_to_f32(h);
  hi[idx] = h;
  lo[idx] = f32_to_bf16(r);
}

// ------------------------------------------------------------------------------------
// embed: h[r] = LN0(emb[token[r]])
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_embed(const uint32_t* tokens, const bf16_t* emb,
                                               const float* w, const float* b, float* h, int C) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  const uint32_t tok = tokens[r];
  const bf16_t* e = emb + (int64_t)tok * C;
  float v[kMaxPerThread];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    v[i] = c < C ? bf16_to_f32(e[c]) : 0.f;
    s += v[i];
  }
  const float mean = block_sum256(s, red) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    const float d = c < C ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(block_sum256(q, red) / (float)C + 1e-5f);
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < C) h[(int64_t)r * C + c] = (v[i] - mean) * rstd * w[c] + b[c];
  }
}

// ------------------------------------------------------------------------------------
// ln_mix: hn = h_in + sum(partials); optionally store hn; xx = LN(hn);
// x_m = xx + (prev - xx) * mu_m (split to bf16 hi/lo); shift state update.
// ------------------------------------------------------------------------------------
__device__ inline void load_residual(const LnMixArgs& a, int src, float* v) {
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    float x = 0.f;
    if (c < a.C) {
      x = a.h_in[(int64_t)src * a.C + c];
      for (int p = 0; p < a.n_part; ++p) x += a.part[p * a.part_stride + (int64_t)src * a.ldp + c];
    }
    v[i] = x;
  }
}

__device__ inline void layer_norm_regs(const LnMixArgs& a, float* v, float* red) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) s += v[i];
  const float mean = block_sum256(s, red) / (float)a.C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    const float d = c < a.C ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(block_sum256(q, red) / (float)a.C + 1e-5f);
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    v[i] = c < a.C ? (v[i] - mean) * rstd * a.ln_w[c] + a.ln_b[c] : 0.f;
  }
}

__global__ __launch_bounds__(256) void k_ln_mix(LnMixArgs a) {
  __shared__ float red[4];
  const int out_row = blockIdx.x;
  const int row = a.row_map ? a.row_map[out_row] : out_row;
  float v[kMaxPerThread];
  load_residual(a, row, v);
  if (a.h_out) {
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < a.C) a.h_out[(int64_t)row * a.C + c] = v[i];
    }
  }
  layer_norm_regs(a, v, red);  // v = xx
  if (!a.shift) {              // ln_out: x = xx
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < a.C) split_store(v[i], a.x_hi, a.x_lo, (int64_t)out_row * a.ldx + c);
    }
    return;
  }
  const int4 info = a.rows[row];  // slot, flags, prev_row, parity
  const int slot = info.x, flags = info.y, prev_row = info.z, par = info.w;
  float pv[kMaxPerThread];
  if (prev_row >= 0) {
    load_residual(a, prev_row, pv);
    layer_norm_regs(a, pv, red);
  } else {
    const float* sh = a.shift + (((int64_t)par * a.S + slot) * a.L + a.layer) * a.C;
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
      const int c = threadIdx.x + i * 256;
      pv[i] = c < a.C ? sh[c] : 0.f;
    }
  }
  for (int m = 0; m < a.n_mix; ++m) {
    const float* mu = a.mu[m];
    bf16_t* hi = a.x_hi + m * a.mix_stride;
    bf16_t* lo = a.x_lo + m * a.mix_stride;
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < a.C) split_store(v[i] + (pv[i] - v[i]) * mu[c], hi, lo, (int64_t)out_row * a.ldx + c);
    }
  }
  if (flags & kRowLast) {
    float* sh = a.shift + (((int64_t)(par ^ 1) * a.S + slot) * a.L + a.layer) * a.C;
#pragma unroll
    for (int i = 0; i < kMaxPerThread; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < a.C) sh[c] = v[i];
    }
  }
}

// ------------------------------------------------------------------------------------
// gemm: out[split][row][col_off + n] = sum_{k in split} X[row][k] * W[n][k]
//   X given as bf16 hi/lo planes; W bf16 [N][K] row-major. MFMA 16x16x32 bf16.
//   Workgroup = 4 waves = 16 output columns x (MT*16) rows x one K slice; the 4 waves split
//   the slice and their accumulators are summed in LDS in fixed order.
//   B fragment (lane l): W[col0 + (l&15)][k0 + 8(l>>4) .. +8]  -> one 16-byte load per lane.
//   A fragment (lane l): X[row0 + (l&15)][k0 + 8(l>>4) .. +8].
// ------------------------------------------------------------------------------------
template <int MT>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs a) {
  __shared__ float red[4 * MT * 4 * 64];
  const int tile = blockIdx.x;
  int s = 0;
  while (s + 1 < a.nseg && tile >= a.seg[s + 1].tile_start) ++s;
  const GemmSeg& sg = a.seg[s];
  const int col0 = (tile - sg.tile_start) * 16;
  const int split = blockIdx.y;
  const int row0 = blockIdx.z * (MT * 16);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int wk = a.kslice >> 2;  // K per wave
  const int kbeg = split * a.kslice + wave * wk;
  int n = col0 + li;
  if (n >= sg.N) n = sg.N - 1;  // clamp (result discarded)
  const bf16_t* wrow = sg.W + (int64_t)n * a.K + kbeg + g * 8;
  const bf16_t* xh[MT];
  const bf16_t* xl[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int64_t ro = (int64_t)(row0 + m * 16 + li) * sg.ldx + kbeg + g * 8;
    xh[m] = sg.Xhi + ro;
    xl[m] = sg.Xlo + ro;
  }
  float4_ acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = (float4_){0.f, 0.f, 0.f, 0.f};
  const int steps = wk >> 5;
  int t = 0;
  for (; t + 4 <= steps; t += 4) {
    short8 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = *(const short8*)(wrow + (t + u) * 32);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const short8 ah = *(const short8*)(xh[m] + (t + u) * 32);
        const short8 al = *(const short8*)(xl[m] + (t + u) * 32);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah),
                                                         __builtin_bit_cast(bf16x8, b[u]), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al),
                                                         __builtin_bit_cast(bf16x8, b[u]), acc[m], 0, 0, 0);
      }
    }
  }
  for (; t < steps; ++t) {
    const short8 b = *(const short8*)(wrow + t * 32);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const short8 ah = *(const short8*)(xh[m] + t * 32);
      const short8 al = *(const short8*)(xl[m] + t * 32);
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah),
                                                       __builtin_bit_cast(bf16x8, b), acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al),
                                                       __builtin_bit_cast(bf16x8, b), acc[m], 0, 0, 0);
    }
  }
  // cross-wave reduction: red[w][m][j][lane]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[((wave * MT + m) * 4 + j) * 64 + lane] = acc[m][j];
  __syncthreads();
  const int j = threadIdx.x >> 6;  // reuse: thread -> (j, lane)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[((w * MT + m) * 4 + j) * 64 + lane];
    const int row = row0 + m * 16 + 4 * g + j;
    const int col = col0 + li;
    if (row < a.M && col < sg.N) {
      if (a.epilogue == kEpiStore) {
        a.out[split * a.split_stride + (int64_t)row * a.ldo + sg.col_off + col] = v;
      } else {  // kEpiRelu2Split
        const float r = v > 0.f ? v : 0.f;
        split_store(r * r, a.out_hi, a.out_lo, (int64_t)row * a.ldo + sg.col_off + col);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// wkv: one workgroup per (slot segment, head); rows of the segment run in order.
//   part columns: [0,C) r | [C,2C) k | [2C,3C) v | [3C, 3C+Dw) w-hidden | +Da a-hidden |
//   +Dv v-hidden | +Dg g-hidden   (split-K partial slabs, summed in fixed order here)
//   Thread t holds S[i = t>>2][16*(t&3) .. +16] of the head's 64x64 state in registers.
// ------------------------------------------------------------------------------------
__device__ inline float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ inline float dot_bf16_row(const bf16_t* w, const float* h, int D) {
  float acc = 0.f;
  for (int d = 0; d < D; d += 8) {
    const short8 q = *(const short8*)(w + d);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += bf16_to_f32((uint16_t)q[e]) * h[d + e];
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_wkv(WkvArgs a) {
  constexpr int N = 64;
  __shared__ float s_hid[kMaxLoraTotal];
  __shared__ float s_r[N], s_k[N], s_v[N], s_w[N], s_kk[N], s_b[N], s_g[N], s_y[N];
  __shared__ float s_lora[4][N];
  __shared__ float red[4];
  const int4 sg = a.segs[blockIdx.x];
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  const int h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = a.C;
  const int i = tid >> 2, jq = (tid & 3) * 16;
  float* Sg = a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N + i * N + jq;
  float S[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4_ v4 = *(const float4_*)(Sg + q * 4);
    S[q * 4 + 0] = v4[0]; S[q * 4 + 1] = v4[1]; S[q * 4 + 2] = v4[2]; S[q * 4 + 3] = v4[3];
  }
  const int Dtot = a.Dw + a.Da + a.Dv + a.Dg;
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    const float* prow = a.part + (int64_t)row * a.ldp;
    // LoRA hidden (whole vectors) with activations
    for (int d = tid; d < Dtot; d += 256) {
      float x = 0.f;
      for (int p = 0; p < a.n_part; ++p) x += prow[p * a.part_stride + 3 * C + d];
      if (d < a.Dw) x = tanhf(x);
      else if (d >= a.Dw + a.Da + a.Dv) x = sigm(x);
      s_hid[d] = x;
    }
    __syncthreads();
    // LoRA up for this head's channels: wave 0: w, 1: a, 2: v, 3: g
    {
      const int c = h * N + lane;
      float acc = 0.f;
      if (wave == 0) acc = dot_bf16_row(a.w2t + (int64_t)c * a.Dw, s_hid, a.Dw);
      else if (wave == 1) acc = dot_bf16_row(a.a2t + (int64_t)c * a.Da, s_hid + a.Dw, a.Da);
      else if (wave == 2) { if (a.layer > 0) acc = dot_bf16_row(a.v2t + (int64_t)c * a.Dv, s_hid + a.Dw + a.Da, a.Dv); }
      else acc = dot_bf16_row(a.g2t + (int64_t)c * a.Dg, s_hid + a.Dw + a.Da + a.Dv, a.Dg);
      s_lora[wave][lane] = acc;
    }
    __syncthreads();
    if (wave == 0) {
      const int c = h * N + lane;
      float r = 0.f, k = 0.f, v = 0.f;
      for (int p = 0; p < a.n_part; ++p) {
        const float* pp = prow + p * a.part_stride;
        r += pp[c];
        k += pp[C + c];
        v += pp[2 * C + c];
      }
      const float w = expf(-0.60653066f * sigm(a.w0[c] + s_lora[0][lane]));
      const float av = sigm(a.a0[c] + s_lora[1][lane]);
      float kk = k * a.k_k[c];
      const float nrm = sqrtf(wave_sum(kk * kk));
      kk = kk / fmaxf(nrm, 1e-12f);
      k = k * (1.0f + (av - 1.0f) * a.k_a[c]);
      float* vf = a.v_first + (int64_t)row * a.ldv + c;
      if (a.layer == 0) {
        *vf = v;
      } else {
        const float gate = sigm(a.v0[c] + s_lora[2][lane]);
        v = v + (*vf - v) * gate;
      }
      s_r[lane] = r; s_k[lane] = k; s_v[lane] = v; s_w[lane] = w;
      s_kk[lane] = kk; s_b[lane] = kk * av; s_g[lane] = s_lora[3][lane];
    }
    __syncthreads();
    // state update: S[i][j] = S[i][j]*w_j - sa_i*b_j + v_i*k_j ; y_i = sum_j S[i][j] r_j
    float sa = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sa += S[q] * s_kk[jq + q];
    sa += __shfl_xor(sa, 1);
    sa += __shfl_xor(sa, 2);
    const float vi = s_v[i];
    float y = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int jj = jq + q;
      S[q] = S[q] * s_w[jj] - sa * s_b[jj] + vi * s_k[jj];
      y += S[q] * s_r[jj];
    }
    y += __shfl_xor(y, 1);
    y += __shfl_xor(y, 2);
    if ((tid & 3) == 0) s_y[i] = y;
    __syncthreads();
    if (wave == 0) {
      const int c = h * N + lane;
      const float yv = s_y[lane];
      const float mean = wave_sum(yv) * (1.0f / N);
      const float dv = yv - mean;
      const float var = wave_sum(dv * dv) * (1.0f / N);
      const float rstd = 1.0f / sqrtf(var + 64e-5f);
      const float bonus = wave_sum(s_r[lane] * s_k[lane] * a.r_k[c]);
      const float gn = dv * rstd * a.lnx_w[c] + a.lnx_b[c];
      split_store((gn + bonus * s_v[lane]) * s_g[lane], a.z_hi, a.z_lo, (int64_t)row * a.ldz + c);
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4_ v4 = {S[q * 4 + 0], S[q * 4 + 1], S[q * 4 + 2], S[q * 4 + 3]};
    *(float4_*)(Sg + q * 4) = v4;
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
void launch_embed(const uint32_t* tokens, const bf16_t* emb, const float* w, const float* b,
                  float* h, int R, int C, hipStream_t st) {
  hipLaunchKernelGGL(k_embed, dim3(R), dim3(256), 0, st, tokens, emb, w, b, h, C);
}
void launch_ln_mix(const LnMixArgs& a, int n_out_rows, hipStream_t st) {
  hipLaunchKernelGGL(k_ln_mix, dim3(n_out_rows), dim3(256), 0, st, a);
}
void launch_gemm(const GemmArgs& a, hipStream_t st) {
  int tiles = a.seg[a.nseg - 1].tile_start + (a.seg[a.nseg - 1].N + 15) / 16;
  const int mt = a.M <= 16 ? 1 : (a.M <= 32 ? 2 : 4);
  const int mg = (a.M + mt * 16 - 1) / (mt * 16);
  dim3 grid(tiles, a.k_split, mg);
  if (mt == 1) hipLaunchKernelGGL(k_gemm<1>, grid, dim3(256), 0, st, a);
  else if (mt == 2) hipLaunchKernelGGL(k_gemm<2>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_gemm<4>, grid, dim3(256), 0, st, a);
}
void launch_wkv(const WkvArgs& a, int n_seg, int H, hipStream_t st) {
  hipLaunchKernelGGL(k_wkv, dim3(n_seg, H), dim3(256), 0, st, a);
}

}  // namespace rwkvtts
