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
// ln_mix: one workgroup per row, thread t owns the 4 columns [4t, 4t+4) (x kLnVec chunks of
// 1024 columns). hn = h_in + sum(partials) (fixed order); optionally store hn; xx = LN(hn);
// x_m = xx + (prev - xx) * mu_m (split to bf16 hi/lo); shift state update. Latency-bound:
// every independent load (partials unrolled 4-wide) is issued before the first reduction.
// ------------------------------------------------------------------------------------
__device__ inline float4_ ld4(const float* p) { return *(const float4_*)p; }

template <int kLnVec>
__device__ inline void ln_load_row(const LnMixArgs& a, int src, float4_* v) {
  const int t4 = 4 * threadIdx.x;
#pragma unroll
  for (int q = 0; q < kLnVec; ++q) {
    const int c = t4 + 1024 * q;
    v[q] = c < a.C ? ld4(a.h_in + (int64_t)src * a.C + c) : (float4_){0.f, 0.f, 0.f, 0.f};
  }
  int p = 0;
  for (; p + 4 <= a.n_part; p += 4) {
    const float* pp = a.part + p * a.part_stride + (int64_t)src * a.ldp;
    float4_ t[4][kLnVec];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < kLnVec; ++q) {
        const int c = t4 + 1024 * q;
        t[u][q] = c < a.C ? ld4(pp + u * a.part_stride + c) : (float4_){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < kLnVec; ++q) v[q] += t[u][q];
  }
  for (; p < a.n_part; ++p) {
    const float* pp = a.part + p * a.part_stride + (int64_t)src * a.ldp;
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) v[q] += ld4(pp + c);
    }
  }
}

// block (256) sum with one barrier: wave shuffles, then 4 partials through LDS slot `slot`
__device__ inline float block_sum_1b(float v, float* red, int slot) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[slot * 4 + (threadIdx.x >> 6)] = v;
  __syncthreads();
  return (red[slot * 4 + 0] + red[slot * 4 + 1]) + (red[slot * 4 + 2] + red[slot * 4 + 3]);
}

template <int kLnVec>
__device__ inline void ln_apply(const LnMixArgs& a, const float4_* w, const float4_* b, float4_* v,
                                float* red, int slot) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < kLnVec; ++q) s += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
  const float mean = block_sum_1b(s, red, slot) / (float)a.C;
  float qs = 0.f;
  const int t4 = 4 * threadIdx.x;
#pragma unroll
  for (int q = 0; q < kLnVec; ++q)
    if (t4 + 1024 * q < a.C)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[q][e] - mean;
        qs += d * d;
      }
  const float rstd = 1.0f / sqrtf(block_sum_1b(qs, red, slot + 1) / (float)a.C + 1e-5f);
#pragma unroll
  for (int q = 0; q < kLnVec; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[q][e] = (v[q][e] - mean) * rstd * w[q][e] + b[q][e];
}

__device__ inline void store_split4(const float4_& x, bf16_t* hi, bf16_t* lo, int64_t idx) {
  uint16_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = f32_to_bf16(x[e]);
    l[e] = f32_to_bf16(x[e] - bf16_to_f32(h[e]));
  }
  *(uint2*)(hi + idx) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
  *(uint2*)(lo + idx) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
}

template <int kLnVec>  // C <= 1024 * kLnVec
__global__ __launch_bounds__(256) void k_ln_mix(LnMixArgs a) {
  __shared__ float red[16];
  const int out_row = blockIdx.x;
  const int row = a.row_map ? a.row_map[out_row] : out_row;
  const int t4 = 4 * threadIdx.x;
  const float4_ z = {0.f, 0.f, 0.f, 0.f};
  float4_ v[kLnVec], w[kLnVec], b[kLnVec], pv[kLnVec], mu[6][kLnVec];
  int slot = 0, flags = 0, prev_row = -1, par = 0;
  if (a.shift) {
    const int4 info = a.rows[row];
    slot = info.x; flags = info.y; prev_row = info.z; par = info.w;
  }
  const float* sh = a.shift ? a.shift + (((int64_t)par * a.S + slot) * a.L + a.layer) * a.C : nullptr;
#pragma unroll
  for (int q = 0; q < kLnVec; ++q) {
    const int c = t4 + 1024 * q;
    const bool ok = c < a.C;
    w[q] = ok ? ld4(a.ln_w + c) : z;
    b[q] = ok ? ld4(a.ln_b + c) : z;
    pv[q] = (ok && sh && prev_row < 0) ? ld4(sh + c) : z;
#pragma unroll
    for (int m = 0; m < 6; ++m) mu[m][q] = (ok && m < a.n_mix && a.mu[m]) ? ld4(a.mu[m] + c) : z;
  }
  ln_load_row<kLnVec>(a, row, v);
  if (a.h_out) {
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) *(float4_*)(a.h_out + (int64_t)row * a.C + c) = v[q];
    }
  }
  ln_apply<kLnVec>(a, w, b, v, red, 0);  // v = xx
  if (!a.shift) {                        // ln_out: x = xx
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) store_split4(v[q], a.x_hi, a.x_lo, (int64_t)out_row * a.ldx + c);
    }
    return;
  }
  if (prev_row >= 0) {  // prefill row: the previous token's LN output, recomputed identically
    ln_load_row<kLnVec>(a, prev_row, pv);
    ln_apply<kLnVec>(a, w, b, pv, red, 2);
  }
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    if (m >= a.n_mix) break;
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) {
        float4_ x;
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = v[q][e] + (pv[q][e] - v[q][e]) * mu[m][q][e];
        store_split4(x, a.x_hi + m * a.mix_stride, a.x_lo + m * a.mix_stride, (int64_t)out_row * a.ldx + c);
      }
    }
  }
  if (flags & kRowLast) {
    float* sn = a.shift + (((int64_t)(par ^ 1) * a.S + slot) * a.L + a.layer) * a.C;
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) *(float4_*)(sn + c) = v[q];
    }
  }
}

// ------------------------------------------------------------------------------------
// gemm: out[split][row][col_off + n] = sum_{k in split} X[row][k] * W[n][k]
//   W bf16 [N][K] row-major; X as bf16 hi/lo planes (or, mode kXRelu2, relu(sum of f32
//   partial slabs)^2 split on the fly). MFMA 16x16x32 bf16.
//   Workgroup = 4 waves = 64 output columns (16 per wave) x MT*16 rows x one K slice.
//   * every wave issues ALL of its weight loads for the slice first (HBM stream, one 16-byte
//     load per lane per 32-deep K step: lane l reads W[col0 + (l&15)][k0 + 8(l>>4) .. +8]);
//   * meanwhile the workgroup stages its X slice into LDS once (shared by the 4 waves);
//   * A fragments come from LDS (ds_read_b128), B fragments from the registers.
//   Each wave owns complete output columns: no cross-wave reduction; split-K partial slabs
//   are summed (fixed order) by the consumer.
// ------------------------------------------------------------------------------------
template <int MT, int KSTEPS, int XMODE>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KS = KSTEPS * 32;      // K slice
  constexpr int LD = KS + 8;           // LDS row stride (elements): +16 B breaks bank aliasing
  constexpr int ROWS = MT * 16;
  bf16_t* xh = (bf16_t*)smem;
  bf16_t* xl = xh + ROWS * LD;
  const int tile = blockIdx.x;
  int s = 0;
  while (s + 1 < a.nseg && tile >= a.seg[s + 1].tile_start) ++s;
  const GemmSeg& sg = a.seg[s];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int col0 = (tile - sg.tile_start) * 64 + wave * 16;
  const int split = blockIdx.y;
  const int kbeg = split * KS;
  const int row0 = blockIdx.z * ROWS;
  // 1) weight stream for this wave's 16 columns
  int n = col0 + li;
  if (n >= sg.N) n = sg.N - 1;
  const bf16_t* wrow = sg.W + (int64_t)n * a.K + kbeg + g * 8;
  short8 b[KSTEPS];
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t) b[t] = __builtin_nontemporal_load((const short8*)(wrow + t * 32));
  // 2) stage X slice
  constexpr int CH = KS / 8;  // 16-byte chunks per row
  if constexpr (XMODE == kXPlanes) {
    constexpr int PER = ROWS * CH / 256;  // 16-byte chunks per thread per plane
    short8 vh[PER], vl[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      const int src = row0 + r;
      vh[u] = vl[u] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
      if (src < a.M) {
        const int64_t o = (int64_t)src * sg.ldx + kbeg + k8;
        vh[u] = *(const short8*)(sg.Xhi + o);
        vl[u] = *(const short8*)(sg.Xlo + o);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      *(short8*)(xh + r * LD + k8) = vh[u];
      *(short8*)(xl + r * LD + k8) = vl[u];
    }
  } else {  // kXRelu2: x = relu(sum_p P[p][row][k])^2, partials summed in order 0..n-1
    constexpr int PER = ROWS * KS / 4 / 256;  // float4 chunks per thread
    float4_ x[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) x[u] = (float4_){0.f, 0.f, 0.f, 0.f};
    for (int p0 = 0; p0 < a.x_nsplit; p0 += 2) {
      float4_ t[2][PER];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int c = threadIdx.x + u * 256;
          const int r = c / (KS / 4), k4 = (c % (KS / 4)) * 4;
          const int src = row0 + r;
          t[pp][u] = (src < a.M && p0 + pp < a.x_nsplit)
                         ? *(const float4_*)(a.x_part + (p0 + pp) * a.x_part_stride + (int64_t)src * a.x_ld + kbeg + k4)
                         : (float4_){0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int u = 0; u < PER; ++u) x[u] += t[pp][u];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / (KS / 4), k4 = (c % (KS / 4)) * 4;
      uint16_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = x[u][e] > 0.f ? x[u][e] * x[u][e] : 0.f;
        h[e] = f32_to_bf16(y);
        l[e] = f32_to_bf16(y - bf16_to_f32(h[e]));
      }
      *(uint2*)(xh + r * LD + k4) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
      *(uint2*)(xl + r * LD + k4) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
  }
  __syncthreads();
  // 3) MFMA over the slice
  float4_ acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = (float4_){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int o = (m * 16 + li) * LD + t * 32 + g * 8;
      const short8 ah = *(const short8*)(xh + o);
      const short8 al = *(const short8*)(xl + o);
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah),
                                                       __builtin_bit_cast(bf16x8, b[t]), acc[m], 0, 0, 0);
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al),
                                                       __builtin_bit_cast(bf16x8, b[t]), acc[m], 0, 0, 0);
    }
  }
  // 4) store (D layout: col = lane&15, row = 4*(lane>>4) + j)
  const int col = col0 + li;
  if (col < sg.N) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = row0 + m * 16 + 4 * g + j;
        if (row < a.M) a.out[split * a.split_stride + (int64_t)row * a.ldo + sg.col_off + col] = acc[m][j];
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


__global__ __launch_bounds__(256) void k_wkv(WkvArgs a) {
  constexpr int N = 64;
  __shared__ float s_hid[kMaxLoraTotal];
  __shared__ float s_r[N], s_k[N], s_v[N], s_w[N], s_kk[N], s_b[N], s_g[N], s_y[N];
  __shared__ float s_lora[4][N];
  __shared__ __attribute__((aligned(16))) bf16_t s_lw[N * (kMaxLoraTotal + 8)];
  const int4 sg = a.segs[blockIdx.x];
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  const int h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = a.C;
  const int c = h * N + lane;  // this lane's channel (waves 0..3 all index the head's channels)
  const int i = tid >> 2, jq = (tid & 3) * 16;
  float* Sg = a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N + i * N + jq;
  // ---- prologue: every load that does not depend on this step's activations
  float S[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4_ v4 = *(const float4_*)(Sg + q * 4);
    S[q * 4 + 0] = v4[0]; S[q * 4 + 1] = v4[1]; S[q * 4 + 2] = v4[2]; S[q * 4 + 3] = v4[3];
  }
  // LoRA-up: 4 threads per channel (cc = tid >> 2, quarter pq = tid & 3 of each rank D)
  const int cc = tid >> 2, pq = tid & 3;
  const int Dv_eff = a.layer > 0 ? a.Dv : 0;
  const int Dq[4] = {a.Dw / 4, a.Da / 4, Dv_eff / 4, a.Dg / 4};
  // the head's LoRA-up rows (64 channels x Dtot bf16) staged once into LDS
  const int Dall = a.Dw + a.Da + a.Dv + a.Dg, LDW = Dall + 8;
  {
    const int moff[4] = {0, a.Dw, a.Dw + a.Da, a.Dw + a.Da + a.Dv};
    const int Dm[4] = {a.Dw, a.Da, a.Dv, a.Dg};
    const bf16_t* Wb[4] = {a.w2t, a.a2t, a.v2t, a.g2t};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int ch8 = Dm[m] / 8;  // 16-byte chunks per row
      for (int q = tid; q < N * ch8; q += 256) {
        const int ch = q / ch8, k8 = (q % ch8) * 8;
        *(short8*)(s_lw + ch * LDW + moff[m] + k8) = *(const short8*)(Wb[m] + (int64_t)(h * N + ch) * Dm[m] + k8);
      }
    }
  }
  float w0 = 0.f, a0 = 0.f, v0 = 0.f, kkc = 0.f, kac = 0.f, rkc = 0.f, lnw = 0.f, lnb = 0.f;
  if (wave == 0) {
    w0 = a.w0[c]; a0 = a.a0[c]; v0 = a.v0[c]; kkc = a.k_k[c]; kac = a.k_a[c];
    rkc = a.r_k[c]; lnw = a.lnx_w[c]; lnb = a.lnx_b[c];
  }
  const int Dtot = a.Dw + a.Da + a.Dv + a.Dg;
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    const float* prow = a.part + (int64_t)row * a.ldp;
    // ---- this row's activations: LoRA hidden (all), r/k/v (wave 0), v_first
    float hx0 = 0.f, hx1 = 0.f;
    for (int p = 0; p < a.n_part; ++p) {
      if (tid < Dtot) hx0 += prow[p * a.part_stride + 3 * C + tid];
      if (tid + 256 < Dtot) hx1 += prow[p * a.part_stride + 3 * C + tid + 256];
    }
    float r = 0.f, k = 0.f, v = 0.f, vf = 0.f;
    if (wave == 0) {
      for (int p = 0; p < a.n_part; ++p) {
        const float* pp = prow + p * a.part_stride;
        r += pp[c];
        k += pp[C + c];
        v += pp[2 * C + c];
      }
      if (a.layer > 0) vf = a.v_first[(int64_t)row * a.ldv + c];
    }
    auto act = [&](int d, float x) {
      if (d < a.Dw) return tanhf(x);
      if (d >= a.Dw + a.Da + a.Dv) return sigm(x);
      return x;
    };
    if (tid < Dtot) s_hid[tid] = act(tid, hx0);
    if (tid + 256 < Dtot) s_hid[tid + 256] = act(tid + 256, hx1);
    __syncthreads();
    // ---- LoRA up for this head's channels from the prefetched rows
    {
      const int hoffs[4] = {0, a.Dw, a.Dw + a.Da, a.Dw + a.Da + a.Dv};
      float accm[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float acc = 0.f;
        const bf16_t* wr = s_lw + cc * LDW + hoffs[m] + pq * Dq[m];
        const float* hh = s_hid + hoffs[m] + pq * Dq[m];
        for (int d = 0; d < Dq[m]; d += 4) {
          const uint2 q = *(const uint2*)(wr + d);
          acc += bf16_to_f32((uint16_t)(q.x & 0xFFFF)) * hh[d + 0];
          acc += bf16_to_f32((uint16_t)(q.x >> 16)) * hh[d + 1];
          acc += bf16_to_f32((uint16_t)(q.y & 0xFFFF)) * hh[d + 2];
          acc += bf16_to_f32((uint16_t)(q.y >> 16)) * hh[d + 3];
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        accm[m] = acc;
      }
      if (pq == 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) s_lora[m][cc] = accm[m];
      }
    }
    __syncthreads();
    if (wave == 0) {
      const float w = expf(-0.60653066f * sigm(w0 + s_lora[0][lane]));
      const float av = sigm(a0 + s_lora[1][lane]);
      float kk = k * kkc;
      const float nrm = sqrtf(wave_sum(kk * kk));
      kk = kk / fmaxf(nrm, 1e-12f);
      k = k * (1.0f + (av - 1.0f) * kac);
      if (a.layer == 0) {
        a.v_first[(int64_t)row * a.ldv + c] = v;
      } else {
        const float gate = sigm(v0 + s_lora[2][lane]);
        v = v + (vf - v) * gate;
      }
      s_r[lane] = r; s_k[lane] = k; s_v[lane] = v; s_w[lane] = w;
      s_kk[lane] = kk; s_b[lane] = kk * av; s_g[lane] = s_lora[3][lane];
    }
    __syncthreads();
    // ---- state update: S[i][j] = S[i][j]*w_j - sa_i*b_j + v_i*k_j ; y_i = sum_j S[i][j] r_j
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
      const float yv = s_y[lane];
      const float mean = wave_sum(yv) * (1.0f / N);
      const float dv = yv - mean;
      const float var = wave_sum(dv * dv) * (1.0f / N);
      const float rstd = 1.0f / sqrtf(var + 64e-5f);
      const float bonus = wave_sum(s_r[lane] * s_k[lane] * rkc);
      const float gn = dv * rstd * lnw + lnb;
      split_store((gn + bonus * s_v[lane]) * s_g[lane], a.z_hi, a.z_lo, (int64_t)row * a.ldz + c);
    }
    if (rr + 1 < n_rows) __syncthreads();
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
  LnMixArgs b = a;
  b.n_rows = n_out_rows;
  const dim3 grid(n_out_rows);
  if (a.C <= 1024) hipLaunchKernelGGL(k_ln_mix<1>, grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL(k_ln_mix<2>, grid, dim3(256), 0, st, b);
}

template <int MT, int KSTEPS>
static void launch_gemm_t(const GemmArgs& a, dim3 grid, hipStream_t st) {
  const size_t lds = (size_t)MT * 16 * (KSTEPS * 32 + 8) * 2 * 2;
  if (a.xmode == kXPlanes) hipLaunchKernelGGL((k_gemm<MT, KSTEPS, kXPlanes>), grid, dim3(256), lds, st, a);
  else hipLaunchKernelGGL((k_gemm<MT, KSTEPS, kXRelu2>), grid, dim3(256), lds, st, a);
}

int gemm_ksteps(int kslice) { return kslice / 32; }

void launch_gemm(const GemmArgs& a, hipStream_t st) {
  const int tiles = a.seg[a.nseg - 1].tile_start + (a.seg[a.nseg - 1].N + 63) / 64;
  const int mt = a.M <= 16 ? 1 : 2;
  const int mg = (a.M + mt * 16 - 1) / (mt * 16);
  dim3 grid(tiles, a.k_split, mg);
  const int ks = a.kslice / 32;
#define GEMM_CASE(KS_)                                          \
  case KS_:                                                     \
    if (mt == 1) launch_gemm_t<1, KS_>(a, grid, st);            \
    else launch_gemm_t<2, KS_>(a, grid, st);                    \
    break;
  switch (ks) {
    GEMM_CASE(4)
    GEMM_CASE(8)
    GEMM_CASE(16)
    default: break;  // rejected at engine init (kslice in {128, 256, 512})
  }
#undef GEMM_CASE
}
void launch_wkv(const WkvArgs& a, int n_seg, int H, hipStream_t st) {
  hipLaunchKernelGGL(k_wkv, dim3(n_seg, H), dim3(256), 0, st, a);
}

}  // namespace rwkvtts
