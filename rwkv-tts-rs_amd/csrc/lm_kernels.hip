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

#include <stdlib.h>

#include <algorithm>

namespace rwkvtts {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Cross-lane sums on DPP moves (no LDS round trip, unlike __shfl_xor's ds_bpermute). Each step
// pairs every lane with a partner holding the other half of its group and both add in the same
// order, so every lane of a group ends with the identical sum.
// NormalFloat-4 code table (RWKVTTS_QUANT_NF4; quant_pack below, k_gemm2 dequantisation)
__device__ __constant__ float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
    -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
    0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

template <int CTRL>
__device__ inline float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ inline float sum16(float v) {  // aligned groups of 16 lanes
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror: the two quads of each half-row
  return v + dpp_mov<0x140>(v);  // row_mirror: the two halves of each row
}
__device__ inline float readlane_f32(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ inline float wave_sum(float v) {  // whole wave (all lanes active); uniform result
  v = sum16(v);
  return (readlane_f32(v, 0) + readlane_f32(v, 16)) + (readlane_f32(v, 32) + readlane_f32(v, 48));
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

__device__ inline void split_store(float x, bf16_t* hi, bf16_t* lo, int64_t idx, bool f16 = false) {
  const uint16_t h = f32_to_w16(x, f16);
  const float r = x - w16_to_f32(h, f16);
  hi[idx] = h;
  lo[idx] = f32_to_w16(r, f16);
}

// ------------------------------------------------------------------------------------
// embed: h[r] = LN0(emb[token[r]])
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_embed(const uint32_t* tokens, const int4* rows, const int* ctrl_tok,
                                               int ctrl_stride, const bf16_t* emb, const float* w, const float* b,
                                               float* h, int C, int f16, unsigned long long* tl, int n_vocab) {
  __shared__ float red[4];
  tl_begin(tl);
  const int r = blockIdx.x;
  const int4 info = rows[r];
  uint32_t tok = (info.y & kRowCtrl) ? (uint32_t)ctrl_tok[(int64_t)info.x * ctrl_stride] : tokens[r];
  if (tok >= (uint32_t)n_vocab) tok = 0;  // ids are validated on the host; never index past the table
  const bf16_t* e = emb + (int64_t)tok * C;
  float v[kMaxPerThread];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerThread; ++i) {
    const int c = threadIdx.x + i * 256;
    v[i] = c < C ? w16_to_f32(e[c], f16 != 0) : 0.f;
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
  tl_end(tl);
}

// ------------------------------------------------------------------------------------
// ln_mix: one workgroup per row, thread t owns the 4 columns [4t, 4t+4) (x kLnVec chunks of
// 1024 columns). hn = h_in + sum(partials) (fixed order); optionally store hn; xx = LN(hn);
// x_m = xx + (prev - xx) * mu_m (split to bf16 hi/lo); shift state update. Latency-bound:
// every independent load (partials unrolled 4-wide) is issued before the first reduction.
// ------------------------------------------------------------------------------------
__device__ inline float4_ ld4(const float* p) { return *(const float4_*)p; }

template <int kLnVec, int NP>  // NP >= 0: exactly NP partial slabs (all loads in flight at once); -1: a.n_part
__device__ inline void ln_load_row(const LnMixArgs& a, int src, float4_* v) {
  const int t4 = 4 * threadIdx.x;
  const float4_ z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < kLnVec; ++q) {
    const int c = t4 + 1024 * q;
    v[q] = c < a.C ? ld4(a.h_in + (int64_t)src * a.C + c) : z;
  }
  if constexpr (NP >= 0) {
    if constexpr (NP > 0) {
      const float* pp = a.part + (int64_t)src * a.ldp;
      float4_ t[NP][kLnVec];
#pragma unroll
      for (int u = 0; u < NP; ++u)
#pragma unroll
        for (int q = 0; q < kLnVec; ++q) {
          const int c = t4 + 1024 * q;
          t[u][q] = c < a.C ? ld4(pp + u * a.part_stride + c) : z;
        }
#pragma unroll
      for (int u = 0; u < NP; ++u)
#pragma unroll
        for (int q = 0; q < kLnVec; ++q) v[q] += t[u][q];
    }
    return;
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
        t[u][q] = c < a.C ? ld4(pp + u * a.part_stride + c) : z;
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

__device__ inline void store_split4(const float4_& x, bf16_t* hi, bf16_t* lo, int64_t idx, bool f16) {
  uint16_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = f32_to_w16(x[e], f16);
    l[e] = f32_to_w16(x[e] - w16_to_f32(h[e], f16), f16);
  }
  *(uint2*)(hi + idx) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
  *(uint2*)(lo + idx) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
}

template <int kLnVec, int NP>  // C <= 1024 * kLnVec; NP: partial slabs (-1: runtime a.n_part)
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
  ln_load_row<kLnVec, NP>(a, row, v);
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
      if (c < a.C) store_split4(v[q], a.x_hi, a.x_lo, (int64_t)out_row * a.ldx + c, a.f16 != 0);
    }
    return;
  }
  if (prev_row >= 0) {  // prefill row: the previous token's LN output, recomputed identically
    ln_load_row<kLnVec, NP>(a, prev_row, pv);
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
        store_split4(x, a.x_hi + m * a.mix_stride, a.x_lo + m * a.mix_stride, (int64_t)out_row * a.ldx + c,
                     a.f16 != 0);
      }
    }
  }
  if (flags & kRowLast) {
    float* sn = a.shift + (((int64_t)(a.inplace ? par : par ^ 1) * a.S + slot) * a.L + a.layer) * a.C;
#pragma unroll
    for (int q = 0; q < kLnVec; ++q) {
      const int c = t4 + 1024 * q;
      if (c < a.C) *(float4_*)(sn + c) = v[q];
    }
  }
}

// The C = 1024 LayerNorm of one row in a 256-thread workgroup, thread t holding columns
// [4t, 4t + 4): two one-barrier block sums (mean, then the centred second moment), x = d * rstd * w
// + b. Shared by ln1024_body and the row-fused GEMM roles (gemm2_body ROLE 5 / 6), so both give the
// same bits.
__device__ __attribute__((always_inline)) inline void ln1024_apply(float4_& x, const float4_& w, const float4_& b,
                                                                   float* red, int slot_base) {
  constexpr int C = 1024;
  const float mean = block_sum_1b((x[0] + x[1]) + (x[2] + x[3]), red, slot_base) * (1.0f / C);
  const float4_ d = x - mean;
  const float var = block_sum_1b((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]), red, slot_base + 1) * (1.0f / C);
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
  x = d * rstd * w + b;
}

// ------------------------------------------------------------------------------------
// ln1024: k_ln_mix for C = 1024 with the weight format, the mix count and the partial-slab count
// as template parameters (no per-element guards, no runtime format select, packed hardware
// bf16/f16 conversion of the hi/lo planes). MODE 1: LN + NMIX token-shift mixes + shift update;
// MODE 0: ln_out (x = LN(h) planes only). Loads that need only the row (residual, slabs, LN and
// mix vectors) are issued before the row descriptor that addresses the shift state.
// ------------------------------------------------------------------------------------
// SC1: the residual and the partial slabs were written earlier in the same (persistent) launch:
// read with sc1 (L1-bypassing) buffer loads from wave-uniform bases
template <bool F16, int MODE, int NMIX, int NP, bool EMB = false, bool SC1 = false>
__device__ __attribute__((always_inline)) void ln1024_body(const LnMixArgs& a, const int out_row) {
  constexpr int C = 1024;
  static_assert(!EMB || (MODE == 1 && NP == 0), "embedding fusion: layer 0's LN + mixes");
  __shared__ float red[16];
  __shared__ __attribute__((aligned(16))) float s_h[EMB ? C : 1];
  bf16_t* e_xhi = a.x_hi;
  bf16_t* e_xlo = a.x_lo;
  int64_t e_mix = a.mix_stride;
  int e_ldx = a.ldx;
  float* e_hout = a.h_out;
  const float* e_hin = a.h_in;
  const float* e_part = a.part;
  int64_t e_pstride = a.part_stride;
  int e_ldp = a.ldp;
  float* e_shift = a.shift;
  int e_S = a.S, e_L = a.L, e_layer = a.layer, e_inpl = a.inplace;

  // MODE 1 (LN + mixes) never remaps rows: no dependent row_map load
  const int row = (MODE == 0 && a.row_map) ? a.row_map[out_row] : out_row;
  const int c = 4 * threadIdx.x;
  // loads that do not depend on the previous launch: LN / mix vectors
  const float4_ w = ld4(a.ln_w + c), b = ld4(a.ln_b + c);
  float4_ mu[NMIX > 0 ? NMIX : 1];
#pragma unroll
  for (int m = 0; m < NMIX; ++m) mu[m] = ld4(a.mu[m] + c);
  // the residual and the partial slabs (the previous launch's output) go out before the row
  // descriptor, whose dependent round trip only addresses the shift state
  float4_ v;
  if constexpr (EMB) {
    // k_embed's arithmetic for this row (thread t: columns t + 256 i, sums in that order, the same
    // block reductions; its zero-padded columns 1024.. add exact zeros), LN0 into LDS, then the
    // row in this kernel's column order
    const int4 info = a.rows[row];
    uint32_t tok = (info.y & kRowCtrl) ? (uint32_t)a.emb_ctrl[(int64_t)info.x * a.emb_ctrl_stride] : a.emb_tok[row];
    if (tok >= (uint32_t)a.n_vocab) tok = 0;
    const bf16_t* er = a.emb + (int64_t)tok * C;
    float ev[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ev[i] = w16_to_f32(er[threadIdx.x + i * 256], F16);
      s += ev[i];
    }
#pragma unroll
    for (int i = 4; i < kMaxPerThread; ++i) s += 0.f;  // k_embed's padded columns (-0 + 0 = +0)
    const float mean0 = block_sum256(s, red) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = ev[i] - mean0;
      q += d * d;
    }
    const float rstd0 = 1.0f / sqrtf(block_sum256(q, red) / (float)C + 1e-5f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cc = threadIdx.x + i * 256;
      s_h[cc] = (ev[i] - mean0) * rstd0 * a.ln0_w[cc] + a.ln0_b[cc];
    }
    __syncthreads();
    v = *(const float4_*)(s_h + c);
  } else {
    if constexpr (SC1)
      v = __builtin_bit_cast(float4_, __builtin_amdgcn_raw_buffer_load_b128(wt_rsrc(e_hin + (int64_t)row * C), c * 4, 0, 16));
    else
      v = ld4(e_hin + (int64_t)row * C + c);
  }
  float4_ t[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if constexpr (SC1)
      t[p] = __builtin_bit_cast(float4_, __builtin_amdgcn_raw_buffer_load_b128(
                                             wt_rsrc(e_part + p * e_pstride + (int64_t)row * e_ldp), c * 4, 0, 16));
    else
      t[p] = ld4(e_part + p * e_pstride + (int64_t)row * e_ldp + c);
  }
  int slot = 0, flags = 0, prev_row = -1, par = 0;
  float4_ pv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 1) {
    const int4 info = a.rows[row];
    slot = info.x; flags = info.y; prev_row = info.z; par = info.w;
    if (prev_row < 0) pv = ld4(e_shift + (((int64_t)par * e_S + slot) * e_L + e_layer) * C + c);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) v += t[p];
  const bool wt = a.wt != 0;
  if (e_hout) {
    if (wt) store_wt(wt_rsrc(e_hout), (int)(((int64_t)row * C + c) * 4), v);
    else *(float4_*)(e_hout + (int64_t)row * C + c) = v;
  }
  auto ln = [&](float4_& x, int slot_base) { ln1024_apply(x, w, b, red, slot_base); };
  ln(v, 0);
  auto store = [&](const float4_& x, bf16_t* hi, bf16_t* lo, int64_t idx) {
    uint32_t h0, l0, h1, l1;
    split2<F16>(x[0], x[1], h0, l0);
    split2<F16>(x[2], x[3], h1, l1);
    if (wt) {
      store_wt(wt_rsrc(hi), (int)(idx * 2), make_uint2(h0, h1));
      store_wt(wt_rsrc(lo), (int)(idx * 2), make_uint2(l0, l1));
    } else {
      *(uint2*)(hi + idx) = make_uint2(h0, h1);
      *(uint2*)(lo + idx) = make_uint2(l0, l1);
    }
  };
  if constexpr (MODE == 0) {
    store(v, e_xhi, e_xlo, (int64_t)out_row * e_ldx + c);
  } else {
    if (prev_row >= 0) {  // prefill row: the previous token's LN output, recomputed identically
      pv = ld4(e_hin + (int64_t)prev_row * C + c);
      float4_ tp[NP > 0 ? NP : 1];
#pragma unroll
      for (int p = 0; p < NP; ++p) tp[p] = ld4(e_part + p * e_pstride + (int64_t)prev_row * e_ldp + c);
#pragma unroll
      for (int p = 0; p < NP; ++p) pv += tp[p];
      ln(pv, 2);
    }
#pragma unroll
    for (int m = 0; m < NMIX; ++m) {
      const float4_ x = v + (pv - v) * mu[m];
      store(x, e_xhi + m * e_mix, e_xlo + m * e_mix, (int64_t)out_row * e_ldx + c);
    }
    if (flags & kRowLast) {
      float* sp = e_shift + (((int64_t)(e_inpl ? par : par ^ 1) * e_S + slot) * e_L + e_layer) * C;
      if (wt) store_wt(wt_rsrc(sp), c * 4, v);
      else *(float4_*)(sp + c) = v;
    }
  }
}

template <bool F16, int MODE, int NMIX, int NP, bool EMB = false>
__global__ __launch_bounds__(256) void k_ln1024(LnMixArgs a) {
  tl_begin(a.tl);
  ln1024_body<F16, MODE, NMIX, NP, EMB>(a, blockIdx.x);
  tl_end(a.tl);
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
template <int MT, int KSTEPS, int XMODE, bool F16>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t s_rexp[MT * 16];  // f16 relu^2 rows: bits of the row maximum if >= 2^15
  constexpr int KS = KSTEPS * 32;      // K slice
  constexpr int LD = KS + 8;           // LDS row stride (elements): +16 B breaks bank aliasing
  constexpr int ROWS = MT * 16;
  bf16_t* xh = (bf16_t*)smem;
  bf16_t* xl = xh + ROWS * LD;
  uint64_t* gst = (a.stamps && threadIdx.x == 0)
                      ? a.stamps + ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 : nullptr;
  if (gst) gst[0] = __builtin_amdgcn_s_memtime();
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
  // 1) weight stream for this wave's 16 columns: W is pre-packed in MFMA fragment order
  // (launch_pack_frag), so each load instruction reads one contiguous 1 KB block and the
  // wave's KSTEPS blocks are consecutive
  int nb = col0 >> 4;
  const int nblk = (sg.N + 15) >> 4;
  if (nb >= nblk) nb = nblk - 1;
  const bf16_t* wp = sg.W + (((int64_t)nb * (a.K >> 5) + (kbeg >> 5)) * 64 + lane) * 8;
  short8 b[KSTEPS];
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t)
    b[t] = __builtin_nontemporal_load((const short8*)(wp + t * 512));
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
    // f16 model: per-row power-of-two range scaling of relu^2 (see k_gemm2)
    if constexpr (F16) {
      if (threadIdx.x < ROWS) s_rexp[threadIdx.x] = 0u;
      __syncthreads();
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int r = (threadIdx.x + u * 256) / (KS / 4);
        float m = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) m = fmaxf(m, x[u][e] > 0.f ? x[u][e] * x[u][e] : 0.f);
        if (m >= 32768.f) atomicMax(&s_rexp[r], as_u32(m));
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / (KS / 4), k4 = (c % (KS / 4)) * 4;
      uint16_t h[4], l[4];
      float sc = 1.f;
      if constexpr (F16) {
        const uint32_t mb = s_rexp[r];
        if (mb) sc = as_f32((uint32_t)(127 - (int)((mb >> 23) & 0xFF) + 127 + 14) << 23);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (x[u][e] > 0.f ? x[u][e] * x[u][e] : 0.f) * sc;
        h[e] = f32_to_w16(y, F16);
        l[e] = f32_to_w16(y - w16_to_f32(h[e], F16), F16);
      }
      *(uint2*)(xh + r * LD + k4) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
      *(uint2*)(xl + r * LD + k4) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
  }
  __syncthreads();
  if (gst) gst[1] = __builtin_amdgcn_s_memtime();
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
      if constexpr (F16) {
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah),
                                                        __builtin_bit_cast(f16x8, b[t]), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, al),
                                                        __builtin_bit_cast(f16x8, b[t]), acc[m], 0, 0, 0);
      } else {
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah),
                                                         __builtin_bit_cast(bf16x8, b[t]), acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al),
                                                         __builtin_bit_cast(bf16x8, b[t]), acc[m], 0, 0, 0);
      }
    }
  }
  if (gst) gst[2] = __builtin_amdgcn_s_memtime() + (uint64_t)(acc[0][0] != acc[0][0]);
  // 4) store (D layout: col = lane&15, row = 4*(lane>>4) + j)
  const int col = col0 + li;
  if (col < sg.N) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = row0 + m * 16 + 4 * g + j;
        float v = acc[m][j];
        if constexpr (F16 && XMODE == kXRelu2) {
          const uint32_t mb = s_rexp[m * 16 + 4 * g + j];
          if (mb) v *= as_f32((uint32_t)((int)((mb >> 23) & 0xFF) - 127 - 14 + 127) << 23);
        }
        if (row < a.M) a.out[split * a.split_stride + (int64_t)row * a.ldo + sg.col_off + col] = v;
      }
  }
  if (gst) gst[3] = __builtin_amdgcn_s_memtime();
}

// ------------------------------------------------------------------------------------
// gemm2: k_gemm with a shorter critical path.
//  * segment lookup without dependent scalar loads: every segment's fields are read in one
//    round and the tile's segment is picked by selects;
//  * the X slice (L2-resident activations) is requested BEFORE the weight stream, so staging X
//    into LDS waits only for X (vmcnt counts in issue order) and overlaps the HBM weight
//    latency; in kXRelu2 mode all NX key slabs are in flight at once;
//  * hi and lo products accumulate in separate MFMA chains (2*MT independent accumulators).
// ------------------------------------------------------------------------------------
// Inter-workgroup hand-offs of the persistent FFN launch (k_ffn_persist): counters kSyncStride
// ints (256 B) apart, [kSyncStride * r] (r < kLnReplicas) = LayerNorm rows published (one replica
// per XCD: every LN workgroup adds to all of them, a key workgroup polls replica blockIdx % 8, so
// 512 pollers do not share one line), [kSyncStride * (kLnReplicas + s)] = key workgroups that
// published their partial slab of value K-slice s.
__device__ inline void sync_stamp(const FfnSync& sy, int slot) {
  if (sy.stamps && threadIdx.x == 0) sy.stamps[blockIdx.x * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}
typedef __attribute__((address_space(1))) int gint_t;
// one lane polls the counter (relaxed agent-scope load = global_load sc1, s_sleep between polls),
// bounded by ~50 ms of s_memrealtime; the other waves wait at the barrier. On a timeout the code
// is ORed into err (the host fails the step) and the workgroup goes on (its output is garbage).
__device__ inline void sync_wait(const int* c, int target, int* err, int code, int opts = 0) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load((gint_t*)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (opts & 2) __builtin_amdgcn_s_sleep(8);
      else __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
        __hip_atomic_fetch_or((gint_t*)err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}
// test hook (RWKVTTS_TEST_DROP_ARRIVE=n): *drop counts the arrivals still to be dropped; takes one
__device__ inline bool take_drop(int* drop) {
  int v = __hip_atomic_load((gint_t*)drop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (v > 0)
    if (__hip_atomic_compare_exchange_strong((gint_t*)drop, &v, v - 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return true;
  return false;
}
// publish: every wave's write-through (sc1) stores drained, then ONE lane counts the workgroup in
// (replicas > 1: lanes 0..replicas-1 of wave 0 add to one replica each, kSyncStride ints apart).
// drop (test hook, replicas == 1 only): lane 0 skips the add if it takes a pending drop
__device__ inline void sync_arrive(int* c, int replicas = 1, int* drop = nullptr, int inc = 1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (drop && threadIdx.x == 0 && take_drop(drop)) return;
  if (threadIdx.x < replicas)
    __hip_atomic_fetch_add((gint_t*)(c + threadIdx.x * kSyncStride), inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// granule hand-off (FfnSync::gran): the tag of this pass and layer, one 8-byte {f32, tag} store
typedef __attribute__((address_space(1))) uint64_t gu64_t;
typedef uint64_t u64x2_ __attribute__((ext_vector_type(2)));
__device__ inline uint32_t gran_tag(const FfnSync& sy) {
  // (an sc1 vector load: the word changed in an earlier launch, a scalar-cache read can be stale).
  // Bit 31 set: a tag is never 0, so a zeroed granule (Engine::reset_persistent) never matches, also
  // once the 32-bit epoch * 64 has wrapped (every 2^25 one-row passes)
  const int ep = __hip_atomic_load((gint_t*)sy.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (((uint32_t)__builtin_amdgcn_readfirstlane(ep) * 64u + (uint32_t)sy.layer) & 0x7FFFFFFFu) | 0x80000000u;
}
// the poll loops re-read their granules with volatile (cache-policy bit 31) 16-byte sc1 buffer loads
// through a wave-uniform resource, two granules per load: a volatile load is re-issued on every pass
// (a plain load in a spin loop may legally be merged or hoisted out of it; the disassembly shows
// the loads inside the loop), sc1 serves it from L2, never a stale L1. Each 8-byte {data, tag}
// granule is written by ONE 8-byte sc1 store and read untorn within the 16-byte load (observed on
// gfx950 / ROCm 7.2, MI355X_MICROARCH.md "R2's granule": not an architectural guarantee -- a torn
// read would fail the tag compare of the half that lags and the poll simply runs another pass).
// (One 64-bit atomic load per granule instead: B = 1 decode 521-523 vs 514-520 us per step,
// profiles/r06f_granule_poll_ab.txt.)
__device__ inline u64x2_ ld_gran2(__amdgpu_buffer_rsrc_t r, int off_bytes) {
  return __builtin_bit_cast(u64x2_, __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, (int)0x80000010u));
}
__device__ inline void gran_store_bits(uint64_t* p, uint32_t bits, uint32_t tag) {
  __hip_atomic_store((gu64_t*)p, ((uint64_t)tag << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void gran_store(uint64_t* p, float v, uint32_t tag) {
  gran_store_bits(p, __builtin_bit_cast(uint32_t, v), tag);
}
// hold a prefetch back until `ticks` (10 ns) after the launch's first s_memrealtime read here
__device__ inline void hold_until(int ticks) {
  if (ticks <= 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(2);
}
// handed-off bytes are read with sc1 (L1-bypassing) buffer loads only (after the hand-off's counter
// wait: never as the polled word itself -- polls are atomic / volatile loads, sync_wait / ld_gran2)
__device__ inline u32x4_ ld_sc1_b128(__amdgpu_buffer_rsrc_t r, int off_bytes) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 16);
}

// ROLE 0: a plain launch. ROLE 1: key workgroup of k_ffn_persist (weights first, then wait for
// the LayerNorm rows, X by sc1 loads, publish the partial slab). ROLE 2: value workgroup (weights
// first, then wait for its K-slice's key slabs, read them by sc1 loads). ROLE 3: rkv workgroup of
// k_att_persist (as ROLE 1; publishes to its head's counter, or the LoRA-down counter). ROLE 4:
// Wo workgroup (weights first, then wait for the WKV workgroups of its K-slice's two heads).
// ROLE 5 / 6: the row-fused forms of ROLE 3 / 1 (one decode row): weights at dispatch, then the
// row's LayerNorm computed here from the residual and the partial slabs (*lr: LN1 with 16 value
// slabs / LN2 with 8 Wo slabs; ln1024_apply, the LayerNorm rows' arithmetic bit for bit) and only
// this K-slice's mix staged as row 0 of the X image -- no LayerNorm rows, no hand-off before the GEMM.
// by: the split index of an xmap-0 grid (blockIdx.y for a plain launch).
template <int MT, int KSTEPS, int XMODE, bool F16, int NX, int MS, bool QW, int ROLE, class GA>
__device__ __attribute__((always_inline)) void gemm2_body(const GA& a, const int bx, const int by,
                                                          const FfnSync& sy, const LnMixArgs* lr = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t s_rexp[MT * 16];  // f16 relu^2 rows: bits of the row maximum if >= 2^15
  __shared__ float s_qlut[QW ? 16 : 1];  // QW: the NF4 code table
  constexpr int KS = KSTEPS * 32;
  constexpr int LD = KS + 8;
  constexpr int ROWS = MT * 16;
  bf16_t* xh = (bf16_t*)smem;
  bf16_t* xl = xh + ROWS * LD;
  float* e_out = a.out;
  int64_t e_sstride = a.split_stride;
  int e_ldo = a.ldo, e_M = a.M;
  int tile = bx, split = by;
  if (a.xmap == 2) {  // consumer-aligned 1-D grid (GemmArgs::xalign)
    const int b = bx, xcd = b & 7, j = b >> 3;
    split = j % a.k_split;
    const int lt = j / a.k_split;
    tile = (xcd + 8 * (lt / a.xalign)) * a.xalign + lt % a.xalign;
    if (tile >= a.ntiles) return;  // padding workgroup
  } else if (a.xmap) {  // XCD-aware 1-D grid (GemmArgs::xmap)
    const int b = bx, xcd = b & 7, j = b >> 3;
    if (a.k_split >= 8) {
      split = xcd + 8 * (j / a.ntiles);
      tile = j % a.ntiles;
    } else {
      split = xcd % a.k_split;
      tile = (xcd / a.k_split) * a.tiles_per_xcd + j;
      if (tile >= a.ntiles) return;  // padding workgroup
    }
  }
  // MS 0: one segment, read from seg[0] directly. MS 1: several segments, looked up from the
  // tile starts (a second, dependent kernel-argument round trip). MS 2: several segments
  // through the per-tile descriptor table (one round trip, addressed by blockIdx alone).
  int s = 0;
  if constexpr (MS == 1) {
#pragma unroll
    for (int j = 1; j < 8; ++j) s += (j < a.nseg && tile >= a.seg[j].tile_start) ? 1 : 0;
  }
  const bf16_t* Wm = a.seg[0].W;
  const bf16_t* Xhi = a.seg[0].Xhi;
  const bf16_t* Xlo = a.seg[0].Xlo;
  int ldx = a.seg[0].ldx, Nn = a.seg[0].N, col_off = a.seg[0].col_off, tstart = a.seg[0].tile_start;
  if constexpr (MS == 1) {
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if (s == j) {
        Wm = a.seg[j].W; Xhi = a.seg[j].Xhi; Xlo = a.seg[j].Xlo;
        ldx = a.seg[j].ldx; Nn = a.seg[j].N; col_off = a.seg[j].col_off; tstart = a.seg[j].tile_start;
      }
  }
  int qf = 0;  // QW: this tile's weight format (0: 16-bit fragments)
  if constexpr (QW && MS != 2) qf = a.q_fmt;
  int tile_mix = 0;  // (MS 2) the tile's mix plane
  if constexpr (MS == 2) {
    const uint32_t ti = a.tinfo[tile];
    if constexpr (QW) qf = (ti >> 31) ? a.q_fmt : 0;
    const int mix = ti & 7;
    tile_mix = mix;
    Wm = a.tw + (int64_t)tile * 64 * a.K;
    Xhi += mix * a.x_mix_stride;
    Xlo += mix * a.x_mix_stride;
    Nn = (ti >> 3) & 127;      // valid columns of this tile (the tile is its own segment)
    col_off = (int)((ti >> 10) & 0x1FFFFFu);
    tstart = tile;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int col0 = (tile - tstart) * 64 + wave * 16;
  const int kbeg = split * KS;
  // row groups: a workgroup runs row groups blockIdx.z, blockIdx.z + gridDim.z, ... (prefill
  // steps; decode steps have one) with its weight fragments loaded once, and requests the next
  // group's X while the current one computes. Every output element takes the same MFMA sequence
  // as with one row group per workgroup: bit-identical.
  // (quantised launches keep one row group per workgroup: the loop's live registers spill there)
  int rg = a.xmap ? 0 : (int)blockIdx.z;
  const int nrg = (a.xmap || QW) ? rg + 1 : (e_M + ROWS - 1) / ROWS;
  int row0 = rg * ROWS;
  int xrow0 = row0;  // the row group load_x requests
  // X slice (activations of the previous launch, L2-resident) and weight stream (packed
  // fragment blocks, 1 KB per wave instruction). X is requested first: staging waits only for X
  // (vmcnt retires in order) while the weights are still in flight.
  constexpr int CH = KS / 8;
  constexpr int PERP = ROWS * CH / 256;        // kXPlanes: 16-byte chunks per thread per plane
  constexpr int PERR = ROWS * KS / 4 / 256;    // kXRelu2: float4 chunks per thread per slab
  short8 vh[XMODE == kXPlanes ? PERP : 1], vl[XMODE == kXPlanes ? PERP : 1];
  float4_ xr[XMODE == kXPlanes ? 1 : NX][XMODE == kXPlanes ? 1 : PERR];
  int nb = col0 >> 4;
  const int nblk = (Nn + 15) >> 4;
  if (nb >= nblk) nb = nblk - 1;
  const bf16_t* wp = Wm + (((int64_t)nb * (a.K >> 5) + (kbeg >> 5)) * 64 + lane) * 8;
  short8 b[KSTEPS];
  // quantised tiles: codes in the same fragment order (column tiles back to back from the
  // launch's first quantised tile), one scale word per (column, K-block) and step
  uint2 bq8[QW ? KSTEPS : 1];
  uint32_t bq4[QW ? KSTEPS : 1], qsc[QW ? KSTEPS : 1];
  if constexpr (QW) {
    if (threadIdx.x < 16) s_qlut[threadIdx.x] = kNF4[threadIdx.x];
  }
  // kXRelu2 element map: chunk u of this thread -> (row, first column) of the K-slice (chunk c =
  // tid + 256 u: row c / (KS / 4)). (Round 5 measured a per-wave map for the persistent value role --
  // wave w = key tile 4 split + w, each wave waiting for its own tile: 1 % slower at 32 rows,
  // tools/experiments/r05_ln_tail_value_stream.patch.)
  auto x_row = [&](int u) { return (int)((threadIdx.x + u * 256) / (KS / 4)); };
  auto x_col = [&](int u) { return (int)(((threadIdx.x + u * 256) % (KS / 4)) * 4); };
  auto load_x = [&]() {
  if constexpr (XMODE == kXPlanes) {
    if constexpr (ROLE != 0) {  // handed-off planes: sc1 loads only
      // rows past M: an offset past the buffer's range, which the load returns as zeros with no
      // memory traffic (a one-row step reads 1/32 of the X bytes; no per-load branch: an
      // exec-masked branch around each load cost the 32-row step 4 %, round 5)
      const auto rh = wt_rsrc(Xhi), rl = wt_rsrc(Xlo);
#pragma unroll
      for (int u = 0; u < PERP; ++u) {
        const int c = threadIdx.x + u * 256;
        const int r = c / CH, k8 = (c % CH) * 8;
        const int o = xrow0 + r < a.M ? ((xrow0 + r) * ldx + kbeg + k8) * 2 : (int)0x80000000u;
        vh[u] = __builtin_bit_cast(short8, ld_sc1_b128(rh, o));
        vl[u] = __builtin_bit_cast(short8, ld_sc1_b128(rl, o));
      }
    } else {
#pragma unroll
    for (int u = 0; u < PERP; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      const int src = min(xrow0 + r, a.M - 1);
      const int64_t o = (int64_t)src * ldx + kbeg + k8;
      vh[u] = *(const short8*)(Xhi + o);
      vl[u] = *(const short8*)(Xlo + o);
    }
    }
  } else {
    if constexpr (ROLE != 0) {  // handed-off key slabs: sc1 loads only (rows past M: zeros, as above)
#pragma unroll
      for (int p = 0; p < NX; ++p) {
        const auto rp = wt_rsrc(a.x_part + p * a.x_part_stride);
#pragma unroll
        for (int u = 0; u < PERR; ++u) {
          const int r = x_row(u), k4 = x_col(u);
          const int o = xrow0 + r < a.M ? ((xrow0 + r) * a.x_ld + kbeg + k4) * 4 : (int)0x80000000u;
          xr[p][u] = __builtin_bit_cast(float4_, ld_sc1_b128(rp, o));
        }
      }
    } else {
#pragma unroll
    for (int p = 0; p < NX; ++p)
#pragma unroll
      for (int u = 0; u < PERR; ++u) {
        const int c = threadIdx.x + u * 256;
        const int r = c / (KS / 4), k4 = (c % (KS / 4)) * 4;
        const int src = min(xrow0 + r, a.M - 1);
        xr[p][u] = *(const float4_*)(a.x_part + p * a.x_part_stride + (int64_t)src * a.x_ld + kbeg + k4);
      }
    }
  }
  };
  auto load_w = [&]() {
    if constexpr (QW) {
      if (qf) {
        const int nbq = MS == 2 ? tile * 4 + wave : nb;
        const int64_t ncol = (int64_t)nbq * 16 + li;
        const int64_t cb = (((int64_t)nbq * (a.K >> 5) + (kbeg >> 5)) * 64 + lane);
        if (qf == 1) {
          typedef uint32_t u32x2q __attribute__((ext_vector_type(2)));
          const u32x2q* qp = (const u32x2q*)(a.qw + cb * 8);
#pragma unroll
          for (int t = 0; t < KSTEPS; ++t) {
            const u32x2q v = __builtin_nontemporal_load(qp + t * 64);
            bq8[t] = make_uint2(v.x, v.y);
          }
#pragma unroll
          for (int t = 0; t < KSTEPS; ++t)
            qsc[t] = ((const uint32_t*)a.qs)[ncol * (a.K / kQ8Block) + ((kbeg + 32 * t) / kQ8Block)];
        } else {
          const uint32_t* qp = (const uint32_t*)(a.qw + cb * 4);
#pragma unroll
          for (int t = 0; t < KSTEPS; ++t) bq4[t] = __builtin_nontemporal_load(qp + t * 64);
#pragma unroll
          for (int t = 0; t < KSTEPS; ++t)
            qsc[t] = ((const uint16_t*)a.qs)[ncol * (a.K / kQ4Block) + ((kbeg + 32 * t) / kQ4Block)];
        }
        return;
      }
    }
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t) b[t] = __builtin_nontemporal_load((const short8*)(wp + t * 512));
  };
  if constexpr (ROLE == 1 || ROLE == 3) {
    // the weight stream does not depend on the LayerNorm: in flight during the wait (opts bit 2:
    // requested after it, so the poll is not queued behind the weights and the LN rows' loads do
    // not compete with them)
    const bool late_w = ROLE == 1 ? (sy.opts & 4) != 0 : (sy.opts & 16) != 0;
    hold_until(ROLE == 1 ? sy.d_k : sy.d_w);
    if (!late_w) load_w();
    sync_wait(sy.cnt + kSyncStride * (blockIdx.x & (kLnReplicas - 1)), sy.ln_rows, sy.err, 1, sy.opts);
    sync_stamp(sy, 1);
    load_x();
    if (late_w) load_w();
  } else if constexpr (ROLE == 4) {
    hold_until(sy.d_late);
    load_w();
    const int h0 = kbeg >> 6;  // the K-slice's first head (64 channels per head)
    for (int hh = h0; hh < h0 + (KS >> 6); ++hh) sync_wait(sy.cnt + kSyncStride * (kAttWkv + hh), sy.ln_rows, sy.err, 8, sy.opts);
    sync_stamp(sy, 1);
    load_x();
  } else if constexpr (ROLE == 8) {
    // Wo workgroup of the granule form (one row): weights at dispatch, then wave 0 polls the z
    // granules of its K-slice (row 0; each granule = the WKV's bf16 / f16 hi | lo << 16 split of one
    // channel, so no re-split) and writes them as row 0 of the X image; rows past 0 are not staged
    static_assert(MT == 1 && XMODE == kXPlanes && KS == 128, "granule Wo role: one row, a 128-channel K-slice");
    hold_until(sy.d_late);
    load_w();
    if (threadIdx.x < 64) {
      const uint32_t tag = gran_tag(sy);
      const auto zr = wt_rsrc(sy.zgran);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t q0, q1;
      for (;;) {
        const u64x2_ qq = ld_gran2(zr, (kbeg + 2 * lane) * 8);
        q0 = qq.x;
        q1 = qq.y;
        const bool ok = (uint32_t)(q0 >> 32) == tag && (uint32_t)(q1 >> 32) == tag;
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
          if (lane == 0) __hip_atomic_fetch_or((gint_t*)sy.err, 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      const uint32_t g0 = (uint32_t)q0, g1 = (uint32_t)q1;  // {hi | lo << 16} of channels 2l, 2l + 1
      *(uint32_t*)(xh + 2 * lane) = (g0 & 0xFFFFu) | (g1 << 16);
      *(uint32_t*)(xl + 2 * lane) = (g0 >> 16) | (g1 & 0xFFFF0000u);
    }
    __syncthreads();
    sync_stamp(sy, 1);
  } else if constexpr (ROLE == 10) {
    // the head GEMM of a one-row step with ln_out fused (a plain launch): weights requested after
    // the row's inputs, the row's LayerNorm computed here (ln1024_body MODE 0's arithmetic: residual
    // + NP10 partial slabs in order, ln1024_apply) and this K-slice staged as row 0 of the X image
    static_assert(MT == 1 && XMODE == kXPlanes, "ln_out-fused head: one row, planes");
    constexpr int C = 1024, NP10 = 16;
    __shared__ float s_lnred10[16];
    const LnMixArgs& L = *lr;
    const int c = 4 * (int)threadIdx.x;
    float4_ v = ld4(L.h_in + c), tp[NP10];
#pragma unroll
    for (int p = 0; p < NP10; ++p) tp[p] = ld4(L.part + p * L.part_stride + c);
    const float4_ lw = ld4(L.ln_w + c), lb = ld4(L.ln_b + c);
    load_w();
#pragma unroll
    for (int p = 0; p < NP10; ++p) v += tp[p];
    ln1024_apply(v, lw, lb, s_lnred10, 0);
    if (c >= kbeg && c < kbeg + KS) {
      uint32_t h0, l0, h1, l1;
      split2<F16>(v[0], v[1], h0, l0);
      split2<F16>(v[2], v[3], h1, l1);
      *(uint2*)(xh + (c - kbeg)) = make_uint2(h0, h1);
      *(uint2*)(xl + (c - kbeg)) = make_uint2(l0, l1);
    }
    static_assert(C == 1024, "");
  } else if constexpr (ROLE == 5 || ROLE == 6) {
    static_assert(MT == 1 && XMODE == kXPlanes, "row-fused LayerNorm: one row, planes");
    // the row's LayerNorm (all 256 threads: thread t owns columns [4t, 4t + 4)), then this
    // K-slice's mix split into row 0 of the X image (rows 1..15 are never stored). The LayerNorm
    // inputs (L2 / MALL hits, written by the previous launch) are requested BEFORE the weight stream
    // (HBM, behind the launch-start burst): loads return in order, so the sums wait for these alone.
    constexpr int C = 1024, NPL = ROLE == 5 ? 16 : 8;
    __shared__ float s_lnred[16];
    const LnMixArgs& L = *lr;
    const int c = 4 * (int)threadIdx.x;
    const float* mup = L.mu[0];
    if constexpr (ROLE == 5) {
#pragma unroll
      for (int m = 1; m < 6; ++m)
        if (tile_mix == m) mup = L.mu[m];
    }
    float4_ v = ld4(L.h_in + c), tp[NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) tp[p] = ld4(L.part + p * L.part_stride + c);
    const float4_ lw = ld4(L.ln_w + c), lb = ld4(L.ln_b + c);
    load_w();
    // (after the weights: the token-shift row's address waits for the row descriptor)
    const int4 info = L.rows[0];
    const float4_ mu = ld4(mup + c);
    const float4_ pv = ld4(L.shift + (((int64_t)info.w * L.S + info.x) * L.L + L.layer) * C + c);
#pragma unroll
    for (int p = 0; p < NPL; ++p) v += tp[p];
    ln1024_apply(v, lw, lb, s_lnred, 0);
    if (c >= kbeg && c < kbeg + KS) {
      const float4_ x = v + (pv - v) * mu;
      uint32_t h0, l0, h1, l1;
      split2<F16>(x[0], x[1], h0, l0);
      split2<F16>(x[2], x[3], h1, l1);
      *(uint2*)(xh + (c - kbeg)) = make_uint2(h0, h1);
      *(uint2*)(xl + (c - kbeg)) = make_uint2(l0, l1);
    }
    sync_stamp(sy, 1);
  } else if constexpr (ROLE == 7) {
    // value workgroup of the granule form (one row): weights at dispatch, then wave 0 polls its
    // K-slice's key granules for row 0 -- lane l: columns kbeg + 4l .. + 3 of the NX key splits,
    // two 16-byte sc1 loads (4 granules) per split -- until every tag is this pass's; the row's
    // x chunks go where load_x would have put them (rows past 0 stay zero)
    static_assert(XMODE == kXRelu2 && NX == 4, "granule value role: the relu^2 X of four key splits");
    hold_until(sy.d_v);
    load_w();
#pragma unroll
    for (int p = 0; p < NX; ++p)
#pragma unroll
      for (int u = 0; u < PERR; ++u) xr[p][u] = (float4_){0.f, 0.f, 0.f, 0.f};
    if (wave == 0) {
      const uint32_t tag = gran_tag(sy);
      const auto gr = wt_rsrc(sy.gran);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int p = 0; p < NX; ++p) {
          // four granules {data | tag << 32} per split, two per volatile 16-byte load (ld_gran2)
          uint64_t q[4];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const u64x2_ qq = ld_gran2(gr, (p * sy.gran_ld + kbeg + 4 * lane + 2 * e) * 8);
            q[2 * e] = qq.x;
            q[2 * e + 1] = qq.y;
          }
          xr[p][0] = (float4_){__builtin_bit_cast(float, (uint32_t)q[0]), __builtin_bit_cast(float, (uint32_t)q[1]),
                               __builtin_bit_cast(float, (uint32_t)q[2]), __builtin_bit_cast(float, (uint32_t)q[3])};
#pragma unroll
          for (int e = 0; e < 4; ++e) ok = ok && (uint32_t)(q[e] >> 32) == tag;
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
          if (lane == 0) __hip_atomic_fetch_or((gint_t*)sy.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    sync_stamp(sy, 1);
  } else if constexpr (ROLE == 2) {
    if (sy.opts & 1)  // weights after the LN rows
      sync_wait(sy.cnt + kSyncStride * (blockIdx.x & (kLnReplicas - 1)), sy.ln_rows, sy.err, 4, sy.opts);
    hold_until(sy.d_v);
    load_w();
    sync_wait(sy.cnt + kSyncStride * (kLnReplicas + split), sy.key_per_slice, sy.err, 2, sy.opts);
    sync_stamp(sy, 1);
    load_x();
  } else {
    load_x();
    load_w();
  }
  for (;;) {
  // 3) X -> LDS (rows past M: zeros in the persistent roles (never fetched), a copy of row M-1 in the
  // plain launches; an MFMA output row depends on its own X row only, and those rows' outputs are not
  // stored)
  if constexpr (ROLE == 5 || ROLE == 6 || ROLE == 8 || ROLE == 10) {
    // (staged by the row-fused LayerNorm / the granule sweep above)
  } else if constexpr (XMODE == kXPlanes) {
#pragma unroll
    for (int u = 0; u < PERP; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      *(short8*)(xh + r * LD + k8) = vh[u];
      *(short8*)(xl + r * LD + k8) = vl[u];
    }
  } else {
    // relu(k)^2 can exceed the f16 range (65504) on real checkpoints: in the f16 model each row
    // of this K-slice is staged as relu^2 * 2^-e_r (e_r >= 0 the smallest power of two that
    // brings the row's maximum under 2^15) and its partial product is scaled back by 2^e_r in
    // the epilogue. Powers of two are exact, so rows in range (e_r = 0) are bit-unchanged.
    // (ROLE 7, one row: only row 0 is staged -- rows past M hold stale bytes, which no stored
    // output reads: an MFMA output row depends on its own X row only)
    float4_ y4[PERR];
#pragma unroll
    for (int u = 0; u < PERR; ++u) {
      if (ROLE == 7 && xrow0 + x_row(u) >= a.M) continue;
      float4_ x = xr[0][u];
#pragma unroll
      for (int p = 1; p < NX; ++p) x += xr[p][u];
#pragma unroll
      for (int e = 0; e < 4; ++e) y4[u][e] = x[e] > 0.f ? x[e] * x[e] : 0.f;
    }
    if constexpr (F16) {
      if (threadIdx.x < ROWS) s_rexp[threadIdx.x] = 0u;
      __syncthreads();
#pragma unroll
      for (int u = 0; u < PERR; ++u) {
        const int r = x_row(u);
        if (ROLE == 7 && xrow0 + r >= a.M) continue;
        const float m = fmaxf(fmaxf(y4[u][0], y4[u][1]), fmaxf(y4[u][2], y4[u][3]));
        if (m >= 32768.f) atomicMax(&s_rexp[r], as_u32(m));  // non-negative floats order as uints
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < PERR; ++u) {
      const int r = x_row(u), k4 = x_col(u);
      if (ROLE == 7 && xrow0 + r >= a.M) continue;
      float y[4] = {y4[u][0], y4[u][1], y4[u][2], y4[u][3]};
      if constexpr (F16) {
        const uint32_t mb = s_rexp[r];
        if (mb) {  // 2^-(E - 14) for a row maximum in [2^E, 2^(E+1)), E >= 15; inf stays inf
          const float sc = as_f32((uint32_t)(127 - (int)((mb >> 23) & 0xFF) + 127 + 14) << 23);
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] *= sc;
        }
      }
      uint32_t h0, l0, h1, l1;
      split2<F16>(y[0], y[1], h0, l0);
      split2<F16>(y[2], y[3], h1, l1);
      *(uint2*)(xh + r * LD + k4) = make_uint2(h0, h1);
      *(uint2*)(xl + r * LD + k4) = make_uint2(l0, l1);
    }
  }
  __syncthreads();
  const int rg_next = rg + (int)gridDim.z;
  if (!QW && rg_next < nrg) {  // the next row group's X, in flight during this group's MFMAs and stores
    xrow0 = rg_next * ROWS;
    load_x();
  }
  // 4) MFMA: hi and lo chains separate
  float4_ acc_h[MT], acc_l[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc_h[m] = acc_l[m] = (float4_){0.f, 0.f, 0.f, 0.f};
  if constexpr (QW) {
    if (qf) {
      // dequantise 8 weights per step, split w = hi + lo, three MFMAs per product (x_hi w_hi,
      // x_lo w_hi, x_hi w_lo): the dequantised weights enter at ~2^-16 relative
#pragma unroll
      for (int t = 0; t < KSTEPS; ++t) {
        float w[8];
        if (qf == 1) {
          const float mn = h16_to_f32((uint16_t)(qsc[t] & 0xFFFFu)), mx = h16_to_f32((uint16_t)(qsc[t] >> 16));
          const float step = (mx - mn) / 255.0f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t q = ((e < 4 ? bq8[t].x : bq8[t].y) >> (8 * (e & 3))) & 255u;
            w[e] = fmaf((float)q, step, mn);
          }
        } else {
          const float sc = h16_to_f32((uint16_t)qsc[t]);
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] = s_qlut[(bq4[t] >> (4 * e)) & 15u] * sc;
        }
        if constexpr (F16) {
          const float up = __builtin_amdgcn_ldexpf(1.0f, a.q_shift);
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] *= up;
        }
        uint32_t hh[4], ll[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split2<F16>(w[2 * e], w[2 * e + 1], hh[e], ll[e]);
        const short8 bh = __builtin_bit_cast(short8, (u32x4_){hh[0], hh[1], hh[2], hh[3]});
        const short8 bl = __builtin_bit_cast(short8, (u32x4_){ll[0], ll[1], ll[2], ll[3]});
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int o = (m * 16 + li) * LD + t * 32 + g * 8;
          const short8 ah = *(const short8*)(xh + o);
          const short8 al = *(const short8*)(xl + o);
          if constexpr (F16) {
            acc_h[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, bh), acc_h[m], 0, 0, 0);
            acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, al), __builtin_bit_cast(f16x8, bh), acc_l[m], 0, 0, 0);
            acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, bl), acc_l[m], 0, 0, 0);
          } else {
            acc_h[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, bh), acc_h[m], 0, 0, 0);
            acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al), __builtin_bit_cast(bf16x8, bh), acc_l[m], 0, 0, 0);
            acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, bl), acc_l[m], 0, 0, 0);
          }
        }
      }
    }
  }
  if (!qf) {
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int o = (m * 16 + li) * LD + t * 32 + g * 8;
      const short8 ah = *(const short8*)(xh + o);
      const short8 al = *(const short8*)(xl + o);
      if constexpr (F16) {
        acc_h[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, b[t]),
                                                          acc_h[m], 0, 0, 0);
        acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, al), __builtin_bit_cast(f16x8, b[t]),
                                                          acc_l[m], 0, 0, 0);
      } else {
        acc_h[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, b[t]),
                                                           acc_h[m], 0, 0, 0);
        acc_l[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al), __builtin_bit_cast(bf16x8, b[t]),
                                                           acc_l[m], 0, 0, 0);
      }
    }
  }
  }
  // 5) store (D layout: col = lane&15, row = 4*(lane>>4) + j)
  const int col = col0 + li;
  auto result = [&](int m, int j) {
    float v = acc_h[m][j] + acc_l[m][j];
    if constexpr (F16 && QW) {
      if (qf) v *= __builtin_amdgcn_ldexpf(1.0f, -a.q_shift);
    }
    if constexpr (F16 && XMODE == kXRelu2) {
      const uint32_t mb = s_rexp[m * 16 + 4 * g + j];
      if (mb) v *= as_f32((uint32_t)((int)((mb >> 23) & 0xFF) - 127 - 14 + 127) << 23);  // 2^(E - 14)
    }
    return v;
  };
  if (ROLE == 6 && sy.gran) {
    // granule form: row 0's 64 columns, one {f32, tag} granule per element (lanes 0..15 of each
    // wave hold row 0: g == 0, j == 0)
    if (g == 0 && col < Nn) gran_store(sy.gran + (int64_t)split * sy.gran_ld + col_off + col, result(0, 0), gran_tag(sy));
  } else if (a.wt) {
    // write-through: the tile is staged in LDS so every lane stores whole 16-byte pieces (a
    // 4-byte sc1 store is one fabric write each)
    constexpr int LDT = 68;
    float* st = (float*)smem;
    __syncthreads();  // every wave is done reading its X fragments
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[(m * 16 + 4 * g + j) * LDT + wave * 16 + li] = result(m, j);
    __syncthreads();
    const int tcol = (tile - tstart) * 64;  // first column of this tile within the segment
    const auto rs = wt_rsrc(e_out);
#pragma unroll
    for (int q = threadIdx.x; q < ROWS * 16; q += 256) {
      const int r = q >> 4, c4 = (q & 15) * 4, row = row0 + r;
      if (row >= e_M || tcol + c4 >= Nn) continue;
      const int64_t o = (int64_t)split * e_sstride + col_off + tcol + c4 + (int64_t)row * e_ldo;
      const float4_ v = *(const float4_*)(st + r * LDT + c4);
      if (tcol + c4 + 4 <= Nn && (o & 3) == 0) {
        store_wt(rs, (int)(o * 4), v);
      } else {
        for (int e = 0; e < 4 && tcol + c4 + e < Nn; ++e) store_wt(rs, (int)((o + e) * 4), v[e]);
      }
    }
  } else if (col < Nn) {
    float* out = e_out + split * e_sstride + col_off + col;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = row0 + m * 16 + 4 * g + j;
        if (row < e_M) out[(int64_t)row * e_ldo] = result(m, j);
      }
  }
  if (QW || rg_next >= nrg) break;
  rg = rg_next;
  row0 = rg * ROWS;
  __syncthreads();  // every wave is done with the LDS X image / store staging
  }
  if constexpr (ROLE != 0) sync_stamp(sy, 2);
  if constexpr (ROLE == 1) sync_arrive(sy.cnt + kSyncStride * (kLnReplicas + tile / sy.key_group));
  if constexpr (ROLE == 6) {  // K-slice counter (replica 0; not in the granule form) and key-done (lane 1)
    if (!sy.gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && !sy.gran)
      __hip_atomic_fetch_add((gint_t*)(sy.cnt + kSyncStride * (kLnReplicas + tile / sy.key_group)), 1,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 1)
      __hip_atomic_fetch_add((gint_t*)(sy.cnt + kSyncStride * kFfnKeyDone), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (ROLE == 3) {
    const int c0 = col_off + (tile - tstart) * 64;  // this tile's first output column
    if (c0 < 3 * sy.C) sync_arrive(sy.cnt + kSyncStride * (kAttHead + ((c0 % sy.C) >> 6)), 1, sy.drop);
    else sync_arrive(sy.cnt + kSyncStride * kAttLora, kLnReplicas);
  }
  if constexpr (ROLE == 5) {  // as ROLE 3, plus rkv-done (lane 8) for the shift writer
    const int c0 = col_off + (tile - tstart) * 64;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c0 < 3 * sy.C) {
      // (test hook as in sync_arrive: a workgroup that takes a pending drop skips its arrival)
      if (threadIdx.x == 0 && !(sy.drop && take_drop(sy.drop)))
        __hip_atomic_fetch_add((gint_t*)(sy.cnt + kSyncStride * (kAttHead + ((c0 % sy.C) >> 6))), 1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (threadIdx.x < kLnReplicas) {
      __hip_atomic_fetch_add((gint_t*)(sy.cnt + kSyncStride * (kAttLora + threadIdx.x)), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 8)
      __hip_atomic_fetch_add((gint_t*)(sy.cnt + kSyncStride * kAttRkvDone), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int MT, int KSTEPS, int XMODE, bool F16, int NX, int MS, bool QW = false>
__global__ __launch_bounds__(256) void k_gemm2(GemmArgs a) {
  tl_begin(a.tl);
  gemm2_body<MT, KSTEPS, XMODE, F16, NX, MS, QW, 0>(a, blockIdx.x, blockIdx.y, FfnSync{});
  tl_end(a.tl);
}

// Prefill (multi-row) planes GEMMs of one segment, NB 64-column tiles per workgroup: each staged X
// slice feeds NB x 64 columns instead of 64 (k_gemm2 re-reads a row group's X slice once per
// 64-column tile: for a 1280-row step's 64-tile FFN key GEMM that is 335 MB of MALL reads). Every
// output element takes k_gemm2's MFMA sequence (the hi and lo chains over the K-slice's 32-wide steps
// in order, hi + lo at the end), so the partial slabs are bit-identical; rows past M are copies of
// row M - 1 (as k_gemm2's plain launches) and are not stored.
template <int KSTEPS, bool F16, int NB>
__global__ __launch_bounds__(256) void k_gemm_wide(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int MT = 2, KS = KSTEPS * 32, LD = KS + 8, ROWS = MT * 16, CH = KS / 8, PERP = ROWS * CH / 256;
  constexpr int LDT = NB * 64 + 4;
  tl_begin(a.tl);
  bf16_t* xh = (bf16_t*)smem;
  bf16_t* xl = xh + ROWS * LD;
  const int split = blockIdx.y, kbeg = split * KS;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const GemmSeg& sg = a.seg[0];
  const bf16_t* Xhi = sg.Xhi;
  const bf16_t* Xlo = sg.Xlo;
  const int ldx = sg.ldx, Nn = sg.N, nblk = (Nn + 15) >> 4;
  const int colw = blockIdx.x * (NB * 64);  // the workgroup's first column within the segment
  const int nrg = (a.M + ROWS - 1) / ROWS;
  int rg = blockIdx.z;
  short8 vh[PERP], vl[PERP];
  auto load_x = [&](int rg_) {
#pragma unroll
    for (int u = 0; u < PERP; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      const int64_t o = (int64_t)min(rg_ * ROWS + r, a.M - 1) * ldx + kbeg + k8;
      vh[u] = *(const short8*)(Xhi + o);
      vl[u] = *(const short8*)(Xlo + o);
    }
  };
  load_x(rg);
  short8 b[NB][KSTEPS];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int nb = min((colw + j * 64 + wave * 16) >> 4, nblk - 1);
    const bf16_t* wp = sg.W + (((int64_t)nb * (a.K >> 5) + (kbeg >> 5)) * 64 + lane) * 8;
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t) b[j][t] = __builtin_nontemporal_load((const short8*)(wp + t * 512));
  }
  for (;;) {
    const int row0 = rg * ROWS;
#pragma unroll
    for (int u = 0; u < PERP; ++u) {
      const int c = threadIdx.x + u * 256;
      const int r = c / CH, k8 = (c % CH) * 8;
      *(short8*)(xh + r * LD + k8) = vh[u];
      *(short8*)(xl + r * LD + k8) = vl[u];
    }
    __syncthreads();
    const int rg_next = rg + (int)gridDim.z;
    if (rg_next < nrg) load_x(rg_next);  // in flight during this group's MFMAs and stores
    float4_ acc_h[NB][MT], acc_l[NB][MT];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc_h[j][m] = acc_l[j][m] = (float4_){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int o = (m * 16 + li) * LD + t * 32 + g * 8;
        const short8 ah = *(const short8*)(xh + o);
        const short8 al = *(const short8*)(xl + o);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (F16) {
            acc_h[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah),
                                                                 __builtin_bit_cast(f16x8, b[j][t]), acc_h[j][m], 0, 0, 0);
            acc_l[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, al),
                                                                 __builtin_bit_cast(f16x8, b[j][t]), acc_l[j][m], 0, 0, 0);
          } else {
            acc_h[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah),
                                                                  __builtin_bit_cast(bf16x8, b[j][t]), acc_h[j][m], 0, 0, 0);
            acc_l[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al),
                                                                  __builtin_bit_cast(bf16x8, b[j][t]), acc_l[j][m], 0, 0, 0);
          }
        }
      }
    }
    // store: the tile staged in LDS (D layout: col = lane & 15, row = 4 (lane >> 4) + jj), then whole
    // 16-byte pieces per lane (write-through where asked, as k_gemm2)
    float* st = (float*)smem;
    __syncthreads();  // every wave is done reading its X fragments
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          st[(m * 16 + 4 * g + jj) * LDT + j * 64 + wave * 16 + li] = acc_h[j][m][jj] + acc_l[j][m][jj];
    __syncthreads();
    float* outp = a.out + (int64_t)split * a.split_stride + sg.col_off;
    const auto rs = wt_rsrc(a.out);
    for (int q = threadIdx.x; q < ROWS * NB * 16; q += 256) {
      const int r = q / (NB * 16), c4 = (q % (NB * 16)) * 4, row = row0 + r, col = colw + c4;
      if (row >= a.M || col >= Nn) continue;
      const int64_t o = (int64_t)row * a.ldo + col;
      const float4_ v = *(const float4_*)(st + r * LDT + c4);
      float* dst = outp + o;
      if (a.wt) {
        const int64_t ob = dst - a.out;  // element offset from the buffer start
        if (col + 4 <= Nn && (ob & 3) == 0) {
          store_wt(rs, (int)(ob * 4), v);
        } else {
          for (int e = 0; e < 4 && col + e < Nn; ++e) store_wt(rs, (int)((ob + e) * 4), v[e]);
        }
      } else {
        for (int e = 0; e < 4 && col + e < Nn; ++e) dst[e] = v[e];
      }
    }
    if (rg_next >= nrg) break;
    rg = rg_next;
    __syncthreads();  // every wave is done with the LDS X image / store staging
  }
  tl_end(a.tl);
}

// the head GEMM of a one-row step with ln_out folded in (gemm2_body ROLE 10): one launch and one
// launch boundary fewer per step; logits bit for bit those of ln_out + k_gemm2
template <bool F16>
__global__ __launch_bounds__(256) void k_gemm2_lnrow(GemmArgs a, LnMixArgs lo) {
  tl_begin(a.tl);
  gemm2_body<1, 16, kXPlanes, F16, 1, 0, false, 10>(a, blockIdx.x, blockIdx.y, FfnSync{}, &lo);
  tl_end(a.tl);
}

bool launch_gemm_lnrow(const GemmArgs& a, const LnMixArgs& lo, hipStream_t st) {
  // one row, the head's shape: one segment of 16-bit planes, 512-wide K-slices, no XCD remap;
  // ln_out's: C = 1024, 16 partial slabs, no row remap beyond row 0
  if (a.M != 1 || a.nseg != 1 || a.kslice != 512 || a.xmode != kXPlanes || a.q_fmt || a.stamps ||
      a.allow_xmap || a.xalign > 0 || lo.C != 1024 || lo.n_part != 16 || lo.n_mix != 1 || lo.h_out != nullptr ||
      a.f16 != lo.f16)
    return false;
  const int tiles = (a.seg[0].N + 63) / 64;
  GemmArgs b = a;
  b.xmap = 0;
  const size_t lds = (size_t)16 * (16 * 32 + 8) * 2 * 2;
  if (a.f16) RT_LAUNCH((k_gemm2_lnrow<true>), dim3(tiles, a.k_split, 1), dim3(256), lds, st, b, lo);
  else RT_LAUNCH((k_gemm2_lnrow<false>), dim3(tiles, a.k_split, 1), dim3(256), lds, st, b, lo);
  return true;
}

// ------------------------------------------------------------------------------------
// ffn_persist: the whole FFN half of a decode step's layer as ONE launch:
//   blocks [0, n_ln_blocks)            LayerNorm 2 + token-shift mix of row b (k_ln1024's
//                                      arithmetic), planes / residual / shift stored
//                                      write-through, then counted into cnt[0];
//   blocks [+0, +n_key)                key GEMM workgroups (consumer-aligned order): weight
//                                      fragments requested at dispatch, wait for all LN rows,
//                                      X planes by sc1 loads, MFMA, partial slab written through,
//                                      counted into their value K-slice's counter;
//   blocks [+n_key, +n_key + 256)      value GEMM workgroups (XCD-aware order): weights at
//                                      dispatch, wait for the K-slice's key slabs, relu^2 staging
//                                      from sc1 loads, MFMA, partial slab out.
// Every dependency points to a lower block index, so in-order dispatch keeps every waited-on
// producer resident or finished (no deadlock with other kernels on the GPU). Every output is the
// three-launch path's, bit for bit (same bodies, same orders). Block 0 zeroes the counters of
// the previously launched layer (that launch has finished: stream order).
// ------------------------------------------------------------------------------------
// FUSED (row-fused form, one decode row): no LayerNorm blocks; key workgroups compute the row's LN2
// themselves (gemm2_body ROLE 6); the last workgroup (after the value ones) waits until every key
// workgroup has staged (kFfnKeyDone) and stores the residual and the new token-shift row.
// Workgroups per CU the persistent kernels' register budgets are sized for (2: 256 VGPRs, two waves
// per SIMD; 3 caps a kernel at 168 VGPRs so that three workgroups are resident per CU).
#ifndef RWKVTTS_FFN_WPC
#define RWKVTTS_FFN_WPC 2
#endif
#ifndef RWKVTTS_ATT_WPC
#define RWKVTTS_ATT_WPC 2
#endif
template <bool F16, bool FUSED>
__global__ __launch_bounds__(256, RWKVTTS_FFN_WPC) void k_ffn_persist(LnMixArgs ln, GemmArgs ka, GemmArgs va, FfnSync sy) {
  int b = blockIdx.x;
  tl_begin(ln.tl);
  sync_stamp(sy, 0);
  // (the previous layer's counters are zeroed inside a role branch -- LayerNorm block 0, or the
  // row-fused form's shift writer: a test ahead of the branch made every workgroup wait for its
  // kernel arguments first, 2 % of the 32-row decode step)
  if (b < sy.n_ln_blocks) {
    if (b == 0 && threadIdx.x < sy.n_prev) sy.cnt_prev[threadIdx.x * kSyncStride] = 0;
    if (b < sy.ln_rows) {
      ln1024_body<F16, 1, 1, 8>(ln, b);
      sync_stamp(sy, 2);
      sync_arrive(sy.cnt, kLnReplicas);
    }
  } else if ((b -= sy.n_ln_blocks) < sy.n_key) {
    if constexpr (FUSED) gemm2_body<1, 8, kXPlanes, F16, 1, 0, false, 6>(ka, b, 0, sy, &ln);
    else gemm2_body<2, 8, kXPlanes, F16, 1, 0, false, 1>(ka, b, 0, sy);
  } else if ((b -= sy.n_key) < sy.n_val || !FUSED) {
    if constexpr (FUSED) {
      if (sy.gran) gemm2_body<1, 8, kXRelu2, F16, 4, 0, false, 7>(va, b, 0, sy);  // (one row: 16-row tile)
      else gemm2_body<2, 8, kXRelu2, F16, 4, 0, false, 2>(va, b, 0, sy);
    } else {
      gemm2_body<2, 8, kXRelu2, F16, 4, 0, false, 2>(va, b, 0, sy);
    }
  } else if constexpr (FUSED) {  // the shift writer
    if (threadIdx.x < sy.n_prev) sy.cnt_prev[threadIdx.x * kSyncStride] = 0;
    sync_wait(sy.cnt + kSyncStride * kFfnKeyDone, sy.n_key, sy.err, 1024, sy.opts);
    ln1024_body<F16, 1, 0, 8>(ln, 0);
  }
  sync_stamp(sy, 3);
  tl_end(ln.tl);
}

// ------------------------------------------------------------------------------------
// wkv: one workgroup per (slot segment, head); rows of the segment run in order.
//   part columns: [0,C) r | [C,2C) k | [2C,3C) v | [3C, 3C+Dw) w-hidden | +Da a-hidden |
//   +Dv v-hidden | +Dg g-hidden   (split-K partial slabs, summed in fixed order here)
//   Thread t holds S[i = t>>2][16*(t&3) .. +16] of the head's 64x64 state in registers.
// ------------------------------------------------------------------------------------
__device__ inline float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }


// MAXL: 8-byte LoRA-up weight units per thread (>= (Dw + Da + Dv + Dg) / 16);
// MAXP: split-K slabs summed per row (>= n_part).
template <int MAXL, int MAXP>
__global__ __launch_bounds__(256, 2) void k_wkv(WkvArgs a) {
  constexpr int N = 64;
  __shared__ __attribute__((aligned(16))) float s_hid[kMaxLoraTotal];
  __shared__ float s_r[N], s_k[N], s_v[N], s_w[N], s_kk[N], s_b[N], s_g[N], s_y[N];
  __shared__ float s_red[2][4];
  uint64_t* stp = (a.stamps && threadIdx.x == 0) ? a.stamps + (blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
#define WKV_STAMP(k) \
  if (stp) stp[k] = __builtin_amdgcn_s_memtime();
  WKV_STAMP(0)
  // segs first: it heads the longest dependent chain (segs -> state / partials)
  const int4 sg = a.segs[blockIdx.x];
  const int h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = a.C;
  const int c = h * N + lane;  // this lane's channel (waves 0..3 all index the head's channels)
  const int i = tid >> 2, jq = (tid & 3) * 16;
  // ---- LoRA-up weights, straight to registers: thread (cc = tid >> 2, pq = tid & 3) owns
  // quarter pq of channel cc's rows of w2t | a2t | v2t | g2t (D/4 each), pre-packed into one
  // contiguous run; these loads depend only on the head, so they are in flight with segs.
  const int cc = tid >> 2, pq = tid & 3;
  const int Dq0 = a.Dw / 4, Dq1 = a.Da / 4, Dq2 = a.Dv / 4, Dq3 = a.Dg / 4;
  const int e1 = Dq0, e2 = Dq0 + Dq1, e3 = Dq0 + Dq1 + Dq2, eq = e3 + Dq3;  // quarter-vector bounds
  uint2 lw[MAXL];
  {
    const bf16_t* src = a.lup + ((int64_t)(h * N + cc) * 4 + pq) * eq;  // one contiguous run
#pragma unroll
    for (int u = 0; u < MAXL; ++u) lw[u] = (u * 4 < eq) ? *(const uint2*)(src + u * 4) : make_uint2(0u, 0u);
  }
  // per-channel parameters: the 4 lanes of channel-owner group cc (all waves) hold channel
  // h*N + cc; wave 0 lane l also holds channel h*N + l for the GroupNorm
  const int co = h * N + cc;
  const float w0 = a.w0[co], a0 = a.a0[co], v0 = a.v0[co], kkc = a.k_k[co], kac = a.k_a[co];
  const float rkc = a.r_k[co];
  float lnw = 0.f, lnb = 0.f;
  if (wave == 0) {
    lnw = a.lnx_w[c]; lnb = a.lnx_b[c];
  }
  // ---- segs-dependent loads: the slot's state tile and the first row's split-K partials
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  float* Sg = a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N + i * N + jq;
  float S[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4_ v4 = *(const float4_*)(Sg + q * 4);
    S[q * 4 + 0] = v4[0]; S[q * 4 + 1] = v4[1]; S[q * 4 + 2] = v4[2]; S[q * 4 + 3] = v4[3];
  }
  const int Dall = a.Dw + a.Da + a.Dv + a.Dg;
  const int Dtot = Dall;
  float hp0[MAXP], hp1[MAXP], rp[MAXP], kp[MAXP], vp[MAXP], vf = 0.f;
  auto load_parts = [&](int row) {
    const float* prow = a.part + (int64_t)row * a.ldp;
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      const float* pp = prow + p * a.part_stride;
      const bool on = p < a.n_part;
      hp0[p] = (on && tid < Dtot) ? pp[3 * C + tid] : 0.f;
      hp1[p] = (on && tid + 256 < Dtot) ? pp[3 * C + tid + 256] : 0.f;
      rp[p] = on ? pp[co] : 0.f;
      kp[p] = on ? pp[C + co] : 0.f;
      vp[p] = on ? pp[2 * C + co] : 0.f;
    }
    vf = a.layer > 0 ? a.v_first[(int64_t)row * a.ldv + co] : 0.f;
  };
  load_parts(r_begin);
  const int hb1 = a.Dw, hb2 = a.Dw + a.Da, hb3 = a.Dw + a.Da + a.Dv;  // s_hid bases per matrix
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    if (rr == 1) { WKV_STAMP(6) }
    if (rr == 2) { WKV_STAMP(7) }
    if (rr > 0) load_parts(row);
    float hx0 = 0.f, hx1 = 0.f, r = 0.f, k = 0.f, v = 0.f;
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      hx0 += hp0[p];
      hx1 += hp1[p];
      r += rp[p];
      k += kp[p];
      v += vp[p];
    }
    // LoRA hidden activations, stored quarter-major: quarter pq of every matrix is one
    // contiguous run s_hq[pq * eq + (w | a | v | g offset) + i], read with uniform stride below
    auto put_hid = [&](int d, float x) {
      int dl, dq, eb;
      float y;
      if (d < hb1) { dl = d; dq = Dq0; eb = 0; y = tanhf(x); }
      else if (d < hb2) { dl = d - hb1; dq = Dq1; eb = e1; y = x; }
      else if (d < hb3) { dl = d - hb2; dq = Dq2; eb = e2; y = x; }
      else { dl = d - hb3; dq = Dq3; eb = e3; y = sigm(x); }
      if (dq > 0) {
        const int qt = dl / dq;
        s_hid[qt * eq + eb + (dl - qt * dq)] = y;
      }
    };
    if (tid < Dtot) put_hid(tid, hx0);
    if (tid + 256 < Dtot) put_hid(tid + 256, hx1);
    __syncthreads();
    if (rr == 0) { WKV_STAMP(1) }
    // ---- LoRA up (branch-free, every LDS read independent) + this channel's mixing terms
    float lo0 = 0.f, lo1 = 0.f, lo2 = 0.f, lo3 = 0.f;
    {
      const float* hq = s_hid + pq * eq;
#pragma unroll
      for (int u = 0; u < MAXL; ++u) {
        const int e = u * 4;
        if (e < eq) {  // uniform
          const float4_ hv = *(const float4_*)(hq + e);
          const uint2 q = lw[u];
          const bool f16 = a.f16 != 0;
          const float d = w16_to_f32((uint16_t)(q.x & 0xFFFF), f16) * hv[0] + w16_to_f32((uint16_t)(q.x >> 16), f16) * hv[1] +
                          w16_to_f32((uint16_t)(q.y & 0xFFFF), f16) * hv[2] + w16_to_f32((uint16_t)(q.y >> 16), f16) * hv[3];
          lo0 += e < e1 ? d : 0.f;
          lo1 += (e >= e1 && e < e2) ? d : 0.f;
          lo2 += (e >= e2 && e < e3) ? d : 0.f;
          lo3 += e >= e3 ? d : 0.f;
        }
      }
      lo0 += dpp_mov<0xB1>(lo0); lo0 += dpp_mov<0x4E>(lo0);
      lo1 += dpp_mov<0xB1>(lo1); lo1 += dpp_mov<0x4E>(lo1);
      lo2 += dpp_mov<0xB1>(lo2); lo2 += dpp_mov<0x4E>(lo2);
      lo3 += dpp_mov<0xB1>(lo3); lo3 += dpp_mov<0x4E>(lo3);
    }
    {
      const float w = expf(-0.60653066f * sigm(w0 + lo0));
      const float av = sigm(a0 + lo1);
      const float kk = k * kkc;
      const float kn = k * (1.0f + (av - 1.0f) * kac);
      float vn = v;
      if (a.layer == 0) {
        if (pq == 0) a.v_first[(int64_t)row * a.ldv + co] = v;
      } else {
        vn = v + (vf - v) * sigm(v0 + lo2);
      }
      // per-wave partial sums over its 16 channels: |kk|^2 and the bonus sum r*k*r_k
      const float ksq = wave_sum(pq == 0 ? kk * kk : 0.f);
      const float bon = wave_sum(pq == 0 ? r * kn * rkc : 0.f);
      if (lane == 0) { s_red[0][wave] = ksq; s_red[1][wave] = bon; }
      if (pq == 0) {
        s_r[cc] = r; s_k[cc] = kn; s_v[cc] = vn; s_w[cc] = w; s_kk[cc] = kk; s_b[cc] = av; s_g[cc] = lo3;
      }
    }
    __syncthreads();
    if (rr == 0) { WKV_STAMP(2) }
    const float nrm = fmaxf(sqrtf(((s_red[0][0] + s_red[0][1]) + s_red[0][2]) + s_red[0][3]), 1e-12f);
    if (rr == 0) { WKV_STAMP(3) }
    // ---- state update: S[i][j] = S[i][j]*w_j - sa_i*b_j + v_i*k_j ; y_i = sum_j S[i][j] r_j
    float kkn[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) kkn[q] = s_kk[jq + q] / nrm;
    float sa = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sa += S[q] * kkn[q];
    sa += dpp_mov<0xB1>(sa);
    sa += dpp_mov<0x4E>(sa);
    const float vi = s_v[i];
    float y = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int jj = jq + q;
      S[q] = S[q] * s_w[jj] - sa * (kkn[q] * s_b[jj]) + vi * s_k[jj];
      y += S[q] * s_r[jj];
    }
    y += dpp_mov<0xB1>(y);
    y += dpp_mov<0x4E>(y);
    if ((tid & 3) == 0) s_y[i] = y;
    __syncthreads();
    if (rr == 0) { WKV_STAMP(4) }
    if (wave == 0) {
      const float yv = s_y[lane];
      const float mean = wave_sum(yv) * (1.0f / N);
      const float dv = yv - mean;
      const float var = wave_sum(dv * dv) * (1.0f / N);
      const float rstd = 1.0f / sqrtf(var + 64e-5f);
      const float bonus = ((s_red[1][0] + s_red[1][1]) + s_red[1][2]) + s_red[1][3];
      const float gn = dv * rstd * lnw + lnb;
      split_store((gn + bonus * s_v[lane]) * s_g[lane], a.z_hi, a.z_lo, (int64_t)row * a.ldz + c, a.f16 != 0);
    }
    if (rr == 0) { WKV_STAMP(5) }
    if (rr + 1 < n_rows) __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4_ v4 = {S[q * 4 + 0], S[q * 4 + 1], S[q * 4 + 2], S[q * 4 + 3]};
    *(float4_*)(Sg + q * 4) = v4;
  }
  if (n_rows == 1) { WKV_STAMP(6) }
#undef WKV_STAMP
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
void launch_embed(const uint32_t* tokens, const int4* rows, const int* ctrl_tok, int ctrl_stride,
                  const bf16_t* emb, const float* w, const float* b, float* h, int R, int C, int f16, hipStream_t st,
                  unsigned long long* tl, int n_vocab) {
  RT_LAUNCH(k_embed, dim3(R), dim3(256), 0, st, tokens, rows, ctrl_tok, ctrl_stride, emb, w, b, h, C, f16, tl,
                     n_vocab);
}
int launch_ln_mix(const LnMixArgs& a, int n_out_rows, hipStream_t st) {
  LnMixArgs b = a;
  b.n_rows = n_out_rows;
  const dim3 grid(n_out_rows);
  if (a.emb) {  // layer 0 of a decode step with the embedding fused in
    if (!(a.C == 1024 && a.shift && a.n_mix == 6 && a.n_part == 0)) return -1;
    if (a.f16) RT_LAUNCH((k_ln1024<true, 1, 6, 0, true>), grid, dim3(256), 0, st, b);
    else RT_LAUNCH((k_ln1024<false, 1, 6, 0, true>), grid, dim3(256), 0, st, b);
    return n_out_rows;
  }
  if (a.C == 1024 && (a.shift ? (a.n_mix == 6 || a.n_mix == 1) : true) &&
      (a.n_part == 0 || a.n_part == 8 || a.n_part == 16)) {
#define LN_CASE(F, MO, NM)                                                                                  \
  switch (a.n_part) {                                                                                      \
    case 0: RT_LAUNCH((k_ln1024<F, MO, NM, 0>), grid, dim3(256), 0, st, b); break;                \
    case 8: RT_LAUNCH((k_ln1024<F, MO, NM, 8>), grid, dim3(256), 0, st, b); break;                \
    default: RT_LAUNCH((k_ln1024<F, MO, NM, 16>), grid, dim3(256), 0, st, b); break;              \
  }
    if (a.f16) {
      if (!a.shift) { LN_CASE(true, 0, 0) } else if (a.n_mix == 6) { LN_CASE(true, 1, 6) } else { LN_CASE(true, 1, 1) }
    } else {
      if (!a.shift) { LN_CASE(false, 0, 0) } else if (a.n_mix == 6) { LN_CASE(false, 1, 6) } else { LN_CASE(false, 1, 1) }
    }
#undef LN_CASE
    return n_out_rows;
  }
  if (a.C <= 1024) {
    switch (a.n_part) {  // slab counts of the 0.4B configuration: every load in flight at once
      case 0: RT_LAUNCH((k_ln_mix<1, 0>), grid, dim3(256), 0, st, b); break;
      case 8: RT_LAUNCH((k_ln_mix<1, 8>), grid, dim3(256), 0, st, b); break;
      case 16: RT_LAUNCH((k_ln_mix<1, 16>), grid, dim3(256), 0, st, b); break;
      default: RT_LAUNCH((k_ln_mix<1, -1>), grid, dim3(256), 0, st, b); break;
    }
  } else {
    RT_LAUNCH((k_ln_mix<2, -1>), grid, dim3(256), 0, st, b);
  }
  return n_out_rows;
}

template <int MT, int KSTEPS>
static void launch_gemm_t(const GemmArgs& a, dim3 grid, hipStream_t st) {
  const size_t lds = (size_t)MT * 16 * (KSTEPS * 32 + 8) * 2 * 2;
  // k_gemm2 (fragment-packed weights, per-tile descriptors) covers the 0.4B shapes; k_gemm is the
  // generic fallback (other slab counts) and the debug-stamp build
  // (quantised weights exist only in k_gemm2: debug stamps / experiments are ignored for them)
  const bool nx_ok = a.x_nsplit == 4 || a.x_nsplit == 2 || (a.x_nsplit == 1 && a.q_fmt);
  if ((a.xmode == kXPlanes || nx_ok) && (a.stamps == nullptr || a.q_fmt)) {
    const int ms = a.nseg > 1 ? (a.n_tinfo > 0 ? 2 : 1) : 0;
    GemmArgs b = a;
    b.xmap = 0;
    if (grid.z == 1 && a.xalign > 0) {
      b.xmap = 2;
      b.ntiles = (int)grid.x;
      const int groups = ((int)grid.x + a.xalign - 1) / a.xalign;
      grid = dim3(8 * ((groups + 7) / 8) * a.xalign * a.k_split);
    } else if (grid.z == 1 && a.allow_xmap && (a.k_split % 8 == 0 || 8 % a.k_split == 0)) {
      b.xmap = 1;
      b.ntiles = (int)grid.x;
      if (a.k_split >= 8) {
        grid = dim3(grid.x * a.k_split);
      } else {
        b.tiles_per_xcd = (int)((grid.x * a.k_split + 7) / 8);
        grid = dim3(8 * b.tiles_per_xcd);
      }
    }
    // prefill steps of one segment with planes X (FFN key / value, Wo): k_gemm_wide, several
    // 64-column tiles per workgroup (bit-identical slabs)
    // (KSTEPS 8: the FFN key / value GEMMs, 47 -> 42 us per launch on a 1280-row step; the Wo GEMM's
    // 4-step slices measured 18 -> 19 us at four tiles per workgroup and keep k_gemm2)
    constexpr int kWideNB = 2;
    if constexpr (MT == 2 && KSTEPS == 8) {
    if (grid.z > 1 && !a.q_fmt && a.xmode == kXPlanes && a.nseg == 1 && a.seg[0].tile_start == 0 &&
        (int)grid.x % kWideNB == 0 && b.xmap == 0) {
      dim3 gw((int)grid.x / kWideNB, grid.y, grid.z);
      const int rpw = std::max(1, (int)gw.z * (int)(gw.x * gw.y) / 1024);
      gw.z = (gw.z + rpw - 1) / rpw;
      const size_t lw = std::max(lds, (size_t)MT * 16 * (kWideNB * 64 + 4) * 4);
      if (a.f16) RT_LAUNCH((k_gemm_wide<KSTEPS, true, kWideNB>), gw, dim3(256), lw, st, b);
      else RT_LAUNCH((k_gemm_wide<KSTEPS, false, kWideNB>), gw, dim3(256), lw, st, b);
      return;
    }
    }
    // prefill steps: several row groups per workgroup (weights loaded once), as many as keep >= 4
    // workgroups per CU (measured over 1 / 2 / 4 / 8 / 10 / 20 / 40 groups per workgroup on a
    // 1280-row step: 9.3 / 8.5 / 8.3 / 8.1 / 8.1 / 8.0 / 10.0 ms)
    if (grid.z > 1 && !a.q_fmt) {
      const int per_group = (int)(grid.x * grid.y);
      const int rpw = std::max(1, (int)grid.z * per_group / 1024);
      grid.z = (grid.z + rpw - 1) / rpw;
    }
#define G2(F, XM, NX_, MS_)                                                               \
  do {                                                                                    \
    if (b.q_fmt) RT_LAUNCH((k_gemm2<MT, KSTEPS, XM, F, NX_, MS_, true>), grid, dim3(256), lds, st, b); \
    else RT_LAUNCH((k_gemm2<MT, KSTEPS, XM, F, NX_, MS_>), grid, dim3(256), lds, st, b);  \
  } while (0)
    if (a.f16) {
      if (a.xmode == kXPlanes) { if (ms == 2) G2(true, kXPlanes, 1, 2); else if (ms == 1) G2(true, kXPlanes, 1, 1); else G2(true, kXPlanes, 1, 0); }
      else if (a.x_nsplit == 4) G2(true, kXRelu2, 4, 0);
      else if (a.x_nsplit == 2) G2(true, kXRelu2, 2, 0);
      else G2(true, kXRelu2, 1, 0);
    } else {
      if (a.xmode == kXPlanes) { if (ms == 2) G2(false, kXPlanes, 1, 2); else if (ms == 1) G2(false, kXPlanes, 1, 1); else G2(false, kXPlanes, 1, 0); }
      else if (a.x_nsplit == 4) G2(false, kXRelu2, 4, 0);
      else if (a.x_nsplit == 2) G2(false, kXRelu2, 2, 0);
      else G2(false, kXRelu2, 1, 0);
    }
#undef G2
    return;
  }
  if (a.f16) {
    if (a.xmode == kXPlanes) RT_LAUNCH((k_gemm<MT, KSTEPS, kXPlanes, true>), grid, dim3(256), lds, st, a);
    else RT_LAUNCH((k_gemm<MT, KSTEPS, kXRelu2, true>), grid, dim3(256), lds, st, a);
  } else {
    if (a.xmode == kXPlanes) RT_LAUNCH((k_gemm<MT, KSTEPS, kXPlanes, false>), grid, dim3(256), lds, st, a);
    else RT_LAUNCH((k_gemm<MT, KSTEPS, kXRelu2, false>), grid, dim3(256), lds, st, a);
  }
}

// Prefill steps (bf16 models): relu(sum of the key GEMM's NX partial slabs)^2 as bf16 hi/lo planes
// once, so the value GEMM stages 4-byte plane pairs instead of re-reading NX f32 slabs in every
// one of its column tiles. Same sum order and split as k_gemm2's kXRelu2 staging: bit-identical.
__global__ __launch_bounds__(256) void k_relu2_planes(const float* part, int nx, int64_t pstride, int ld, int F,
                                                      bf16_t* hi, bf16_t* lo) {
  const int row = blockIdx.y, c = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (c >= F) return;
  const int64_t o = (int64_t)row * ld + c;
  float4_ x = *(const float4_*)(part + o);
  for (int p = 1; p < nx; ++p) x += *(const float4_*)(part + p * pstride + o);
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = x[e] > 0.f ? x[e] * x[e] : 0.f;
  uint32_t h0, l0, h1, l1;
  split2<false>(y[0], y[1], h0, l0);
  split2<false>(y[2], y[3], h1, l1);
  const int64_t q = (int64_t)row * F + c;
  *(uint2*)(hi + q) = make_uint2(h0, h1);
  *(uint2*)(lo + q) = make_uint2(l0, l1);
}
void launch_relu2_planes(const float* part, int nx, int64_t pstride, int ld, int F, int R, bf16_t* hi, bf16_t* lo,
                         hipStream_t st) {
  RT_LAUNCH(k_relu2_planes, dim3((F / 4 + 255) / 256, R), dim3(256), 0, st, part, nx, pstride, ld, F, hi, lo);
}

// The FFN half of a decode step as one launch (k_ffn_persist); false: a shape it does not cover
// (the caller runs the three launches). ln / key / val: the three launches' arguments as built by
// the engine; cnt / cnt_prev: this and the previous layer's counter blocks ((1 + kFfnSlices) x
// kSyncStride ints, zero before this layer's first use); err: the give-up word.
// Holds of the dispatch-time prefetches (FfnSync::d_w / d_k / d_late / d_s / d_v, 10 ns ticks).
// The rkv / key weight streams wait 1 us, so the LayerNorm rows at the head of each persistent
// launch load their slabs with less traffic beside them while the weights still land before the
// LayerNorm ends (same-box decode A/B at B = 32: 771-776 -> 756-764 us per step, tokens unchanged;
// holding the value / Wo weights or the WKV state is slower, profiles/r04h_pf_hold_ab.txt).
constexpr int kHoldRkv = 100, kHoldKey = 100;
// The row-fused (one-row) forms hold the Wo and the FFN value weight streams instead (the rkv /
// key ones feed the first GEMM there): 4 / 1 us (same-box B = 1 A/B: 525 -> 513-517 us per step,
// round 5, profiles/r05u_holds1_ab.txt).
constexpr int kHold1Wo = 400, kHold1Value = 100;
static void prefetch_holds(FfnSync& sy) {
  sy.d_w = kHoldRkv;
  sy.d_late = 0;
  sy.d_s = 0;
  sy.d_v = 0;
  sy.d_k = kHoldKey;
}

struct FfnPrep {
  LnMixArgs l;
  GemmArgs ka, va;
  FfnSync sy;
  int nv;
};
static bool prep_ffn_persist(const LnMixArgs& ln, const GemmArgs& key, const GemmArgs& val, int* cnt, int* cnt_prev,
                             int* err, int R, uint64_t* stamps, int opts, FfnPrep& P) {
  if (ln.C != 1024 || !ln.shift || ln.n_mix != 1 || ln.n_part != 8 || ln.emb || R < 1 || R > 32 ||
      key.xmode != kXPlanes || val.xmode != kXRelu2 || val.x_nsplit != 4 || key.kslice != 256 ||
      val.kslice != 256 || key.M != R || val.M != R || key.nseg != 1 || val.nseg != 1 || key.q_fmt || val.q_fmt ||
      key.stamps || val.stamps || key.xalign <= 0 || key.f16 != val.f16 || key.f16 != ln.f16 ||
      cnt == cnt_prev)
    return false;
  const int kt = (key.seg[0].N + 63) / 64, vt = (val.seg[0].N + 63) / 64;
  const int groups = kt / key.xalign;
  // no padding blocks (every value K-slice gets exactly xalign x k_split producers; key tile t
  // belongs to K-slice t / xalign), the value grid's XCD order (split = xcd + 8 j) needs
  // k_split % 8 == 0, and the counters cover kFfnSlices K-slices
  if (kt % key.xalign || groups % 8 || groups != val.k_split || val.k_split % 8 || val.k_split > kFfnSlices ||
      key.xalign * 64 != val.kslice)
    return false;
  LnMixArgs& l = P.l;
  l = ln;
  l.n_rows = R;
  l.wt = 1;
  GemmArgs& ka = P.ka;
  GemmArgs& va = P.va;
  ka = key;
  va = val;
  ka.xmap = 2; ka.ntiles = kt; ka.wt = 1;
  va.xmap = 1; va.ntiles = vt;
  FfnSync& sy = P.sy;
  sy = FfnSync{};
  sy.cnt = cnt;
  sy.cnt_prev = cnt_prev;
  sy.err = err;
  sy.n_ln_blocks = 32;  // rows padded to 32 (a multiple of 8: the GEMM blocks keep their XCD order)
  sy.ln_rows = R;
  sy.n_key = kt * key.k_split;
  sy.key_group = key.xalign;
  sy.key_per_slice = key.xalign * key.k_split;
  sy.stamps = stamps;
  sy.opts = opts;
  prefetch_holds(sy);
  sy.n_prev = kLnReplicas + kFfnSlices;
  P.nv = vt * val.k_split;
  sy.n_val = P.nv;
  return true;
}

// the FFN half's arguments, its row-fused form (n_fix = 1: the trailing shift writer) and the
// granule hand-off where they apply
static bool ffn_setup(const LnMixArgs& ln, const GemmArgs& key, const GemmArgs& val, int* cnt, int* cnt_prev, int* err,
                      int R, uint64_t* stamps, int opts, bool fused_ln, uint64_t* gran, const int* epoch, FfnPrep& P,
                      int& n_fix) {
  if (!prep_ffn_persist(ln, key, val, cnt, cnt_prev, err, R, stamps, opts, P)) return false;
  const bool fused = fused_ln && R == 1 && ln.inplace;
  n_fix = 0;
  if (fused) {
    P.sy.n_ln_blocks = 0;
    P.sy.d_k = 0;
    P.sy.opts &= ~1;  // (no LayerNorm rows for the value workgroups to wait for)
    P.sy.d_v = kHold1Value;
    n_fix = 1;
    // the granule key -> value hand-off: four key splits (the value role's NX), one segment
    if (gran && epoch && key.k_split == 4 && key.nseg == 1 && ln.layer < 64) {
      P.sy.gran = gran;
      P.sy.epoch = epoch;
      P.sy.gran_ld = key.seg[0].N;
      P.sy.layer = ln.layer;
    }
  }
  return true;
}

bool launch_ffn_persist(const LnMixArgs& ln, const GemmArgs& key, const GemmArgs& val, int* cnt, int* cnt_prev,
                        int* err, int R, hipStream_t st, uint64_t* stamps, int opts, bool fused_ln, uint64_t* gran,
                        const int* epoch) {
  FfnPrep P;
  int n_fix = 0;
  if (!ffn_setup(ln, key, val, cnt, cnt_prev, err, R, stamps, opts, fused_ln, gran, epoch, P, n_fix)) return false;
  const bool fused = n_fix == 1;
  LnMixArgs& l = P.l;
  GemmArgs& ka = P.ka;
  GemmArgs& va = P.va;
  FfnSync& sy = P.sy;
  const size_t lds = (size_t)2 * 16 * (8 * 32 + 8) * 2 * 2;
  const dim3 grid(sy.n_ln_blocks + sy.n_key + P.nv + n_fix);
  if (key.f16) {
    if (fused) RT_LAUNCH((k_ffn_persist<true, true>), grid, dim3(256), lds, st, l, ka, va, sy);
    else RT_LAUNCH((k_ffn_persist<true, false>), grid, dim3(256), lds, st, l, ka, va, sy);
  } else {
    if (fused) RT_LAUNCH((k_ffn_persist<false, true>), grid, dim3(256), lds, st, l, ka, va, sy);
    else RT_LAUNCH((k_ffn_persist<false, false>), grid, dim3(256), lds, st, l, ka, va, sy);
  }
  return true;
}

int gemm_ksteps(int kslice) { return kslice / 32; }

bool gemm_tile_table(GemmArgs& a, int64_t x_mix_stride) {
  a.n_tinfo = 0;
  if (a.nseg < 2 || x_mix_stride <= 0) return false;
  const int tiles = a.seg[a.nseg - 1].tile_start + (a.seg[a.nseg - 1].N + 63) / 64;
  if (tiles > 128) return false;
  const bf16_t* base = a.seg[0].W;
  for (int j = 0; j < a.nseg; ++j) {
    const GemmSeg& g = a.seg[j];
    const int64_t dx = g.Xhi - a.seg[0].Xhi;
    if (g.W != base + (int64_t)g.tile_start * 64 * a.K || g.ldx != a.seg[0].ldx || dx % x_mix_stride != 0 ||
        g.Xlo - a.seg[0].Xlo != dx || dx / x_mix_stride < 0 || dx / x_mix_stride > 7 || g.col_off > (1 << 21))
      return false;
    for (int t = 0; t < (g.N + 63) / 64; ++t) {
      const int nv = std::min(64, g.N - t * 64);
      a.tinfo[g.tile_start + t] = (uint32_t)(dx / x_mix_stride) | ((uint32_t)nv << 3) | ((uint32_t)(g.col_off + t * 64) << 10);
    }
  }
  a.tw = base;
  a.x_mix_stride = x_mix_stride;
  a.n_tinfo = tiles;
  return true;
}

int launch_gemm(const GemmArgs& a, hipStream_t st) {
  const int tiles = a.seg[a.nseg - 1].tile_start + (a.seg[a.nseg - 1].N + 63) / 64;
  // one or two 16-row blocks per workgroup, also for prefill steps: 64- and 128-row groups
  // (fewer weight re-reads, 135 KB X images, one workgroup per CU) were measured slower on a
  // 1280-row prefill step (10.6 vs 9.2 ms): the launches are latency-bound, not weight-bound
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
  return (int)(grid.x * grid.y * grid.z);
}
// W [N][K] -> MFMA B-fragment blocks: block (nb, kb) = 16 columns x 32 k = 1 KB, lane
// l = 16 g + li holding W[16 nb + li][32 kb + 8 g .. + 8]; blocks ordered nb-major. Rows >= N are 0.
__global__ void k_pack_frag(const bf16_t* W, int N, int K, bf16_t* out) {
  const int64_t nblk = (N + 15) / 16, total = nblk * 16 * K;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(idx & 7), lane = (int)((idx >> 3) & 63);
    const int64_t blk = idx >> 9;
    const int kb = (int)(blk % (K / 32)), nb = (int)(blk / (K / 32));
    const int n = nb * 16 + (lane & 15), k = kb * 32 + (lane >> 4) * 8 + e;
    out[idx] = n < N ? W[(int64_t)n * K + k] : (bf16_t)0;
  }
}

void launch_pack_frag(const bf16_t* W, int N, int K, bf16_t* out, hipStream_t st) {
  RT_LAUNCH(k_pack_frag, dim3(4096), dim3(256), 0, st, W, N, K, out);
}

// ------------------------------------------------------------------------------------
// quant_pack: web-rwkv 0.10.16's Quant::Int8 / Quant::NF4 matrix quantisation, restated (the
// crate is not vendored: parity unpinned; the oracle restates the same rules independently,
// oracle/rwkv7.c). One thread per (column n, K-block):
//  Int8 (128 k): mn = f16(min), mx = f16(max); q = floor(fma(clamp((x - mn) / (mx - mn), 0, 1),
//    255, 0.5)) (0 when mx == mn); dequantised w = fma(q, (mx - mn) / 255, mn).
//  NF4 (64 k): s = f16(max |x|); q = #{i < 15 : x / s > (t[i] + t[i+1]) / 2} (7 when s == 0);
//    dequantised w = t[q] * s, t = the NormalFloat-4 code table.
// ------------------------------------------------------------------------------------
__device__ inline float f16_round(float x) { return (float)(_Float16)x; }
// byte offset of element (n, k) in the fragment order, for e-byte lanes (int8: 8 per lane)
__device__ inline int64_t frag_elem(int n, int k, int K) {
  const int nb = n >> 4, li = n & 15, kb = k >> 5, g = (k >> 3) & 3, e = k & 7;
  return (((int64_t)nb * (K >> 5) + kb) * 64 + 16 * g + li) * 8 + e;
}
template <int QT>
__global__ void k_quant_pack(const uint16_t* W, int N, int K, int f16, uint8_t* codes, void* scales) {
  constexpr int BS = QT == 1 ? kQ8Block : kQ4Block;
  const int nkb = K / BS;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)N * nkb) return;
  const int n = (int)(id / nkb), kb = (int)(id % nkb);
  const uint16_t* row = W + (int64_t)n * K + kb * BS;
  auto at = [&](int i) { return f16 ? h16_to_f32(row[i]) : bf16_to_f32(row[i]); };
  if constexpr (QT == 1) {
    float lo = at(0), hi = at(0);
    for (int i = 1; i < BS; ++i) { lo = fminf(lo, at(i)); hi = fmaxf(hi, at(i)); }
    const float mn = f16_round(lo), mx = f16_round(hi), d = mx - mn;
    for (int i = 0; i < BS; ++i) {
      uint32_t q = 0;
      if (mx != mn) {
        const float v = fminf(fmaxf((at(i) - mn) / d, 0.0f), 1.0f);
        q = (uint32_t)floorf(fmaf(v, 255.0f, 0.5f));
      }
      codes[frag_elem(n, kb * BS + i, K)] = (uint8_t)q;
    }
    ((uint32_t*)scales)[id] = (uint32_t)f32_to_h16(mn) | ((uint32_t)f32_to_h16(mx) << 16);
  } else {
    float am = 0.0f;
    for (int i = 0; i < BS; ++i) am = fmaxf(am, fabsf(at(i)));
    const float sc = f16_round(am);
    for (int i = 0; i < BS; i += 2) {
      uint32_t q2[2];
      for (int u = 0; u < 2; ++u) {
        uint32_t q = 7;
        if (sc != 0.0f) {
          const float v = at(i + u) / sc;
          q = 0;
          for (int t = 0; t < 15; ++t) q += v > 0.5f * (kNF4[t] + kNF4[t + 1]) ? 1u : 0u;
        }
        q2[u] = q;
      }
      // nibble pair (k, k + 1) = byte (frag_elem / 2): low nibble the even k
      codes[frag_elem(n, kb * BS + i, K) >> 1] = (uint8_t)(q2[0] | (q2[1] << 4));
    }
    ((uint16_t*)scales)[id] = f32_to_h16(sc);
  }
}

void launch_quant_pack(const uint16_t* W, int N, int K, int f16, int qt, uint8_t* codes, void* scales, hipStream_t st) {
  const int64_t n = (int64_t)N * (K / (qt == 1 ? kQ8Block : kQ4Block));
  const dim3 grid((unsigned)((n + 255) / 256));
  if (qt == 1) hipLaunchKernelGGL(k_quant_pack<1>, grid, dim3(256), 0, st, W, N, K, f16, codes, scales);
  else hipLaunchKernelGGL(k_quant_pack<2>, grid, dim3(256), 0, st, W, N, K, f16, codes, scales);
}

__global__ void k_pack_lora(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                            int Dw, int Da, int Dv, int Dg, bf16_t* out) {
  const int Dall = Dw + Da + Dv + Dg, eq = Dall / 4;
  const int e1 = Dw / 4, e2 = e1 + Da / 4, e3 = e2 + Dv / 4;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < (int64_t)C * Dall;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(idx / Dall), r = (int)(idx % Dall), pq = r / eq, e = r % eq;
    bf16_t v;
    if (e < e1) v = w2t[(int64_t)co * Dw + pq * (Dw / 4) + e];
    else if (e < e2) v = a2t[(int64_t)co * Da + pq * (Da / 4) + (e - e1)];
    else if (e < e3) v = v2t[(int64_t)co * Dv + pq * (Dv / 4) + (e - e2)];
    else v = g2t[(int64_t)co * Dg + pq * (Dg / 4) + (e - e3)];
    out[idx] = v;
  }
}

// LoRA-up rows in k_wkv4's register order: per head h, entry u (w 0..3 | a 4..7 | v 8..9 |
// g 10..17, 8 bf16 each) of thread t = 2 i + hf (channel 64 h + i, half hf) at uint4 index
// (h * 18 + u) * 128 + t, so each wave-wide load is 1 KB contiguous.
__global__ void k_pack_lora4(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                             bf16_t* out) {
  const int64_t total = (int64_t)(C / 64) * 18 * 128;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(idx % 128), u = (int)((idx / 128) % 18), h = (int)(idx / (128 * 18));
    const int c = h * 64 + (t >> 1), hf = t & 1;
    const bf16_t* src;
    if (u < 4) src = w2t + (int64_t)c * 64 + hf * 32 + u * 8;
    else if (u < 8) src = a2t + (int64_t)c * 64 + hf * 32 + (u - 4) * 8;
    else if (u < 10) src = v2t + (int64_t)c * 32 + hf * 16 + (u - 8) * 8;
    else src = g2t + (int64_t)c * 128 + hf * 64 + (u - 10) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) out[idx * 8 + e] = src[e];
  }
}

void launch_pack_lora4(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                       bf16_t* out, hipStream_t st) {
  RT_LAUNCH(k_pack_lora4, dim3(256), dim3(256), 0, st, w2t, a2t, v2t, g2t, C, out);
}

// k_wkv6's register order: thread t = 4 i + qq holds quarter qq of channel c = 64 h + i's rows
// (w 16 | a 16 | v 8 | g 32 values = 9 entries of 8); entry u of thread t at uint4 u * 256 + t.
__global__ void k_pack_lora6(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                             bf16_t* out) {
  const int64_t total = (int64_t)(C / 64) * 9 * 256;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(idx % 256), u = (int)((idx / 256) % 9), h = (int)(idx / (256 * 9));
    const int c = h * 64 + (t >> 2), qq = t & 3;
    const bf16_t* src;
    if (u < 2) src = w2t + (int64_t)c * 64 + qq * 16 + u * 8;
    else if (u < 4) src = a2t + (int64_t)c * 64 + qq * 16 + (u - 2) * 8;
    else if (u == 4) src = v2t + (int64_t)c * 32 + qq * 8;
    else src = g2t + (int64_t)c * 128 + qq * 32 + (u - 5) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) out[idx * 8 + e] = src[e];
  }
}
void launch_pack_lora6(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                       bf16_t* out, hipStream_t st) {
  RT_LAUNCH(k_pack_lora6, dim3(256), dim3(256), 0, st, w2t, a2t, v2t, g2t, C, out);
}

void launch_pack_lora(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                      int Dw, int Da, int Dv, int Dg, bf16_t* out, hipStream_t st) {
  RT_LAUNCH(k_pack_lora, dim3(1024), dim3(256), 0, st, w2t, a2t, v2t, g2t, C, Dw, Da, Dv, Dg, out);
}

// ------------------------------------------------------------------------------------
// wkv, two waves per (slot segment, head): thread t = (row i = t >> 1, half hf = t & 1) owns
// state row S[i][32 hf .. 32 hf + 31] (32 VGPRs) and half of channel c = h*64 + i's LoRA-up
// dot products (halves combined by one shuffle), so reductions over j are in-lane plus one
// pair shuffle; per-channel vectors (w, kk, a, k, r) and the LoRA hidden go through LDS as
// broadcasts; cross-wave sums (|kk|^2, bonus, GroupNorm moments) take one barrier each.
// Loads that need only the head (LoRA-up rows, parameters) are issued before the segment
// descriptor arrives.
// ------------------------------------------------------------------------------------
template <int DW, int DA, int DV, int DG, int MAXP>
__global__ __launch_bounds__(128) void k_wkv2(WkvArgs a) {
  constexpr int N = 64, DALL = DW + DA + DV + DG;
  __shared__ __attribute__((aligned(16))) float s_hid[DALL];
  __shared__ __attribute__((aligned(16))) float s_vec[5][N];  // w, kk (unnormalised), a, k, r
  __shared__ float s_red[4][2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i = t >> 1, hf = t & 1;
  uint64_t* stp = (a.stamps && t == 0) ? a.stamps + (blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
  if (stp) stp[0] = __builtin_amdgcn_s_memtime();
  const int h = blockIdx.y, C = a.C, c = h * N + i;
  const int4 sg = a.segs[blockIdx.x];
  // ---- head-only loads: half of channel c's LoRA-up rows (bf16) and its parameters
  constexpr int UW = DW / 16, UA = DA / 16, UV = DV / 16, UG = DG / 16, UL = UW + UA + UV + UG;
  short8 lw[UL];
#pragma unroll
  for (int u = 0; u < UW; ++u) lw[u] = *(const short8*)(a.w2t + (int64_t)c * DW + hf * (DW / 2) + u * 8);
#pragma unroll
  for (int u = 0; u < UA; ++u) lw[UW + u] = *(const short8*)(a.a2t + (int64_t)c * DA + hf * (DA / 2) + u * 8);
#pragma unroll
  for (int u = 0; u < UV; ++u) lw[UW + UA + u] = *(const short8*)(a.v2t + (int64_t)c * DV + hf * (DV / 2) + u * 8);
#pragma unroll
  for (int u = 0; u < UG; ++u)
    lw[UW + UA + UV + u] = *(const short8*)(a.g2t + (int64_t)c * DG + hf * (DG / 2) + u * 8);
  const float w0 = a.w0[c], a0 = a.a0[c], v0 = a.v0[c], kkc = a.k_k[c], kac = a.k_a[c];
  const float rkc = a.r_k[c], lnw = a.lnx_w[c], lnb = a.lnx_b[c];
  // ---- segment-dependent loads, issued speculatively for slot = row = segment index (the
  // decode layout: rows in slot order, one row per slot) and redone if the descriptor differs
  const int spec = blockIdx.x;
  const int64_t soff = a.layer_off + (int64_t)h * N * N + i * N + hf * 32;
  float S[32];
  auto load_state = [&](int slot) {
    const float* Sp = a.state + (int64_t)slot * a.slot_stride + soff;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4_ v4 = *(const float4_*)(Sp + q * 4);
      S[q * 4 + 0] = v4[0]; S[q * 4 + 1] = v4[1]; S[q * 4 + 2] = v4[2]; S[q * 4 + 3] = v4[3];
    }
  };
  load_state(spec < a.n_slots ? spec : 0);
  constexpr int HPL = (DALL + 127) / 128;  // hidden elements per thread
  float hp[MAXP][HPL], rp[MAXP], kp[MAXP], vp[MAXP], vf = 0.f;
  auto load_parts = [&](int row) {
    const float* prow = a.part + (int64_t)row * a.ldp;
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      const bool on = p < a.n_part;
      const float* pp = prow + p * a.part_stride;
#pragma unroll
      for (int e = 0; e < HPL; ++e) {
        const int d = t + 128 * e;
        hp[p][e] = (on && d < DALL) ? pp[3 * C + d] : 0.f;
      }
      rp[p] = on ? pp[c] : 0.f;
      kp[p] = on ? pp[C + c] : 0.f;
      vp[p] = on ? pp[2 * C + c] : 0.f;
    }
    vf = a.layer > 0 ? a.v_first[(int64_t)row * a.ldv + c] : 0.f;
  };
  load_parts(spec);
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  float* Srow = a.state + (int64_t)slot * a.slot_stride + soff;
  if (slot != spec) load_state(slot);
  if (r_begin != spec) load_parts(r_begin);
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    if (rr > 0) load_parts(row);
#pragma unroll
    for (int e = 0; e < HPL; ++e) {
      float x = 0.f;
#pragma unroll
      for (int p = 0; p < MAXP; ++p) x += hp[p][e];
      const int d = t + 128 * e;
      if (d < DALL) s_hid[d] = d < DW ? tanhf(x) : (d >= DW + DA + DV ? sigm(x) : x);
    }
    float r = 0.f, k = 0.f, v = 0.f;
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      r += rp[p];
      k += kp[p];
      v += vp[p];
    }
    __syncthreads();
    if (stp && rr == 0) stp[1] = __builtin_amdgcn_s_memtime();
    // ---- LoRA up: this thread's half of channel c's four dot products, pair-combined
    float lo0 = 0.f, lo1 = 0.f, lo2 = 0.f, lo3 = 0.f;
    auto dot8 = [&](const short8 q, const float* hsrc) {
      const float4_ h0 = *(const float4_*)hsrc;
      const float4_ h1 = *(const float4_*)(hsrc + 4);
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += w16_to_f32((uint16_t)q[e], a.f16 != 0) * h0[e];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += w16_to_f32((uint16_t)q[4 + e], a.f16 != 0) * h1[e];
      return acc;
    };
#pragma unroll
    for (int u = 0; u < UW; ++u) lo0 += dot8(lw[u], s_hid + hf * (DW / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < UA; ++u) lo1 += dot8(lw[UW + u], s_hid + DW + hf * (DA / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < UV; ++u) lo2 += dot8(lw[UW + UA + u], s_hid + DW + DA + hf * (DV / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < UG; ++u) lo3 += dot8(lw[UW + UA + UV + u], s_hid + DW + DA + DV + hf * (DG / 2) + u * 8);
    lo0 += dpp_mov<0xB1>(lo0);
    lo1 += dpp_mov<0xB1>(lo1);
    lo2 += dpp_mov<0xB1>(lo2);
    lo3 += dpp_mov<0xB1>(lo3);
    // ---- channel mixing terms (both threads of the pair compute channel c)
    const float w = expf(-0.60653066f * sigm(w0 + lo0));
    const float av = sigm(a0 + lo1);
    const float kk = k * kkc;
    k = k * (1.0f + (av - 1.0f) * kac);
    if (a.layer == 0) {
      if (hf == 0) a.v_first[(int64_t)row * a.ldv + c] = v;
    } else {
      v = v + (vf - v) * sigm(v0 + lo2);
    }
    {
      const float ksq = wave_sum(hf == 0 ? kk * kk : 0.f);
      const float bon = wave_sum(hf == 0 ? r * k * rkc : 0.f);
      if (lane == 0) { s_red[0][wave] = ksq; s_red[1][wave] = bon; }
    }
    if (hf == 0) {
      s_vec[0][i] = w; s_vec[1][i] = kk; s_vec[2][i] = av; s_vec[3][i] = k; s_vec[4][i] = r;
    }
    __syncthreads();
    if (stp && rr == 0) stp[2] = __builtin_amdgcn_s_memtime();
    const float inv = 1.0f / fmaxf(sqrtf(s_red[0][0] + s_red[0][1]), 1e-12f);
    const float bonus = s_red[1][0] + s_red[1][1];
    // ---- state half-row update: S[i][j] = S[i][j]*w_j - sa_i*kk_j*a_j + v_i*k_j ; y_i = S[i].r
    const float* vj = &s_vec[0][hf * 32];
    float sa = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) sa += S[q * 4 + e] * (kq[e] * inv);
    }
    sa += dpp_mov<0xB1>(sa);
    float y = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4_ wq = *(const float4_*)(vj + q * 4);
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
      const float4_ aq = *(const float4_*)(vj + 2 * N + q * 4);
      const float4_ k4 = *(const float4_*)(vj + 3 * N + q * 4);
      const float4_ rq = *(const float4_*)(vj + 4 * N + q * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float& sv = S[q * 4 + e];
        sv = sv * wq[e] - sa * ((kq[e] * inv) * aq[e]) + v * k4[e];
        y += sv * rq[e];
      }
    }
    y += dpp_mov<0xB1>(y);
    // ---- GroupNorm over the head's 64 rows (eps 64e-5): one-barrier moments
    {
      const float s1 = wave_sum(hf == 0 ? y : 0.f);
      const float s2 = wave_sum(hf == 0 ? y * y : 0.f);
      if (lane == 0) { s_red[2][wave] = s1; s_red[3][wave] = s2; }
    }
    __syncthreads();
    if (stp && rr == 0) stp[3] = __builtin_amdgcn_s_memtime();
    const float mean = (s_red[2][0] + s_red[2][1]) * (1.0f / N);
    const float var = fmaxf((s_red[3][0] + s_red[3][1]) * (1.0f / N) - mean * mean, 0.f);
    if (hf == 0) {
      const float gn = (y - mean) * (1.0f / sqrtf(var + 64e-5f)) * lnw + lnb;
      split_store((gn + bonus * v) * lo3, a.z_hi, a.z_lo, (int64_t)row * a.ldz + c, a.f16 != 0);
    }
    if (stp && rr == 0) stp[4] = __builtin_amdgcn_s_memtime();
    if (stp && rr == 1) stp[6] = __builtin_amdgcn_s_memtime();
    if (rr + 1 < n_rows) __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float4_ v4 = {S[q * 4 + 0], S[q * 4 + 1], S[q * 4 + 2], S[q * 4 + 3]};
    *(float4_*)(Srow + q * 4) = v4;
  }
  if (stp) stp[5] = __builtin_amdgcn_s_memtime();
}

// ------------------------------------------------------------------------------------
// wkv4: the 0.4B shape (LoRA ranks 64/64/32/128, 4 split-K slabs) cut down to the instruction
// stream the arithmetic needs. The decode WKV is VALU-issue-bound (one wave per SIMD, every
// wave a straight ~2k-instruction program), so this variant removes work rather than adding
// parallelism: the weight format is a template (no runtime f16/bf16 select), the LoRA hidden
// is summed from float4 slab loads by 72 threads, LoRA-up dot products and the state update run
// on packed f32 pairs (v_pk_fma_f32), sigmoid / tanh / exp use the hardware exp2 (|rel err|
// ~1e-7, far inside the logits tolerance), and the slot / row speculation of k_wkv2 is kept.
// Thread t = (channel i = t >> 1, half hf = t & 1) owns state row S[i][32 hf .. 32 hf + 31].
// ------------------------------------------------------------------------------------
__device__ inline float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ inline float fsigm(float x) { return __builtin_amdgcn_rcpf(1.0f + fexp(-x)); }
__device__ inline float ftanh(float x) {
  const float e = fexp(2.0f * fminf(fmaxf(x, -20.f), 20.f));
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}
template <bool F16>
__device__ inline float2_ w2f(uint32_t u) {  // two packed 16-bit weights -> f32 pair
  if constexpr (F16) {
    return (float2_){h16_to_f32((uint16_t)(u & 0xFFFFu)), h16_to_f32((uint16_t)(u >> 16))};
  } else {
    return (float2_){__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xFFFF0000u)};
  }
}

template <bool F16>
__global__ __launch_bounds__(128) void k_wkv4(WkvArgs a) {
  constexpr int N = 64, DW = 64, DA = 64, DV = 32, DG = 128, DALL = DW + DA + DV + DG, NP = 4;
  __shared__ __attribute__((aligned(16))) float s_hid[DALL];
  __shared__ __attribute__((aligned(16))) float s_vec[5][N];  // w, kk (unnormalised), a, k, r
  __shared__ float s_red[4][2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i = t >> 1, hf = t & 1;
  int seg_i = blockIdx.x, h = blockIdx.y;
  if (a.xmap) {  // 1-D grid: head h's workgroups share one XCD (its LoRA-up rows stay in one L2)
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    h = xcd + 8 * (j / a.n_seg);
    seg_i = j % a.n_seg;
  }
  const int C = a.C, c = h * N + i;
  tl_begin(a.tl);
  // debug phase stamps (RWKVTTS_WKV_STAMPS, layer 5 only; null in production): [0] realtime
  // start, [1..6] core clock at phase ends, [7] realtime end
  uint64_t* stp = (a.stamps && t == 0) ? a.stamps + ((int64_t)h * a.n_seg + seg_i) * 8 : nullptr;
  if (stp) { stp[0] = __builtin_amdgcn_s_memrealtime(); stp[1] = __builtin_amdgcn_s_memtime(); }
  bf16_t* e_zhi = a.z_hi;
  bf16_t* e_zlo = a.z_lo;
  int e_ldz = a.ldz;
  const int4 sg = a.segs[seg_i];
  uint4 lw[18];  // 8 bf16 per entry: w 0..3 | a 4..7 | v 8..9 | g 10..17
  {  // packed per head by launch_pack_lora4: entry u of thread t at uint4 index u * 128 + t
    const uint4* pl = (const uint4*)(a.lup + (int64_t)h * 18 * 128 * 8);
#pragma unroll
    for (int u = 0; u < 18; ++u) lw[u] = pl[u * 128 + t];
  }
  // ---- head-only loads: half of channel c's LoRA-up rows + parameters
  const float w0 = a.w0[c], a0 = a.a0[c], v0 = a.v0[c], kkc = a.k_k[c], kac = a.k_a[c];
  const float rkc = a.r_k[c], lnw = a.lnx_w[c], lnb = a.lnx_b[c];
  // ---- segment-dependent loads, speculated for slot = row = segment index (decode layout)
  const int spec = seg_i < a.n_slots ? seg_i : 0;
  // state block layout (engine.hip perm_index): this thread's q-th float4 at index q * 128 + t
  const int64_t soff = a.layer_off + (int64_t)h * N * N + (int64_t)t * 4;
  float4_ S4[8];
  auto load_state = [&](int slot) {
    const float4_* Sp = (const float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
#pragma unroll
    for (int q = 0; q < 8; ++q) S4[q] = Sp[q * 128];
  };
  const bool hid_thread = t < DALL / 4;
  float4_ hp[NP];
  float rp[NP], kp[NP], vp[NP], vf = 0.f;
  auto load_parts = [&](int row) {
    const float* prow = a.part + (int64_t)row * a.ldp;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float* pp = prow + p * a.part_stride;
      hp[p] = *(const float4_*)(pp + 3 * C + (hid_thread ? 4 * t : 0));
      rp[p] = pp[c];
      kp[p] = pp[C + c];
      vp[p] = pp[2 * C + c];
    }
    vf = a.layer > 0 ? a.v_first[(int64_t)row * a.ldv + c] : 0.f;
  };
  load_parts(spec);
  // the state goes out last (vmcnt retires in issue order): the LoRA / mixing phase starts
  // while it is still in flight (measured: the LoRA-up rows first, then the partials, is best
  // here; k_wkv6 prefers partials first)
  load_state(spec);
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  if (r_begin != spec) load_parts(r_begin);
  if (slot != spec) load_state(slot);
  float4_* Srow = (float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    if (rr > 0) load_parts(row);
    // LoRA hidden: threads 0..71 each own 4 consecutive entries (one region: w | a | v | g)
    if (hid_thread) {
      float4_ x = hp[0];
#pragma unroll
      for (int p = 1; p < NP; ++p) x += hp[p];
      float4_ y;
      if (t < DW / 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = ftanh(x[e]);
      } else if (t < (DW + DA + DV) / 4) {
        y = x;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = fsigm(x[e]);
      }
      *(float4_*)(s_hid + 4 * t) = y;
    }
    float r = rp[0], k = kp[0], v = vp[0];
#pragma unroll
    for (int p = 1; p < NP; ++p) {
      r += rp[p];
      k += kp[p];
      v += vp[p];
    }
    __syncthreads();
    if (stp && rr == 0) stp[2] = __builtin_amdgcn_s_memtime() + (uint64_t)(r != r);
    // ---- LoRA up on packed pairs: this thread's half of channel c's four dot products
    float2_ l0 = {0.f, 0.f}, l1 = {0.f, 0.f}, l2 = {0.f, 0.f}, l3 = {0.f, 0.f};
    auto dot = [&](float2_ acc, const uint4 q, const float* hsrc) {
      const float4_ h0 = *(const float4_*)hsrc;
      const float4_ h1 = *(const float4_*)(hsrc + 4);
      acc += w2f<F16>(q.x) * (float2_){h0[0], h0[1]};
      acc += w2f<F16>(q.y) * (float2_){h0[2], h0[3]};
      acc += w2f<F16>(q.z) * (float2_){h1[0], h1[1]};
      acc += w2f<F16>(q.w) * (float2_){h1[2], h1[3]};
      return acc;
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) l0 = dot(l0, lw[u], s_hid + hf * (DW / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u) l1 = dot(l1, lw[4 + u], s_hid + DW + hf * (DA / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < 2; ++u) l2 = dot(l2, lw[8 + u], s_hid + DW + DA + hf * (DV / 2) + u * 8);
#pragma unroll
    for (int u = 0; u < 8; ++u) l3 = dot(l3, lw[10 + u], s_hid + DW + DA + DV + hf * (DG / 2) + u * 8);
    float lo0 = l0[0] + l0[1], lo1 = l1[0] + l1[1], lo2 = l2[0] + l2[1], lo3 = l3[0] + l3[1];
    lo0 += dpp_mov<0xB1>(lo0);
    lo1 += dpp_mov<0xB1>(lo1);
    lo2 += dpp_mov<0xB1>(lo2);
    lo3 += dpp_mov<0xB1>(lo3);
    // ---- channel mixing terms (both threads of the pair compute channel c)
    const float w = fexp(-0.60653066f * fsigm(w0 + lo0));
    const float av = fsigm(a0 + lo1);
    const float kk = k * kkc;
    k = k * (1.0f + (av - 1.0f) * kac);
    if (a.layer == 0) {
      if (hf == 0) a.v_first[(int64_t)row * a.ldv + c] = v;
    } else {
      v = v + (vf - v) * fsigm(v0 + lo2);
    }
    {
      const float ksq = wave_sum(hf == 0 ? kk * kk : 0.f);
      const float bon = wave_sum(hf == 0 ? r * k * rkc : 0.f);
      if (lane == 0) { s_red[0][wave] = ksq; s_red[1][wave] = bon; }
    }
    if (hf == 0) {
      s_vec[0][i] = w; s_vec[1][i] = kk; s_vec[2][i] = av; s_vec[3][i] = k; s_vec[4][i] = r;
    }
    __syncthreads();
    if (stp && rr == 0) stp[3] = __builtin_amdgcn_s_memtime();
    const float inv = __builtin_amdgcn_rcpf(fmaxf(sqrtf(s_red[0][0] + s_red[0][1]), 1e-12f));
    const float bonus = s_red[1][0] + s_red[1][1];
    // ---- state half-row update on packed pairs: S = S*w - sa*(kk*inv*a) + v*k ; y = S.r
    const float* vj = &s_vec[0][hf * 32];
    float2_ sa2 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
      sa2 += (float2_){S4[q][0], S4[q][1]} * (float2_){kq[0], kq[1]};
      sa2 += (float2_){S4[q][2], S4[q][3]} * (float2_){kq[2], kq[3]};
    }
    float sa = (sa2[0] + sa2[1]) * inv;
    sa += dpp_mov<0xB1>(sa);
    float2_ y2 = {0.f, 0.f};
    const float2_ sav = {sa * inv, sa * inv}, vv = {v, v};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4_ wq = *(const float4_*)(vj + q * 4);
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
      const float4_ aq = *(const float4_*)(vj + 2 * N + q * 4);
      const float4_ k4 = *(const float4_*)(vj + 3 * N + q * 4);
      const float4_ rq = *(const float4_*)(vj + 4 * N + q * 4);
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        float2_ sv = (float2_){S4[q][e], S4[q][e + 1]} * (float2_){wq[e], wq[e + 1]};
        sv -= sav * ((float2_){kq[e], kq[e + 1]} * (float2_){aq[e], aq[e + 1]});
        sv += vv * (float2_){k4[e], k4[e + 1]};
        S4[q][e] = sv[0];
        S4[q][e + 1] = sv[1];
        y2 += sv * (float2_){rq[e], rq[e + 1]};
      }
    }
    if (stp && rr == 0) stp[4] = __builtin_amdgcn_s_memtime() + (uint64_t)(y2[0] != y2[0]);
    if (rr + 1 == n_rows) {  // the segment's final state: stored before the GroupNorm tail
      if (a.wt) {
        const auto rs = wt_rsrc(a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N);
#pragma unroll
        for (int q = 0; q < 8; ++q) store_wt(rs, (q * 128 + t) * 16, S4[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) Srow[q * 128] = S4[q];
      }
    }
    float y = y2[0] + y2[1];
    y += dpp_mov<0xB1>(y);
    {
      const float s1 = wave_sum(hf == 0 ? y : 0.f);
      const float s2 = wave_sum(hf == 0 ? y * y : 0.f);
      if (lane == 0) { s_red[2][wave] = s1; s_red[3][wave] = s2; }
    }
    __syncthreads();
    if (stp && rr == 0) stp[5] = __builtin_amdgcn_s_memtime();
    const float mean = (s_red[2][0] + s_red[2][1]) * (1.0f / N);
    const float var = fmaxf((s_red[3][0] + s_red[3][1]) * (1.0f / N) - mean * mean, 0.f);
    if (hf == 0) {
      const float gn = (y - mean) * __builtin_amdgcn_rsqf(var + 64e-5f) * lnw + lnb;
      split_store((gn + bonus * v) * lo3, e_zhi, e_zlo, (int64_t)row * e_ldz + c, F16);
    }
    if (rr + 1 < n_rows) __syncthreads();
  }
  if (stp) { stp[6] = __builtin_amdgcn_s_memtime(); stp[7] = __builtin_amdgcn_s_memrealtime(); }
  tl_end(a.tl);
}

// ------------------------------------------------------------------------------------
// wkv6: k_wkv4 on four waves. Thread t = (channel i = t >> 2, quarter qq = t & 3) owns state
// row S[i][16 qq .. 16 qq + 15] and a quarter of channel c's LoRA-up dot products, so each
// thread executes half of k_wkv4's per-row arithmetic and two waves share every SIMD (the
// dependent chains of one hide behind the other's). Quarter sums are two quad shuffles.
// State blocks: thread t's q-th float4 at float4 index q * 256 + t (engine.hip perm_index,
// layout 2); LoRA-up rows: entry u of thread t at uint4 index u * 256 + t (launch_pack_lora6).
// ------------------------------------------------------------------------------------
// ROLE 0: a plain launch. ROLE 1: WKV workgroup of k_att_persist (decode rows only): the LoRA-up
// rows and the state (independent of this layer's rkv launch) are requested at dispatch, then
// the workgroup waits for its head's r / k / v tiles and the LoRA-down tiles, reads the partials
// by sc1 loads, and publishes its z row (staged in LDS, stored write-through by one wave) to
// its head's counter.
template <bool F16, int ROLE>
__device__ __attribute__((always_inline)) void wkv6_body(const WkvArgs& a, const int bx, const int by,
                                                         const FfnSync& sy) {
  constexpr int N = 64, DW = 64, DA = 64, DV = 32, DG = 128, DALL = DW + DA + DV + DG, NP = 4;
  __shared__ __attribute__((aligned(16))) uint16_t s_zh[ROLE ? N : 4], s_zl[ROLE ? N : 4];
  __shared__ __attribute__((aligned(16))) float s_hid[DALL];
  __shared__ __attribute__((aligned(16))) float s_vec[5][N];  // w, kk (unnormalised), a, k, r
  __shared__ float s_red[4][4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i = t >> 2, qq = t & 3;
  int seg_i = bx, h = by;
  if (a.xmap) {  // 1-D grid: head h's workgroups share one XCD (its LoRA-up rows stay in one L2)
    const int b = bx, xcd = b & 7, j = b >> 3;
    h = xcd + 8 * (j / a.n_seg);
    seg_i = j % a.n_seg;
  }
  const int C = a.C, c = h * N + i;
  // debug phase stamps (as k_wkv4: RWKVTTS_WKV_STAMPS, layer 5 only; null in production)
  uint64_t* stp = (a.stamps && t == 0) ? a.stamps + ((int64_t)h * a.n_seg + seg_i) * 8 : nullptr;
  if (stp) { stp[0] = __builtin_amdgcn_s_memrealtime(); stp[1] = __builtin_amdgcn_s_memtime(); }
  const int4 sg = a.segs[seg_i];
  const float w0 = a.w0[c], a0 = a.a0[c], v0 = a.v0[c], kkc = a.k_k[c], kac = a.k_a[c];
  const float rkc = a.r_k[c], lnw = a.lnx_w[c], lnb = a.lnx_b[c];
  const int spec = seg_i < a.n_slots ? seg_i : 0;
  const int64_t soff = a.layer_off + (int64_t)h * N * N + (int64_t)t * 4;
  float4_ S4[4];
  auto load_state = [&](int slot) {
    const float4_* Sp = (const float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
#pragma unroll
    for (int q = 0; q < 4; ++q) S4[q] = Sp[q * 256];
  };
  const bool hid_thread = t < DALL / 4;
  float4_ hp[NP];
  float rp[NP], kp[NP], vp[NP], vf = 0.f;
  auto load_parts = [&](int row) {
    const float* prow = a.part + (int64_t)row * a.ldp;
    if constexpr (ROLE >= 1) {  // handed-off partial slabs: sc1 loads only
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const auto rs = wt_rsrc(prow + p * a.part_stride);
        hp[p] = __builtin_bit_cast(float4_, ld_sc1_b128(rs, (3 * C + (hid_thread ? 4 * t : 0)) * 4));
        rp[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, c * 4, 0, 16));
        kp[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (C + c) * 4, 0, 16));
        vp[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (2 * C + c) * 4, 0, 16));
      }
    } else {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float* pp = prow + p * a.part_stride;
      hp[p] = *(const float4_*)(pp + 3 * C + (hid_thread ? 4 * t : 0));
      rp[p] = pp[c];
      kp[p] = pp[C + c];
      vp[p] = pp[2 * C + c];
    }
    }
    if constexpr (ROLE >= 1)
      vf = a.layer > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     wt_rsrc(a.v_first + (int64_t)row * a.ldv), c * 4, 0, 16))
                       : 0.f;
    else
      vf = a.layer > 0 ? a.v_first[(int64_t)row * a.ldv + c] : 0.f;
  };
  // issue order = need order (vmcnt retires in order): partials (hidden nonlinearity), then the
  // LoRA-up rows (LoRA / mixing phase), then the state (update phase)
  uint4 lw[9];  // 8 bf16 per entry: w 0..1 | a 2..3 | v 4 | g 5..8
  const uint4* pl = (const uint4*)(a.lup + (int64_t)h * 9 * 256 * 8);
  int slot, r_begin, n_rows;
  if constexpr (ROLE >= 1) {
    // LoRA-up rows and the state first (they do not depend on this layer's rkv workgroups), then
    // wait for the head's r / k / v tiles and the LoRA-down tiles, then their partials
    slot = sg.x; r_begin = sg.y; n_rows = sg.z;
    // (opts bit 3: only once the LN rows are published -- the LN phase then runs without this
    // prefetch beside it; the rkv phase still hides it)
    if (sy.opts & 8) sync_wait(sy.cnt + kSyncStride * (kAttLn + (blockIdx.x & (kLnReplicas - 1))), sy.ln_rows, sy.err, 64, sy.opts);
    hold_until(sy.d_s);
#pragma unroll
    for (int u = 0; u < 9; ++u) lw[u] = pl[u * 256 + t];
    load_state(slot);
    sync_wait(sy.cnt + kSyncStride * (kAttHead + h), sy.head_target, sy.err, 16, sy.opts);
    sync_wait(sy.cnt + kSyncStride * (kAttLora + (blockIdx.x & (kLnReplicas - 1))), sy.lora_target, sy.err, 32,
              sy.opts);
    sync_stamp(sy, 1);
    load_parts(r_begin);
  } else {
  load_parts(spec);
#pragma unroll
  for (int u = 0; u < 9; ++u) lw[u] = pl[u * 256 + t];
  load_state(spec);
  slot = sg.x; r_begin = sg.y; n_rows = sg.z;
  if (r_begin != spec) load_parts(r_begin);
  if (slot != spec) load_state(slot);
  }
  float4_* Srow = (float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
  auto quad_sum = [](float x) {
    x += dpp_mov<0xB1>(x);
    return x + dpp_mov<0x4E>(x);
  };
  for (int rr = 0; rr < n_rows; ++rr) {
    const int row = r_begin + rr;
    if (hid_thread) {
      float4_ x = hp[0];
#pragma unroll
      for (int p = 1; p < NP; ++p) x += hp[p];
      float4_ y;
      if (t < DW / 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = ftanh(x[e]);
      } else if (t < (DW + DA + DV) / 4) {
        y = x;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = fsigm(x[e]);
      }
      *(float4_*)(s_hid + 4 * t) = y;
    }
    float r = rp[0], k = kp[0], v = vp[0];
#pragma unroll
    for (int p = 1; p < NP; ++p) {
      r += rp[p];
      k += kp[p];
      v += vp[p];
    }
    // prefill segments: the next row's partials go out now and arrive during this row's work
    const float vf_row = vf;
    if (rr + 1 < n_rows) load_parts(row + 1);
    __syncthreads();
    if (stp && rr == 0) stp[2] = __builtin_amdgcn_s_memtime() + (uint64_t)(r != r);
    float2_ l0 = {0.f, 0.f}, l1 = {0.f, 0.f}, l2 = {0.f, 0.f}, l3 = {0.f, 0.f};
    auto dot = [&](float2_ acc, const uint4 q, const float* hsrc) {
      const float4_ h0 = *(const float4_*)hsrc;
      const float4_ h1 = *(const float4_*)(hsrc + 4);
      acc += w2f<F16>(q.x) * (float2_){h0[0], h0[1]};
      acc += w2f<F16>(q.y) * (float2_){h0[2], h0[3]};
      acc += w2f<F16>(q.z) * (float2_){h1[0], h1[1]};
      acc += w2f<F16>(q.w) * (float2_){h1[2], h1[3]};
      return acc;
    };
#pragma unroll
    for (int u = 0; u < 2; ++u) l0 = dot(l0, lw[u], s_hid + qq * (DW / 4) + u * 8);
#pragma unroll
    for (int u = 0; u < 2; ++u) l1 = dot(l1, lw[2 + u], s_hid + DW + qq * (DA / 4) + u * 8);
    l2 = dot(l2, lw[4], s_hid + DW + DA + qq * (DV / 4));
#pragma unroll
    for (int u = 0; u < 4; ++u) l3 = dot(l3, lw[5 + u], s_hid + DW + DA + DV + qq * (DG / 4) + u * 8);
    const float lo0 = quad_sum(l0[0] + l0[1]), lo1 = quad_sum(l1[0] + l1[1]);
    const float lo2 = quad_sum(l2[0] + l2[1]), lo3 = quad_sum(l3[0] + l3[1]);
    const float w = fexp(-0.60653066f * fsigm(w0 + lo0));
    const float av = fsigm(a0 + lo1);
    const float kk = k * kkc;
    k = k * (1.0f + (av - 1.0f) * kac);
    if (a.layer == 0) {
      if (qq == 0) {
        if constexpr (ROLE >= 1) store_wt(wt_rsrc(a.v_first + (int64_t)row * a.ldv), c * 4, v);
        else a.v_first[(int64_t)row * a.ldv + c] = v;
      }
    } else {
      v = v + (vf_row - v) * fsigm(v0 + lo2);
    }
    {
      const float ksq = wave_sum(qq == 0 ? kk * kk : 0.f);
      const float bon = wave_sum(qq == 0 ? r * k * rkc : 0.f);
      if (lane == 0) { s_red[0][wave] = ksq; s_red[1][wave] = bon; }
    }
    if (qq == 0) {
      s_vec[0][i] = w; s_vec[1][i] = kk; s_vec[2][i] = av; s_vec[3][i] = k; s_vec[4][i] = r;
    }
    __syncthreads();
    if (stp && rr == 0) stp[3] = __builtin_amdgcn_s_memtime();
    const float inv =
        __builtin_amdgcn_rcpf(fmaxf(sqrtf((s_red[0][0] + s_red[0][1]) + (s_red[0][2] + s_red[0][3])), 1e-12f));
    const float bonus = (s_red[1][0] + s_red[1][1]) + (s_red[1][2] + s_red[1][3]);
    const float* vj = &s_vec[0][qq * 16];
    float2_ sa2 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
      sa2 += (float2_){S4[q][0], S4[q][1]} * (float2_){kq[0], kq[1]};
      sa2 += (float2_){S4[q][2], S4[q][3]} * (float2_){kq[2], kq[3]};
    }
    const float sa = quad_sum((sa2[0] + sa2[1]) * inv);
    float2_ y2 = {0.f, 0.f};
    const float2_ sav = {sa * inv, sa * inv}, vv = {v, v};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4_ wq = *(const float4_*)(vj + q * 4);
      const float4_ kq = *(const float4_*)(vj + N + q * 4);
      const float4_ aq = *(const float4_*)(vj + 2 * N + q * 4);
      const float4_ k4 = *(const float4_*)(vj + 3 * N + q * 4);
      const float4_ rq = *(const float4_*)(vj + 4 * N + q * 4);
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        float2_ sv = (float2_){S4[q][e], S4[q][e + 1]} * (float2_){wq[e], wq[e + 1]};
        sv -= sav * ((float2_){kq[e], kq[e + 1]} * (float2_){aq[e], aq[e + 1]});
        sv += vv * (float2_){k4[e], k4[e + 1]};
        S4[q][e] = sv[0];
        S4[q][e + 1] = sv[1];
        y2 += sv * (float2_){rq[e], rq[e + 1]};
      }
    }
    if (rr + 1 == n_rows && ROLE == 0) {  // (ROLE 1 stores the state after its hand-off)
      if (a.wt) {
        const auto rs = wt_rsrc(a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N);
#pragma unroll
        for (int q = 0; q < 4; ++q) store_wt(rs, (q * 256 + t) * 16, S4[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) Srow[q * 256] = S4[q];
      }
    }
    if (stp && rr == 0) stp[4] = __builtin_amdgcn_s_memtime() + (uint64_t)(y2[0] != y2[0]);
    const float y = quad_sum(y2[0] + y2[1]);
    {
      const float s1 = wave_sum(qq == 0 ? y : 0.f);
      const float s2 = wave_sum(qq == 0 ? y * y : 0.f);
      if (lane == 0) { s_red[2][wave] = s1; s_red[3][wave] = s2; }
    }
    __syncthreads();
    if (stp && rr == 0) stp[5] = __builtin_amdgcn_s_memtime();
    const float mean = ((s_red[2][0] + s_red[2][1]) + (s_red[2][2] + s_red[2][3])) * (1.0f / N);
    const float var =
        fmaxf(((s_red[3][0] + s_red[3][1]) + (s_red[3][2] + s_red[3][3])) * (1.0f / N) - mean * mean, 0.f);
    if constexpr (ROLE == 2) {
      // granule form: the channel's split as ONE granule {hi | lo << 16, tag} (same expression
      // and threads as below, so the same bits) -- the Wo workgroups poll these directly
      if (qq == 0) {
        const float gn = (y - mean) * __builtin_amdgcn_rsqf(var + 64e-5f) * lnw + lnb;
        const float zx = (gn + bonus * v) * lo3;
        const uint16_t hb = f32_to_w16(zx, F16);
        const uint16_t lb = f32_to_w16(zx - w16_to_f32(hb, F16), F16);
        gran_store_bits(sy.zgran + c, (uint32_t)hb | ((uint32_t)lb << 16), gran_tag(sy));
      }
    } else if constexpr (ROLE == 1) {
      // the row's 64 z values split by the same threads and expression as split_store (the
      // compiler fuses the product into the 16-bit conversion, so the split must stay here to
      // keep the bits), the planes through LDS; wave 0's lanes 0..15 store 4 channels each as one
      // 8-byte write-through store per plane
      if (qq == 0) {
        const float gn = (y - mean) * __builtin_amdgcn_rsqf(var + 64e-5f) * lnw + lnb;
        const float zx = (gn + bonus * v) * lo3;
        const uint16_t hb = f32_to_w16(zx, F16);
        s_zh[i] = hb;
        s_zl[i] = f32_to_w16(zx - w16_to_f32(hb, F16), F16);
      }
      __syncthreads();
      if (t < 16) {
        const uint2 hv = *(const uint2*)(s_zh + 4 * t), lv = *(const uint2*)(s_zl + 4 * t);
        const int64_t zo = ((int64_t)row * a.ldz + h * N + 4 * t) * 2;
        store_wt(wt_rsrc(a.z_hi), (int)zo, hv);
        store_wt(wt_rsrc(a.z_lo), (int)zo, lv);
      }
    } else {
    if (qq == 0) {
      const float gn = (y - mean) * __builtin_amdgcn_rsqf(var + 64e-5f) * lnw + lnb;
      split_store((gn + bonus * v) * lo3, a.z_hi, a.z_lo, (int64_t)row * a.ldz + c, F16);
    }
    }
    if (rr + 1 < n_rows) __syncthreads();
  }
  if (stp) { stp[6] = __builtin_amdgcn_s_memtime(); stp[7] = __builtin_amdgcn_s_memrealtime(); }
  if constexpr (ROLE >= 1) {
    sync_stamp(sy, 2);
    if constexpr (ROLE == 1) sync_arrive(sy.cnt + kSyncStride * (kAttWkv + h));
    // the final state (read by the next step's launch only) goes out after the hand-off, so its
    // write-through drain is not on the Wo workgroups' path
    const auto rs = wt_rsrc(a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N);
#pragma unroll
    for (int q = 0; q < 4; ++q) store_wt(rs, (q * 256 + t) * 16, S4[q]);
  }
}

// ------------------------------------------------------------------------------------
// wkv6_rows: k_wkv6's arithmetic for steps whose segments hold several rows (prefill and mixed
// steps), in three phases per chunk of kRowsChunk rows instead of one whole row at a time
// (SURVEY §2.1 K5p):
//  A  everything that does not depend on the state, kRowsGroup rows per pair of barriers: the LoRA
//     hidden nonlinearities, the LoRA-up dot products, decay / in-context rate / key / value
//     mixing, the key-norm and bonus sums -> per-row vectors in LDS;
//  B  the recurrence alone, row after row: the state update and y = S r from registers and those
//     vectors, with no barrier (a state row lives in one quad of one wave);
//  C  the GroupNorm, bonus and gate of kRowsGroup rows per pair of barriers, z planes out.
// Every element takes the one-row code's expressions and reduction orders (the quad sums, the wave
// sums, the four waves' partials combined (0 + 1) + (2 + 3)), so the z planes and the state are
// bitwise those of wkv6_body's row loop (the prefill chunk- and batch-invariance tests compare
// prefill rows with graph-replayed decode rows, whose WKV is wkv6_body).
constexpr int kRowsChunk = 16, kRowsGroup = 2;
template <bool F16>
__device__ __attribute__((always_inline)) void wkv6_rows(const WkvArgs& a, const int bx, const int by) {
  constexpr int N = 64, DW = 64, DA = 64, DV = 32, DG = 128, DALL = DW + DA + DV + DG, NP = 4;
  constexpr int CH = kRowsChunk, G = kRowsGroup;
  __shared__ __attribute__((aligned(16))) float s_hidG[G][DALL];
  __shared__ float s_redG[G][4][4];
  __shared__ __attribute__((aligned(16))) float s_vecC[CH][5][N];  // w, kk (unnormalised), a, k, r
  __shared__ float s_vC[CH][N], s_gC[CH][N], s_yC[CH][N];        // mixed v, gate, y per channel
  __shared__ float s_invC[CH], s_bonC[CH];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i = t >> 2, qq = t & 3;
  int seg_i = bx, h = by;
  if (a.xmap) {  // 1-D grid: head h's workgroups share one XCD (as wkv6_body)
    const int b = bx, xcd = b & 7, j = b >> 3;
    h = xcd + 8 * (j / a.n_seg);
    seg_i = j % a.n_seg;
  }
  const int C = a.C, c = h * N + i;
  const int4 sg = a.segs[seg_i];
  const int slot = sg.x, r_begin = sg.y, n_rows = sg.z;
  uint4 lw[9];  // 8 bf16 per entry: w 0..1 | a 2..3 | v 4 | g 5..8 (launch_pack_lora6)
  {
    const uint4* pl = (const uint4*)(a.lup + (int64_t)h * 9 * 256 * 8);
#pragma unroll
    for (int u = 0; u < 9; ++u) lw[u] = pl[u * 256 + t];
  }
  const float w0 = a.w0[c], a0 = a.a0[c], v0 = a.v0[c], kkc = a.k_k[c], kac = a.k_a[c];
  const float rkc = a.r_k[c], lnw = a.lnx_w[c], lnb = a.lnx_b[c];
  const int64_t soff = a.layer_off + (int64_t)h * N * N + (int64_t)t * 4;
  float4_ S4[4];
  {
    const float4_* Sp = (const float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
#pragma unroll
    for (int q = 0; q < 4; ++q) S4[q] = Sp[q * 256];
  }
  const bool hid_thread = t < DALL / 4;
  auto quad_sum = [](float x) {
    x += dpp_mov<0xB1>(x);
    return x + dpp_mov<0x4E>(x);
  };
  auto dot = [&](float2_ acc, const uint4 q, const float* hsrc) {
    const float4_ h0 = *(const float4_*)hsrc;
    const float4_ h1 = *(const float4_*)(hsrc + 4);
    acc += w2f<F16>(q.x) * (float2_){h0[0], h0[1]};
    acc += w2f<F16>(q.y) * (float2_){h0[2], h0[3]};
    acc += w2f<F16>(q.z) * (float2_){h1[0], h1[1]};
    acc += w2f<F16>(q.w) * (float2_){h1[2], h1[3]};
    return acc;
  };
  for (int cb = 0; cb < n_rows; cb += CH) {
    const int nr = min(CH, n_rows - cb);
    // ---- A: the state-independent part, G rows per round
    for (int g0 = 0; g0 < nr; g0 += G) {
      float4_ hp[G][NP];
      float rp[G][NP], kp[G][NP], vp[G][NP], vf[G];
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        const int row = r_begin + cb + g0 + min(gi, nr - g0 - 1);  // (past the chunk: the last row again)
        const float* prow = a.part + (int64_t)row * a.ldp;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const float* pp = prow + p * a.part_stride;
          hp[gi][p] = *(const float4_*)(pp + 3 * C + (hid_thread ? 4 * t : 0));
          rp[gi][p] = pp[c];
          kp[gi][p] = pp[C + c];
          vp[gi][p] = pp[2 * C + c];
        }
        vf[gi] = a.layer > 0 ? a.v_first[(int64_t)row * a.ldv + c] : 0.f;
      }
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        if (hid_thread) {
          float4_ x = hp[gi][0];
#pragma unroll
          for (int p = 1; p < NP; ++p) x += hp[gi][p];
          float4_ y;
          if (t < DW / 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = ftanh(x[e]);
          } else if (t < (DW + DA + DV) / 4) {
            y = x;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = fsigm(x[e]);
          }
          *(float4_*)(&s_hidG[gi][4 * t]) = y;
        }
      }
      __syncthreads();
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        if (g0 + gi >= nr) break;
        const int rc = g0 + gi, row = r_begin + cb + rc;
        float r = rp[gi][0], k = kp[gi][0], v = vp[gi][0];
#pragma unroll
        for (int p = 1; p < NP; ++p) {
          r += rp[gi][p];
          k += kp[gi][p];
          v += vp[gi][p];
        }
        const float* sh = s_hidG[gi];
        float2_ l0 = {0.f, 0.f}, l1 = {0.f, 0.f}, l2 = {0.f, 0.f}, l3 = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) l0 = dot(l0, lw[u], sh + qq * (DW / 4) + u * 8);
#pragma unroll
        for (int u = 0; u < 2; ++u) l1 = dot(l1, lw[2 + u], sh + DW + qq * (DA / 4) + u * 8);
        l2 = dot(l2, lw[4], sh + DW + DA + qq * (DV / 4));
#pragma unroll
        for (int u = 0; u < 4; ++u) l3 = dot(l3, lw[5 + u], sh + DW + DA + DV + qq * (DG / 4) + u * 8);
        const float lo0 = quad_sum(l0[0] + l0[1]), lo1 = quad_sum(l1[0] + l1[1]);
        const float lo2 = quad_sum(l2[0] + l2[1]), lo3 = quad_sum(l3[0] + l3[1]);
        const float w = fexp(-0.60653066f * fsigm(w0 + lo0));
        const float av = fsigm(a0 + lo1);
        const float kk = k * kkc;
        k = k * (1.0f + (av - 1.0f) * kac);
        if (a.layer == 0) {
          if (qq == 0) a.v_first[(int64_t)row * a.ldv + c] = v;
        } else {
          v = v + (vf[gi] - v) * fsigm(v0 + lo2);
        }
        {
          const float ksq = wave_sum(qq == 0 ? kk * kk : 0.f);
          const float bon = wave_sum(qq == 0 ? r * k * rkc : 0.f);
          if (lane == 0) { s_redG[gi][0][wave] = ksq; s_redG[gi][1][wave] = bon; }
        }
        if (qq == 0) {
          s_vecC[rc][0][i] = w; s_vecC[rc][1][i] = kk; s_vecC[rc][2][i] = av; s_vecC[rc][3][i] = k;
          s_vecC[rc][4][i] = r;
          s_vC[rc][i] = v;
          s_gC[rc][i] = lo3;
        }
      }
      __syncthreads();
      if (t < G && g0 + t < nr) {  // the row's key-norm reciprocal and bonus, as every thread forms them
        const float* r0 = s_redG[t][0];
        const float* r1 = s_redG[t][1];
        s_invC[g0 + t] = __builtin_amdgcn_rcpf(fmaxf(sqrtf((r0[0] + r0[1]) + (r0[2] + r0[3])), 1e-12f));
        s_bonC[g0 + t] = (r1[0] + r1[1]) + (r1[2] + r1[3]);
      }
    }
    __syncthreads();
    // ---- B: the recurrence, row after row, registers and LDS only
    for (int rc = 0; rc < nr; ++rc) {
      const float inv = s_invC[rc];
      const float v = s_vC[rc][i];
      const float* vj = &s_vecC[rc][0][qq * 16];
      float2_ sa2 = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4_ kq = *(const float4_*)(vj + N + q * 4);
        sa2 += (float2_){S4[q][0], S4[q][1]} * (float2_){kq[0], kq[1]};
        sa2 += (float2_){S4[q][2], S4[q][3]} * (float2_){kq[2], kq[3]};
      }
      const float sa = quad_sum((sa2[0] + sa2[1]) * inv);
      float2_ y2 = {0.f, 0.f};
      const float2_ sav = {sa * inv, sa * inv}, vv = {v, v};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4_ wq = *(const float4_*)(vj + q * 4);
        const float4_ kq = *(const float4_*)(vj + N + q * 4);
        const float4_ aq = *(const float4_*)(vj + 2 * N + q * 4);
        const float4_ k4 = *(const float4_*)(vj + 3 * N + q * 4);
        const float4_ rq = *(const float4_*)(vj + 4 * N + q * 4);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          float2_ sv = (float2_){S4[q][e], S4[q][e + 1]} * (float2_){wq[e], wq[e + 1]};
          sv -= sav * ((float2_){kq[e], kq[e + 1]} * (float2_){aq[e], aq[e + 1]});
          sv += vv * (float2_){k4[e], k4[e + 1]};
          S4[q][e] = sv[0];
          S4[q][e + 1] = sv[1];
          y2 += sv * (float2_){rq[e], rq[e + 1]};
        }
      }
      const float y = quad_sum(y2[0] + y2[1]);
      if (qq == 0) s_yC[rc][i] = y;
    }
    __syncthreads();
    // ---- C: GroupNorm + bonus + gate, G rows per round, z planes out
    for (int g0 = 0; g0 < nr; g0 += G) {
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        if (g0 + gi >= nr) break;
        const float y = s_yC[g0 + gi][i];
        const float s1 = wave_sum(qq == 0 ? y : 0.f);
        const float s2 = wave_sum(qq == 0 ? y * y : 0.f);
        if (lane == 0) { s_redG[gi][2][wave] = s1; s_redG[gi][3][wave] = s2; }
      }
      __syncthreads();
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        if (g0 + gi >= nr) break;
        const int rc = g0 + gi, row = r_begin + cb + rc;
        const float mean = ((s_redG[gi][2][0] + s_redG[gi][2][1]) + (s_redG[gi][2][2] + s_redG[gi][2][3])) * (1.0f / N);
        const float var =
            fmaxf(((s_redG[gi][3][0] + s_redG[gi][3][1]) + (s_redG[gi][3][2] + s_redG[gi][3][3])) * (1.0f / N) - mean * mean, 0.f);
        if (qq == 0) {
          const float y = s_yC[rc][i], v = s_vC[rc][i], lo3 = s_gC[rc][i], bonus = s_bonC[rc];
          const float gn = (y - mean) * __builtin_amdgcn_rsqf(var + 64e-5f) * lnw + lnb;
          split_store((gn + bonus * v) * lo3, a.z_hi, a.z_lo, (int64_t)row * a.ldz + c, F16);
        }
      }
      __syncthreads();  // (s_redG / the chunk's LDS rows are reused)
    }
  }
  if (a.wt) {
    const auto rs = wt_rsrc(a.state + (int64_t)slot * a.slot_stride + a.layer_off + (int64_t)h * N * N);
#pragma unroll
    for (int q = 0; q < 4; ++q) store_wt(rs, (q * 256 + t) * 16, S4[q]);
  } else {
    float4_* Srow = (float4_*)(a.state + (int64_t)slot * a.slot_stride + soff);
#pragma unroll
    for (int q = 0; q < 4; ++q) Srow[q * 256] = S4[q];
  }
}

// (multi-row steps: two workgroups per CU -- without the bound the compiler took 256 VGPRs + 2 AGPRs,
// one wave per SIMD, so the 512 workgroups of a 32-slot prefill step ran in two rounds)
template <bool F16, bool MULTI_ROW = false>  // MULTI_ROW: steps whose segments hold several rows (wkv6_rows)
__global__ __launch_bounds__(256, MULTI_ROW ? 2 : 1) void k_wkv6(WkvArgs a) {
  tl_begin(a.tl);
  if constexpr (MULTI_ROW) wkv6_rows<F16>(a, blockIdx.x, blockIdx.y);
  else wkv6_body<F16, 0>(a, blockIdx.x, blockIdx.y, FfnSync{});
  tl_end(a.tl);
}

// ------------------------------------------------------------------------------------
// att_persist: the attention half of a decode step's layer as ONE launch:
//   blocks [0, n_ln_blocks)        LayerNorm 1 + six token-shift mixes of row b (k_ln1024's
//                                  arithmetic; layer 0 with the embedding folded in), planes /
//                                  residual / shift written through, counted into the LN replicas;
//   blocks [+0, +n_key)            rkv + LoRA-down workgroups (tile = b % tiles, split = b / tiles):
//                                  weights at dispatch, wait for the LN rows, X planes by sc1
//                                  loads, MFMA, partial slab written through, counted into their
//                                  head's counter (r / k / v tiles) or the LoRA-down replicas;
//   blocks [+n_key, +n_wkv)        WKV workgroups (slot, head; head h on one XCD): LoRA-up rows and
//                                  state at dispatch, wait for the head's tiles and the LoRA-down
//                                  tiles, partials by sc1 loads, z row written through, counted
//                                  into the head's WKV counter (two slots per workgroup, so that
//                                  every WKV workgroup is resident at dispatch, measured slower in
//                                  round 5: 758 -> 803 us per step at B = 32, 624 -> 655 at B = 1 --
//                                  a slot's WKV arithmetic is latency the second slot does not hide);
//   blocks [+n_wkv, +n_wo)         Wo workgroups (XCD-aware): weights at dispatch, wait for the
//                                  WKV workgroups of their K-slice's two heads, z by sc1 loads.
// Dependencies point to lower block indices only (see k_ffn_persist); outputs are the four
// launches', bit for bit. Block 0 zeroes the previous layer's counters.
// ------------------------------------------------------------------------------------
// FUSED (row-fused form, one decode row, layers > 0): no LayerNorm blocks; rkv workgroups compute
// the row's LN1 themselves (gemm2_body ROLE 5); the last workgroup waits until every rkv workgroup
// has staged (kAttRkvDone) and stores the residual and the new token-shift row.
template <bool F16, bool EMB, bool FUSED>
__global__ __launch_bounds__(256, RWKVTTS_ATT_WPC) void k_att_persist(LnMixArgs ln, GemmArgs ga, WkvArgs wa, GemmArgs go, FfnSync sy) {
  int b = blockIdx.x;
  tl_begin(ln.tl);
  sync_stamp(sy, 0);
  if (b < sy.n_ln_blocks) {  // (zeroing: as in k_ffn_persist)
    if (b == 0 && threadIdx.x < sy.n_prev) sy.cnt_prev[threadIdx.x * kSyncStride] = 0;
    if (b == 0 && threadIdx.x == 64 && sy.epoch_bump)  // a new pass for the granule hand-offs
      __hip_atomic_fetch_add((gint_t*)sy.epoch_bump, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (b < sy.ln_rows) {
      if constexpr (EMB) ln1024_body<F16, 1, 6, 0, true>(ln, b);
      else ln1024_body<F16, 1, 6, 16>(ln, b);
      sync_stamp(sy, 2);
      sync_arrive(sy.cnt + kSyncStride * kAttLn, kLnReplicas);
    }
  } else if ((b -= sy.n_ln_blocks) < sy.n_key) {
    if constexpr (FUSED) gemm2_body<1, 8, kXPlanes, F16, 1, 2, false, 5>(ga, b % sy.rkv_tiles, b / sy.rkv_tiles, sy, &ln);
    else gemm2_body<2, 8, kXPlanes, F16, 1, 2, false, 3>(ga, b % sy.rkv_tiles, b / sy.rkv_tiles, sy);
  } else if ((b -= sy.n_key) < sy.n_wkv) {
    if constexpr (FUSED && !EMB) {
      if (sy.gran) wkv6_body<F16, 2>(wa, b, 0, sy);
      else wkv6_body<F16, 1>(wa, b, 0, sy);
    } else {
      wkv6_body<F16, 1>(wa, b, 0, sy);
    }
  } else if ((b -= sy.n_wkv) < 16 * go.k_split || !FUSED) {
    if constexpr (FUSED && !EMB) {
      if (sy.gran) gemm2_body<1, 4, kXPlanes, F16, 1, 0, false, 8>(go, b, 0, sy);
      else gemm2_body<2, 4, kXPlanes, F16, 1, 0, false, 4>(go, b, 0, sy);
    } else {
      gemm2_body<2, 4, kXPlanes, F16, 1, 0, false, 4>(go, b, 0, sy);
    }
  } else if constexpr (FUSED && !EMB) {  // the shift writer
    if (threadIdx.x < sy.n_prev) sy.cnt_prev[threadIdx.x * kSyncStride] = 0;
    if (threadIdx.x == 64 && sy.epoch_bump)
      __hip_atomic_fetch_add((gint_t*)sy.epoch_bump, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sync_wait(sy.cnt + kSyncStride * kAttRkvDone, sy.n_key, sy.err, 2048, sy.opts);
    ln1024_body<F16, 1, 0, 16>(ln, 0);
  }
  sync_stamp(sy, 3);
  tl_end(ln.tl);
}

struct AttPrep {
  LnMixArgs l;
  GemmArgs ga, gw;
  WkvArgs wa;
  FfnSync sy;
};
static bool prep_att_persist(const LnMixArgs& ln, const GemmArgs& rkv, const WkvArgs& wkv, const GemmArgs& wo, int* cnt,
                             int* cnt_prev, int* err, int R, int H, uint64_t* stamps, int opts, AttPrep& P) {
  const bool emb = ln.emb != nullptr;
  const int rkv_tiles = rkv.seg[rkv.nseg - 1].tile_start + (rkv.seg[rkv.nseg - 1].N + 63) / 64;
  const int lora_tiles = rkv_tiles - 3 * ln.C / 64;
  if (ln.C != 1024 || H != 16 || !ln.shift || ln.n_mix != 6 || ln.n_part != (emb ? 0 : 16) || R < 1 || R > 32 ||
      rkv.xmode != kXPlanes || rkv.n_tinfo != rkv_tiles || rkv.kslice != 256 || rkv.k_split != 4 || rkv.M != R ||
      rkv.q_fmt || rkv.stamps || rkv.xalign || lora_tiles < 1 || rkv.ldo != wkv.ldp ||
      wkv.perm != 2 || wkv.n_part != 4 || wkv.multi_row || !wkv.allow_xmap || wkv.n_seg != R || wkv.stamps ||
      wkv.Dw != 64 || wkv.Da != 64 || wkv.Dv != 32 || wkv.Dg != 128 ||
      wo.xmode != kXPlanes || wo.kslice != 128 || wo.k_split != 8 || wo.nseg != 1 || wo.M != R || wo.q_fmt ||
      wo.stamps || (wo.seg[0].N + 63) / 64 != 16 ||
      rkv.f16 != ln.f16 || wo.f16 != ln.f16 || wkv.f16 != ln.f16 || cnt == cnt_prev)
    return false;
  LnMixArgs& l = P.l;
  l = ln;
  l.n_rows = R;
  l.wt = 1;
  GemmArgs& ga = P.ga;
  GemmArgs& gw = P.gw;
  ga = rkv;
  gw = wo;
  ga.xmap = 0; ga.ntiles = rkv_tiles; ga.wt = 1;
  gw.xmap = 1; gw.ntiles = 16;
  gw.wt = 1;
  WkvArgs& wa = P.wa;
  wa = wkv;
  wa.xmap = 1; wa.wt = 1;
  FfnSync& sy = P.sy;
  sy = FfnSync{};
  sy.cnt = cnt;
  sy.cnt_prev = cnt_prev;
  sy.n_prev = kAttCounters;
  sy.err = err;
  sy.n_ln_blocks = 32;
  sy.ln_rows = R;
  sy.n_key = rkv_tiles * rkv.k_split;
  sy.rkv_tiles = rkv_tiles;
  sy.n_wkv = R * H;
  sy.head_target = 3 * rkv.k_split;
  sy.lora_target = lora_tiles * rkv.k_split;
  sy.C = ln.C;
  sy.opts = opts;
  prefetch_holds(sy);
  sy.stamps = stamps;
  return true;
}

// the attention half's arguments, its row-fused form (n_fix = 1: the trailing shift writer) and
// the granule hand-offs where they apply
static bool att_setup(const LnMixArgs& ln, const GemmArgs& rkv, const WkvArgs& wkv, const GemmArgs& wo, int* cnt,
                      int* cnt_prev, int* err, int R, int H, uint64_t* stamps, int opts, int* drop, bool fused_ln,
                      int* epoch_bump, uint64_t* gran, const int* epoch, AttPrep& P, int& n_fix) {
  if (!prep_att_persist(ln, rkv, wkv, wo, cnt, cnt_prev, err, R, H, stamps, opts, P)) return false;
  P.sy.drop = drop;
  P.sy.epoch_bump = epoch_bump;
  const bool fused = fused_ln && R == 1 && ln.emb == nullptr && ln.inplace;
  n_fix = 0;
  if (fused) {
    P.sy.n_ln_blocks = 0;
    P.sy.d_w = 0;  // (the hold only kept the weight streams off the LayerNorm rows' loads)
    P.sy.d_late = kHold1Wo;
    n_fix = 1;
    // the granule hand-off WKV -> Wo: 64-channel heads, 128-channel Wo K-slices (its granule role's KS)
    if (gran && epoch && wkv.C == 16 * 64 && wo.k_split == 8 && ln.layer < 64) {
      P.sy.gran = gran;
      P.sy.zgran = gran;
      P.sy.gran_ld = 0;
      P.sy.epoch = epoch;
      P.sy.layer = ln.layer;
    }
  }
  return true;
}

bool launch_att_persist(const LnMixArgs& ln, const GemmArgs& rkv, const WkvArgs& wkv, const GemmArgs& wo, int* cnt,
                        int* cnt_prev, int* err, int R, int H, hipStream_t st, uint64_t* stamps, int opts,
                        int* drop, bool fused_ln, int* epoch_bump, uint64_t* gran, const int* epoch) {
  AttPrep P;
  int n_fix = 0;  // the row-fused form's shift writer
  if (!att_setup(ln, rkv, wkv, wo, cnt, cnt_prev, err, R, H, stamps, opts, drop, fused_ln, epoch_bump, gran, epoch, P,
                 n_fix))
    return false;
  const bool fused = n_fix == 1;
  const bool emb = ln.emb != nullptr;
  LnMixArgs& l = P.l;
  GemmArgs& ga = P.ga;
  GemmArgs& gw = P.gw;
  WkvArgs& wa = P.wa;
  FfnSync& sy = P.sy;
  const int n_wo = 16 * wo.k_split;
  const size_t lds = (size_t)2 * 16 * (8 * 32 + 8) * 2 * 2;  // the rkv body's X image (the largest)
  const dim3 grid(sy.n_ln_blocks + sy.n_key + sy.n_wkv + n_wo + n_fix);
  if (ln.f16) {
    if (emb) RT_LAUNCH((k_att_persist<true, true, false>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
    else if (fused) RT_LAUNCH((k_att_persist<true, false, true>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
    else RT_LAUNCH((k_att_persist<true, false, false>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
  } else {
    if (emb) RT_LAUNCH((k_att_persist<false, true, false>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
    else if (fused) RT_LAUNCH((k_att_persist<false, false, true>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
    else RT_LAUNCH((k_att_persist<false, false, false>), grid, dim3(256), lds, st, l, ga, wa, gw, sy);
  }
  return true;
}

int wkv_perm_layout(int Dw, int Da, int Dv, int Dg, int n_part, int max_slots, int variant) {
  if (!(Dw == 64 && Da == 64 && Dv == 32 && Dg == 128 && n_part == 4)) return 0;
  if (variant == 1 || variant == 2) return variant;
  // auto: k_wkv6 (measured, timeline of a graph-replayed 32-slot step: 4.85 vs 5.33 us per
  // launch once its loads are issued in need order and the XCD-aware grid keeps a head's
  // LoRA-up rows in one L2; 1 % faster at one slot as well)
  (void)max_slots;
  return 2;
}
int launch_wkv(const WkvArgs& a, int n_seg, int H, hipStream_t st) {
  const dim3 grid(n_seg, H);
  if (a.Dw == 64 && a.Da == 64 && a.Dv == 32 && a.Dg == 128 && a.n_part == 4 && (a.perm == 1 || a.perm == 2)) {
    WkvArgs b = a;
    b.xmap = (H % 8 == 0 && a.allow_xmap) ? 1 : 0;
    b.n_seg = n_seg;
    const dim3 g = b.xmap ? dim3(n_seg * H) : grid;
    if (a.perm == 2) {
      if (a.multi_row) {
        if (a.f16) RT_LAUNCH((k_wkv6<true, true>), g, dim3(256), 0, st, b);
        else RT_LAUNCH((k_wkv6<false, true>), g, dim3(256), 0, st, b);
      } else {
        if (a.f16) RT_LAUNCH((k_wkv6<true>), g, dim3(256), 0, st, b);
        else RT_LAUNCH((k_wkv6<false>), g, dim3(256), 0, st, b);
      }
    } else {
      if (a.f16) RT_LAUNCH((k_wkv4<true>), g, dim3(128), 0, st, b);
      else RT_LAUNCH((k_wkv4<false>), g, dim3(128), 0, st, b);
    }
    return n_seg * H;
  }
  if (a.Dw == 16 && a.Da == 16 && a.Dv == 16 && a.Dg == 32 && a.n_part <= 1) {
    RT_LAUNCH((k_wkv2<16, 16, 16, 32, 1>), grid, dim3(128), 0, st, a);
    return n_seg * H;
  }
  if (a.Dw == 32 && a.Da == 32 && a.Dv == 16 && a.Dg == 64 && a.n_part <= 1) {
    RT_LAUNCH((k_wkv2<32, 32, 16, 64, 1>), grid, dim3(128), 0, st, a);
    return n_seg * H;
  }
  const int units = (a.Dw + a.Da + a.Dv + a.Dg + 15) / 16;
  if (units <= 8 && a.n_part <= 4) RT_LAUNCH((k_wkv<8, 4>), grid, dim3(256), 0, st, a);
  else if (units <= 20 && a.n_part <= 4) RT_LAUNCH((k_wkv<20, 4>), grid, dim3(256), 0, st, a);
  else RT_LAUNCH((k_wkv<32, 8>), grid, dim3(256), 0, st, a);
  return n_seg * H;
}

}  // namespace rwkvtts
