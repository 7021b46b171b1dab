// codec.hip -- MI355X BiCodec decoder: replaces the ORT CPU session that runs
// BiCodecDetokenize.onnx at src/lightweight_tts_pipeline.rs:706-730 (decode_audio :606-622,
// decode_audio_batch :625-703).  Architecture: include/rwkvtts_codec_layout.h.
//
// Every conv / ConvTranspose / pointwise linear of the decoder runs through ONE implicit-GEMM
// MFMA kernel (k_conv): D[t][co] = sum_{tap, ci} act(X[pos(t, tap)][ci]) * W[co][tap][ci], with
//   * activations f32 channel-last [t][c] in HBM, staged into LDS as bf16 hi + lo planes
//     (x = hi + lo to ~2^-17 relative) so two bf16 MFMAs give ~f32 products against the
//     bf16 weights (the synthetic codec weights are bf16-exact);
//   * the Snake1d of the producing block fused into the staging (x + sin^2(a x) / (a + 1e-9));
//   * ConvTranspose1d(k, s, p=(k-s)/2) decomposed into s output phases, each a stride-1 conv
//     with ceil((k - kr)/s) taps -- no zero-stuffed input, no wasted MACs;
//   * bias, GELU, layer-scale gamma, residual add and a per-utterance bias (+ d_vector) fused
//     into the epilogue.
// Utterances of one batch run in the same launches (blockIdx.z), each with its own length.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "../../include/rwkvtts_codec_layout.h"

namespace rwkvtts {

typedef __bf16 cbf16x8 __attribute__((ext_vector_type(8)));

struct ConvArgs {
  const bf16_t* xh;  // input planes (already activated): x = hi + lo, channel-last [t][Ci]
  const bf16_t* xl;
  int64_t x_bs;      // per-utterance stride (elements)
  int Ci, tin_mul;
  const bf16_t* w;   // [Co][K][Ci]: bf16 hi part of the f32 weights
  const bf16_t* wl;  // WLO kernels: bf16 lo part (w_f32 = hi + lo to ~2^-16 relative)
  int K, Co;
  int mode;          // 0: conv (dil, pad), 1: ConvTranspose (stride s, pad (K - s) / 2)
  int dil, pad, s;
  const float* bias;   // [Co]
  const float* rbias;  // per-utterance bias [n][Co] (nullable)
  int64_t rb_bs;
  const float* gamma;  // epilogue scale (nullable)
  const float* res;    // f32 residual, layout of y (nullable; may alias y)
  int act;             // 0 none, 1 exact GELU
  float* y;            // f32 output (nullable)
  bf16_t* yh;          // output planes (nullable): act_out(v) split hi + lo
  bf16_t* yl;
  const float* y_alpha;  // Snake1d alpha applied to the planes output (nullable)
  int64_t y_bs;
  // FUSE kernels (a whole residual unit at 96 channels: conv7 -> Snake -> conv1 -> + residual):
  // the conv7 result (+ bias) goes through Snake(mid_alpha) into an LDS image of bf16 hi + lo
  // planes, the pointwise conv w1 ([Co][Co]) runs on it, and the epilogue above uses bias1
  const float* mid_alpha;
  const bf16_t* w1;
  const float* bias1;
  const int* ntok;     // tokens per utterance; input length = ntok * tin_mul
  const bf16_t* zeros; // >= 16 zero bytes (source of out-of-range window rows)
  // channel-blocked planes: [C / 32][rows][32] per utterance, the chunk stride (rows * 32 elements)
  // given; 0: channel-last [t][C]. A 32-channel chunk's window is then one contiguous run of
  // 64-B rows instead of 64 B out of every C * 2-B row.
  int64_t x_cs, y_cs;
  // XCD-aware 1-D grid (xmap = 1): the gy column tiles of time tile x run back to back on one XCD
  // (blocks b and b + 8 share one), so the input window they all read is fetched into that XCD's
  // L2 once instead of once per column tile
  int xmap, gx, gy;
};

__device__ inline float snake(float v, float a) {
  const float s = sinf(a * v);
  return v + (1.0f / (a + 1e-9f)) * (s * s);
}
// Snake with the hardware sine (v_sin_f32; |error| ~1e-6 for the |a x| < ~100 seen here)
__device__ inline float snake_fast(float v, float a) {
  const float s = __sinf(a * v);
  return v + (1.0f / (a + 1e-9f)) * (s * s);
}
__device__ inline void split_store(bf16_t* h, bf16_t* l, int64_t o, float v) {
  const uint16_t hb = f32_to_bf16(v);
  h[o] = hb;
  l[o] = f32_to_bf16(v - bf16_to_f32(hb));
}

// output rows (time) per workgroup: 32 per wave. The 7-tap convolutions run 8-wave workgroups
// (256 rows): their double-buffered chunk window (the 7 taps' weights + the activation window,
// 92-104 KB at 128 rows) leaves room for one workgroup per CU only, so a 4-wave workgroup would
// run one wave per SIMD and expose every wait; 8 waves share the same weight tiles.
constexpr int conv_waves(int KT) { return KT == 7 ? 8 : 4; }
// 16-row staging blocks per wave and chunk (one buffer offset register each): 17 for the 4-wave
// fused residual unit, whose dilation-9 window (192 rows, hi + lo) and 7-tap weights are 66 blocks
constexpr int conv_maxb(int nwv, bool fuse) { return fuse && nwv == 4 ? 17 : 16; }
template <int NWV, bool FUSE> struct ConvMaxB { static constexpr int v = FUSE && NWV == 4 ? 17 : 16; };

// every k_conv instantiation the host dispatches: (column tile, taps class, weight lo plane, waves)
#define RT_CONV_KERNELS(X)                                                                       \
  X(32, 1, false, 4) X(32, 3, false, 4) X(32, 7, false, 8) X(48, 1, false, 4) X(48, 3, false, 4)    \
  X(48, 7, false, 8) X(64, 1, false, 4) X(64, 3, false, 4) X(64, 7, false, 8) X(96, 1, false, 4)    \
  X(96, 3, false, 4) X(96, 7, false, 8) X(192, 1, false, 4)                                         \
  X(32, 1, true, 4) X(48, 1, true, 4) X(64, 1, true, 4) X(96, 1, true, 4)                           \
  X(32, 3, true, 4) X(48, 3, true, 4) X(64, 3, true, 4) X(96, 3, true, 4)                           \
  X(32, 7, true, 8) X(48, 7, true, 8) X(64, 7, true, 8) X(96, 7, true, 8)                           \
  X(48, 7, true, 4) X(64, 7, true, 4) X(96, 7, true, 4)
// fused residual units (conv7 -> Snake -> conv1 in one launch, 96 channels, bf16-exact weights)
#define RT_CONV_FUSED(X) X(96, 7, false, 8) X(96, 7, false, 4)

// LDS image of a 32-channel chunk: 64-B rows of four 16-B pieces, piece p of row r stored at
// slot p ^ ((r >> 1) & 3): the MFMA fragment reads (16 rows x 4 pieces per ds_read_b128 lane
// group) are then bank-conflict free. The image is filled by global_load_lds_dwordx4 (one
// 1-KiB, 16-row block per wave-instruction, LDS destination lane-linear), so the swizzle is
// applied to each lane's SOURCE address and undone by the reads (the same involution).
__device__ inline int swz(int row, int piece) { return row * 64 + ((piece ^ ((row >> 1) & 3)) << 4); }
__device__ inline void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// Workgroup = NWV waves along time, each 32 rows x TN channels (2 x TN/16 MFMA 16x16x32 tiles).
// Per 32-channel chunk the workgroup stages (double-buffered, async global->LDS) the input
// window that ALL taps read -- TM + (ntaps - 1) * |tap stride| rows of the hi and lo planes --
// and the chunk of every tap's weights, then runs ntaps x 2 x NT x 2 MFMAs per wave while the
// next chunk streams in. WLO: f32 weights that bf16 cannot hold (real checkpoints; the reference
// runs this decoder in fp32 on ORT) are staged as hi + lo planes too, and every product takes a
// third MFMA x_hi * w_lo: weights enter at ~2^-16 relative, as the activations do. With w_lo = 0
// the third MFMA adds exact zeros, so a WLO launch on bf16-exact weights is bit-identical.
// (A single-buffered variant at two workgroups per CU measured the vocoder alone 2 ms faster but
// left no LDS for a decode workgroup beside it, and the bench equal or lower: DESIGN.md §14.)
template <int TN, int KT, bool WLO = false, int NWV = conv_waves(KT), bool FUSE = false>
__global__ __launch_bounds__(64 * NWV, NWV == 8 ? 1 : 2) void k_conv(ConvArgs a) {
  constexpr int TM = 32 * NWV, NT = TN / 16;
  static_assert(!FUSE || (TN == 96 && !WLO), "fused residual unit: 96 channels, bf16-exact weights");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int req = blockIdx.z;
  const int Tin = a.ntok[req] * a.tin_mul;
  int bx = blockIdx.x, by = blockIdx.y;
  if (a.xmap) {
    const int k = blockIdx.x >> 3;
    by = k % a.gy;
    bx = (blockIdx.x & 7) + 8 * (k / a.gy);
    if (bx >= a.gx) return;
  }
  const int q0 = bx * TM;
  if (q0 >= Tin) return;
  const int ncot = a.Co / TN;
  const int phase = by / ncot, co0 = (by % ncot) * TN;
  int ntaps, k0, kstep, pbase, pstep, ostr;
  if (a.mode == 0) {
    ntaps = a.K; k0 = 0; kstep = 1; pbase = -a.pad; pstep = a.dil; ostr = 1;
  } else {
    const int p = (a.K - a.s) / 2, kr = (phase + p) % a.s;
    ntaps = (a.K - kr + a.s - 1) / a.s; k0 = kr; kstep = a.s; pbase = (phase + p - kr) / a.s;
    pstep = -1; ostr = a.s;
  }
  const int span = (ntaps - 1) * (pstep < 0 ? -pstep : pstep);
  const int WRp = (TM + span + 15) & ~15;  // window rows, whole 16-row blocks
  const int wlo = pstep < 0 ? -span : 0;   // window row 0 <-> position q0 + pbase + wlo
  const int wstart = q0 + pbase + wlo;
  const int nWblk = ntaps * (TN / 16);  // one weight plane's blocks
  const int nAblk = 2 * WRp / 16, nblk = nAblk + (WLO ? 2 : 1) * nWblk;
  const int buf_bytes = nblk * 1024;
  // wave index read back as a scalar: every per-wave decision below (which staging blocks a wave
  // issues) is then a scalar branch instead of an exec-masked one
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), li = lane & 15, g = lane >> 4;
  const int64_t xoff = req * a.x_bs;
  const int nck = a.Ci / 32;
  const int lrow = lane >> 2, lslot = lane & 3;

  // This wave's share of the chunk's 16-row blocks, staged by buffer loads straight into LDS:
  // per block u a 32-bit byte offset (per lane, computed once) into one of four buffer resources
  // (this utterance's input hi / lo plane, the weights' hi / lo plane); a chunk adds a scalar
  // offset (the input's chunk stride, or 32 channels of weights). Out-of-range window rows get
  // an offset past the resources' range, which the buffer load returns as zeros.
  constexpr int MAXB = ConvMaxB<NWV, FUSE>::v;
  constexpr uint32_t kOob = 0x80000000u;
  auto rsrc = [](const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rxh = rsrc(a.xh + xoff), rxl = rsrc(a.xl + xoff), rwh = rsrc(a.w),
                               rwl = rsrc(WLO ? a.wl : a.w);
  static_assert(MAXB <= 17, "staging offsets");
  uint32_t voff[17];  // (a constant bound: a template-dependent one made hipcc drop every k_conv host stub)
#pragma unroll
  for (int u = 0; u < MAXB; ++u) {
    const int b = wave + NWV * u;
    uint32_t o = kOob;
    if (b < nAblk) {
      const int plane = b >= WRp / 16, row = (b - plane * (WRp / 16)) * 16 + lrow;
      const int piece = lslot ^ ((row >> 1) & 3), pos = wstart + row;
      if (pos >= 0 && pos < Tin) o = (uint32_t)(pos * (a.x_cs ? 32 : a.Ci) + piece * 8) * 2u;
    } else if (b < nblk) {
      const int wb0 = b - nAblk, lo = wb0 >= nWblk, wb = wb0 - (lo ? nWblk : 0);
      const int tap = wb / (TN / 16), co = (wb % (TN / 16)) * 16 + lrow;
      const int piece = lslot ^ ((co >> 1) & 3);
      o = (uint32_t)((((co0 + co) * a.K + k0 + tap * kstep) * a.Ci + piece * 8) * 2);
    }
    voff[u] = o;
  }
  auto issue = [&](int ck, uint8_t* buf) {
    const int aso = (int)((a.x_cs ? ck * a.x_cs : ck * 32) * 2), wso = ck * 64;  // bytes
#pragma unroll
    for (int u = 0; u < MAXB; ++u) {
      const int b = __builtin_amdgcn_readfirstlane(wave + NWV * u);  // wave-uniform: scalar branches
      if (b >= nblk) continue;
      auto* dst = (__attribute__((address_space(3))) void*)(buf + b * 1024);
      // one call site per resource: the resource stays in SGPRs
      if (b < nAblk) {
        if (b >= WRp / 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rxl, dst, 16, voff[u], aso, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rxh, dst, 16, voff[u], aso, 0, 0);
      } else if (WLO && b - nAblk >= nWblk) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rwl, dst, 16, voff[u], wso, 0, 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rwh, dst, 16, voff[u], wso, 0, 0);
      }
    }
  };

  float4_ acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = (float4_){0.f, 0.f, 0.f, 0.f};

  auto mma_tap = [&](const uint8_t* cur, int j) {
    const uint8_t* sA = cur;
    const uint8_t* sW = cur + nAblk * 1024;
    const uint8_t* sWl = sW + nWblk * 1024;
    {
      short8 bw[NT], bwl[WLO ? NT : 1];
#pragma unroll
      for (int n = 0; n < NT; ++n) bw[n] = *(const short8*)(sW + j * TN * 64 + swz(n * 16 + li, g));
      if constexpr (WLO) {
#pragma unroll
        for (int n = 0; n < NT; ++n) bwl[n] = *(const short8*)(sWl + j * TN * 64 + swz(n * 16 + li, g));
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int wr = wave * 32 + m * 16 + li + j * pstep - wlo;
        const short8 ah = *(const short8*)(sA + swz(wr, g));
        const short8 al = *(const short8*)(sA + WRp * 64 + swz(wr, g));
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, ah),
                                                              __builtin_bit_cast(cbf16x8, bw[n]), acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, al),
                                                              __builtin_bit_cast(cbf16x8, bw[n]), acc[m][n], 0, 0, 0);
          if constexpr (WLO)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, ah),
                                                                __builtin_bit_cast(cbf16x8, bwl[n]), acc[m][n], 0, 0, 0);
        }
      }
    }
  };
  // (a hand-pipelined form -- tap j + 1's fragments requested before tap j's MFMAs, two register
  // sets, scheduling barriers -- measured 1-3 % slower per 7-tap launch: not the bound)
  auto mma_chunk = [&](const uint8_t* cur) {
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      if (j >= ntaps) break;
      mma_tap(cur, j);
    }
  };
  issue(0, lds);
  for (int ck = 0; ck < nck; ++ck) {
    __syncthreads();  // chunk ck has landed; every wave is done with the other buffer
    uint8_t* cur = lds + (ck & 1) * buf_bytes;
    if (ck + 1 < nck) issue(ck + 1, lds + ((ck + 1) & 1) * buf_bytes);
    mma_chunk(cur);
  }
  if constexpr (FUSE) {
    // ---- residual unit, second half: v = conv7 + bias -> Snake(mid_alpha) -> hi + lo planes in an
    // LDS image laid out like a chunk window (3 chunks of 32 channels, rows = the TM time rows),
    // W1 staged beside it, the pointwise conv on the image; the epilogue below then adds bias1
    // and the residual. Saves the intermediate planes' HBM round trip (4 B per element).
    constexpr int LDE0 = TN + 4;
    constexpr int NCH = TN / 32;
    __syncthreads();  // every wave is done with the chunk buffers
    float* sE0 = (float*)lds + wave * 32 * LDE0;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const float b = a.bias[co0 + n * 16 + li];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) sE0[(m * 16 + 4 * g + j) * LDE0 + n * 16 + li] = acc[m][n][j] + b;
    }
    constexpr int NIT0 = TN / 8;
    // a lane's channels repeat with period 3 over the iterations (TN = 96): alphas and reciprocals
    // taken once; hi / lo by the hardware RNE convert (the bits of f32_to_bf16)
    float ma[3][4], mi[3][4];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ma[p][e] = a.mid_alpha[co0 + ((lane + 64 * p) % (TN / 4)) * 4 + e];
        mi[p][e] = 1.0f / (ma[p][e] + 1e-9f);
      }
    uint2 ph[NIT0], pl[NIT0];
#pragma unroll
    for (int it = 0; it < NIT0; ++it) {
      const int idx = lane + 64 * it, r = idx / (TN / 4), c4 = (idx % (TN / 4)) * 4;
      const float4_ v = *(const float4_*)(sE0 + r * LDE0 + c4);
      float pv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float s = __sinf(ma[it % 3][e] * v[e]);
        pv[e] = v[e] + mi[it % 3][e] * (s * s);
      }
      uint32_t h01, l01, h23, l23;
      split2<false>(pv[0], pv[1], h01, l01);
      split2<false>(pv[2], pv[3], h23, l23);
      ph[it] = make_uint2(h01, h23);
      pl[it] = make_uint2(l01, l23);
    }
    __syncthreads();  // every wave has read its sE0 tile: the image may overwrite it
    uint8_t* img = lds;                              // [NCH][2 planes][TM rows][64 B]
    uint8_t* wimg = lds + NCH * 2 * TM * 64;         // [NCH][TN rows][64 B]
#pragma unroll
    for (int it = 0; it < NIT0; ++it) {
      const int idx = lane + 64 * it, r = idx / (TN / 4), c4 = (idx % (TN / 4)) * 4;
      const int row = wave * 32 + r, ch = c4 >> 5, piece = (c4 & 31) >> 3, half = (c4 & 7) >> 2;
      uint8_t* base = img + ch * 2 * TM * 64 + swz(row, piece) + half * 8;
      *(uint2*)base = ph[it];
      *(uint2*)(base + TM * 64) = pl[it];
    }
    // W1 [Co][Ci = TN] chunks into the swizzled image (16-row blocks, one per wave-instruction)
    for (int blk = wave; blk < NCH * (TN / 16); blk += NWV) {
      const int ch = blk / (TN / 16), co = (blk % (TN / 16)) * 16 + lrow;
      const int piece = lslot ^ ((co >> 1) & 3);
      glds16(a.w1 + (int64_t)(co0 + co) * a.Co + ch * 32 + piece * 8, wimg + ch * TN * 64 + (blk % (TN / 16)) * 1024);
    }
    __syncthreads();  // the image and W1 have landed
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[m][n] = (float4_){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      short8 bw[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) bw[n] = *(const short8*)(wimg + ch * TN * 64 + swz(n * 16 + li, g));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int wr = wave * 32 + m * 16 + li;
        const short8 ah = *(const short8*)(img + ch * 2 * TM * 64 + swz(wr, g));
        const short8 al = *(const short8*)(img + ch * 2 * TM * 64 + TM * 64 + swz(wr, g));
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, ah),
                                                              __builtin_bit_cast(cbf16x8, bw[n]), acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, al),
                                                              __builtin_bit_cast(cbf16x8, bw[n]), acc[m][n], 0, 0, 0);
        }
      }
    }
  }
  // Epilogue. (1) bias / GELU / gamma in the MFMA layout (col = lane & 15 -> co,
  // row = 4 * (lane >> 4) + j -> q), staged through this wave's LDS tile [32][TN + 4] f32;
  // (2) read back row-contiguous so each lane moves 16 B of f32 (residual, y) and 8 B per
  // plane, with the output Snake applied once per element.
  // TN = 96 (the pointwise conv of the last stage, memory-bound): residual rows (f32,
  // row-contiguous, this lane's epilogue elements) are requested now, before any store -- res may
  // alias y, and loads issued after a store to y cannot be hoisted above it (every element is read
  // and then written by the same lane, so the early read is the same value). 1.2x on that launch;
  // at TN 32 / 64 the 8-16 extra float4 registers cost more occupancy than they save.
  const int64_t yoff = req * a.y_bs;
  constexpr int NIT = TN / 8;
  constexpr bool kPreRes = TN == 96;
  float4_ rv[kPreRes ? NIT : 1];
#pragma unroll
  for (int it = 0; it < (kPreRes ? NIT : 0); ++it) {
    const int idx = lane + 64 * it, r = idx / (TN / 4), c4 = (idx % (TN / 4)) * 4;
    const int q = q0 + wave * 32 + r;
    rv[it] = (float4_){0.f, 0.f, 0.f, 0.f};
    if (a.res && q < Tin) rv[it] = *(const float4_*)(a.res + yoff + (int64_t)(q * ostr + phase) * a.Co + co0 + c4);
  }
  __syncthreads();  // every wave is done with the chunk buffers
  constexpr int LDE = TN + 4;
  constexpr int NH = 1, RH = 32 / NH;  // epilogue passes, rows per pass
  float* sE = (float*)lds + wave * RH * LDE;
  // A lane's readback channels repeat with period kCP over the iterations (1 for TN 32 / 64, 3 for
  // TN 48 / 96 / 192): their Snake alphas and 1 / (alpha + 1e-9) are taken once (the stores below
  // may alias y_alpha as far as the compiler knows, so it would reload and divide per element).
  // The planes' hi / lo split is the hardware RNE convert (split2: the bits of f32_to_bf16).
  constexpr int kGcd = (TN / 4) % 16 == 0 ? 16 : ((TN / 4) % 8 == 0 ? 8 : 4);  // gcd(64, TN / 4)
  constexpr int kCP = (TN / 4) / kGcd;
  static_assert(kCP <= 3 && NIT % kCP == 0, "readback channel period");
  float ya[kCP][4], yi[kCP][4];
#pragma unroll
  for (int p = 0; p < kCP; ++p) {
    const int c4 = ((lane + 64 * p) % (TN / 4)) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ya[p][e] = a.y_alpha ? a.y_alpha[co0 + c4 + e] : 0.f;
      yi[p][e] = 1.0f / (ya[p][e] + 1e-9f);
    }
  }
#pragma unroll
  for (int hh = 0; hh < NH; ++hh) {
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int co = co0 + n * 16 + li;
    const float b = (FUSE ? a.bias1 : a.bias)[co] + (a.rbias ? a.rbias[req * a.rb_bs + co] : 0.0f);
    const float gm = a.gamma ? a.gamma[co] : 1.0f;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (NH == 2 && m != hh) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[m][n][j] + b;
        if (a.act == 1) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
        sE[((NH == 2 ? 0 : m * 16) + 4 * g + j) * LDE + n * 16 + li] = v * gm;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < NIT / NH; ++it) {
    const int idx = lane + 64 * it, r = idx / (TN / 4), c4 = (idx % (TN / 4)) * 4;
    const int q = q0 + wave * 32 + hh * RH + r;
    if (q >= Tin) continue;
    float4_ v = *(const float4_*)(sE + r * LDE + c4);
    const int64_t o = yoff + (int64_t)(q * ostr + phase) * a.Co + co0 + c4;
    if (a.res) {
      if constexpr (kPreRes) v += rv[it];
      else v += *(const float4_*)(a.res + o);
    }
    if (a.y) *(float4_*)(a.y + o) = v;
    if (a.yh) {
      const int64_t op = a.y_cs ? yoff + ((co0 + c4) >> 5) * a.y_cs + (int64_t)(q * ostr + phase) * 32 + ((co0 + c4) & 31) : o;
      float pv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pv[e] = v[e];
        if (a.y_alpha) {
          const float al = ya[it % kCP][e], inv = yi[it % kCP][e];
          const float s = __sinf(al * v[e]);
          pv[e] = v[e] + inv * (s * s);
        }
      }
      uint32_t h01, l01, h23, l23;
      split2<false>(pv[0], pv[1], h01, l01);
      split2<false>(pv[2], pv[3], h23, l23);
      *(uint2*)(a.yh + op) = make_uint2(h01, h23);
      *(uint2*)(a.yl + op) = make_uint2(l01, l23);
    }
  }
  }
}

// semantic FVQ: z[t][c] = b[c] + sum_k W[c][k] * codebook[tok][k]   (-> planes)
__global__ void k_fvq(const int* tok, int Tmax, const int* ntok, const float* cb, int cd,
                      const float* w, const float* b, int L, bf16_t* zh, bf16_t* zl) {
  const int t = blockIdx.x, req = blockIdx.y;
  if (t >= ntok[req]) return;
  const float* e = cb + (int64_t)tok[req * Tmax + t] * cd;
  const int64_t base = ((int64_t)req * Tmax + t) * L;
  for (int c = threadIdx.x; c < L; c += blockDim.x) {
    float acc = 0.0f;
    for (int k = 0; k < cd; ++k) acc += w[c * cd + k] * e[k];
    split_store(zh, zl, base + c, acc + b[c]);
  }
}

// speaker FSQ: h[c * G + t] = b[c] + sum_k W[c][k] * code_k(global[t])
__global__ void k_fsq(const int* glob, int G, int levels, int dims, const float* w, const float* b,
                      int Q, float* h) {
  const int req = blockIdx.x;
  for (int i = threadIdx.x; i < Q * G; i += blockDim.x) {
    const int c = i / G, t = i % G;
    int idx = glob[req * G + t];
    const int half = levels / 2;
    float acc = 0.0f;
    for (int k = 0; k < dims; ++k) {
      const float code = (float)((idx % levels) - half) / (float)half;
      idx /= levels;
      acc += w[c * dims + k] * code;
    }
    h[(int64_t)req * Q * G + i] = acc + b[c];
  }
}

// out[req][r] = b[r] + W[r] . v[req]   (one wave per output row)
__global__ __launch_bounds__(256) void k_gemv(const float* w, const float* b, int rows, int cols,
                                              const float* v, int64_t v_bs, float* out, int64_t o_bs) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63, req = blockIdx.y;
  if (r >= rows) return;
  const float* wr = w + (int64_t)r * cols;
  const float* vr = v + req * v_bs;
  float acc = 0.0f;
  for (int i = lane; i < cols; i += 64) acc += wr[i] * vr[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) out[req * o_bs + r] = acc + b[r];
}

// the AdaLN scale / shift projections of every prenet layer in one launch (blockIdx.z = job; each
// job is k_gemv's arithmetic on its own weights and output)
constexpr int kMaxGemvJobs = 32;
struct GemvJobs {
  const float* w[kMaxGemvJobs];
  const float* b[kMaxGemvJobs];
  float* out[kMaxGemvJobs];
};
__global__ __launch_bounds__(256) void k_gemv_jobs(GemvJobs jb, int rows, int cols, const float* v, int64_t v_bs,
                                                   int64_t o_bs) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63, req = blockIdx.y, job = blockIdx.z;
  if (r >= rows) return;
  const float* wr = jb.w[job] + (int64_t)r * cols;
  const float* vr = v + req * v_bs;
  float acc = 0.0f;
  for (int i = lane; i < cols; i += 64) acc += wr[i] * vr[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) jb.out[job][req * o_bs + r] = acc + jb.b[job][r];
}

// [optional depthwise conv k7 pad 3] -> LayerNorm (eps 1e-6) -> * scale + shift
// scale/shift: [n][P] (AdaLN, stride P) or [P] (plain LN affine, stride 0).
// Output: f32 y (nullable) and/or planes yh/yl (nullable).
__global__ __launch_bounds__(128) void k_dw_ln(const float* x, float* y, bf16_t* yh, bf16_t* yl, int Tmax,
                                               const int* ntok, int P, const float* dw_w, const float* dw_b,
                                               const float* scale, const float* shift, int64_t ss_bs) {
  constexpr int MAXV = 4;  // P <= 512
  __shared__ float s_red[2][2];
  const int t = blockIdx.x, req = blockIdx.y;
  const int T = ntok[req];
  if (t >= T) return;
  const float* X = x + (int64_t)req * Tmax * P;
  float v[MAXV];
  float sum = 0.0f;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    const int c = threadIdx.x + u * 128;
    v[u] = 0.0f;
    if (c < P) {
      if (dw_w) {
        float acc = 0.0f;
        for (int k = 0; k < 7; ++k) {
          const int p = t + k - 3;
          if (p >= 0 && p < T) acc += dw_w[c * 7 + k] * X[(int64_t)p * P + c];
        }
        v[u] = acc + dw_b[c];
      } else {
        v[u] = X[(int64_t)t * P + c];
      }
      sum += v[u];
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) s_red[0][wv] = sum;
  __syncthreads();
  const float mean = (s_red[0][0] + s_red[0][1]) / (float)P;
  float sq = 0.0f;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    const int c = threadIdx.x + u * 128;
    if (c < P) sq += (v[u] - mean) * (v[u] - mean);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
  if (lane == 0) s_red[1][wv] = sq;
  __syncthreads();
  const float inv = 1.0f / sqrtf((s_red[1][0] + s_red[1][1]) / (float)P + 1e-6f);
  const int64_t base = ((int64_t)req * Tmax + t) * P;
#pragma unroll
  for (int u = 0; u < MAXV; ++u) {
    const int c = threadIdx.x + u * 128;
    if (c < P) {
      const float o = (v[u] - mean) * inv * scale[req * ss_bs + c] + shift[req * ss_bs + c];
      if (y) y[base + c] = o;
      if (yh) split_store(yh, yl, base + c, o);
    }
  }
}

// final conv7 (C -> 1) over the snake-activated planes -> tanh. kOutT samples per workgroup of
// kOutT threads: the input window (kOutT + 6 rows) is staged once into LDS as f32 (hi + lo) with
// 16-byte global loads (8 channels per load and plane; C % 8 == 0) at row stride C + 1
// (conflict-free walks); each thread then walks its 7 x C window against the weights (scalar
// operands). 128 samples: 52 KB of LDS at 96 channels, three workgroups per CU (256 samples took
// 101 KB, one per CU, and the walks of one workgroup left the CU's memory path idle).
constexpr int kOutT = 128;
__global__ __launch_bounds__(kOutT) void k_conv_out(const bf16_t* xh, const bf16_t* xl, int64_t x_bs, int64_t x_cs,
                                                  int C, int tin_mul, const int* ntok, const float* w,
                                                  const float* b, float* pcm, int64_t p_bs) {
  extern __shared__ float s_x[];
  const int req = blockIdx.y, T = ntok[req] * tin_mul, t0 = blockIdx.x * kOutT;
  if (t0 >= T) return;
  const int LDX = C + 1, rows = kOutT + 6, c8n = C / 8;
  const int64_t xo = req * x_bs;
  // staged in batches of 8 pieces per thread: all 16 loads of a batch are requested before the
  // first conversion, so the window's memory latency is paid once per batch, not once per piece
  constexpr int kBatch = 8;
  const int total = rows * c8n;
  for (int i0 = threadIdx.x; i0 < total; i0 += kOutT * kBatch) {
    uint4 h[kBatch], l[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = i0 + kOutT * j;
      const int r = i / c8n, c8 = (i - r * c8n) * 8, p = t0 - 3 + r;
      h[j] = l[j] = make_uint4(0u, 0u, 0u, 0u);
      if (i < total && p >= 0 && p < T) {
        const int64_t o = x_cs ? xo + (c8 >> 5) * x_cs + (int64_t)p * 32 + (c8 & 31) : xo + (int64_t)p * C + c8;
        h[j] = *(const uint4*)(xh + o);
        l[j] = *(const uint4*)(xl + o);
      }
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int i = i0 + kOutT * j;
      if (i >= total) break;
      const int r = i / c8n, c8 = (i - r * c8n) * 8;
      float* dst = s_x + r * LDX + c8;
      const uint32_t hw[4] = {h[j].x, h[j].y, h[j].z, h[j].w}, lw[4] = {l[j].x, l[j].y, l[j].z, l[j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // zero words (rows outside the utterance) give +0
        dst[2 * e] = as_f32(hw[e] << 16) + as_f32(lw[e] << 16);
        dst[2 * e + 1] = as_f32(hw[e] & 0xFFFF0000u) + as_f32(lw[e] & 0xFFFF0000u);
      }
    }
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc = 0.0f;
  for (int k = 0; k < 7; ++k) {
    const float* xr = s_x + (threadIdx.x + k) * LDX;
    const float* wr = w + k * C;
    for (int c = 0; c < C; ++c) acc += wr[c] * xr[c];
  }
  pcm[req * p_bs + t] = tanhf(acc + b[0]);
}

// f32 weights -> bf16 hi + lo planes (w = hi + lo to ~2^-16 relative; lo = 0 for bf16-exact w)
__global__ void k_f32_split_bf16(const float* in, bf16_t* hi, bf16_t* lo, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t h = f32_to_bf16(in[i]);
    hi[i] = h;
    if (lo) lo[i] = f32_to_bf16(in[i] - bf16_to_f32(h));
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct Planes {  // activated activations as bf16 hi + lo (x = hi + lo)
  bf16_t* h = nullptr;
  bf16_t* l = nullptr;
  int64_t cs = 0;  // channel-blocked layout's chunk stride (ConvArgs::x_cs); 0: channel-last
};

class Codec {
 public:
  rwkvtts_codec_dims d{};
  int device = 0;
  hipStream_t stream = nullptr;
  float* wf = nullptr;   // f32 blob on device
  bf16_t* zeros = nullptr;
  bf16_t* wb = nullptr;  // bf16 mirror (same element offsets) for MFMA operands: hi part
  bf16_t* wlb = nullptr; // lo part (f32 - hi), read by the WLO conv kernels
  bool wlo = false;      // some conv weight is not bf16-exact: three MFMAs per product
  uint32_t forms = 0;    // RWKVTTS_CODEC_FORM_* of later decode calls (rwkvtts_codec_set_forms)
  int cap_n = 0, cap_T = 0;
  int *d_tok = nullptr, *d_glob = nullptr, *d_ntok = nullptr;
  // prenet: x f32 residual stream [n][T][P]; zp/up/hp planes [n][T][L|P|I]
  float *xb = nullptr, *hs = nullptr, *dvec = nullptr, *cond = nullptr, *pcm = nullptr;
  Planes zp, up, hp;
  // WaveGenerator: xf f32 residual stream and two planes buffers, big_per_tok elements per frame
  float* xf = nullptr;
  Planes pp[2];
  int64_t big_per_tok = 0;
  std::vector<void*> bufs;
  // profiling (HIP events around each launch class)
  bool profiling = false;
  std::vector<std::pair<std::string, std::pair<int64_t, double>>> prof;

  ~Codec() {
    release();
    if (wf) (void)hipFree(wf);
    if (wb) (void)hipFree(wb);
    if (wlb) (void)hipFree(wlb);
    if (zeros) (void)hipFree(zeros);
    if (stream) (void)hipStreamDestroy(stream);
  }
  void release() {
    for (void* p : bufs) (void)hipFree(p);
    bufs.clear();
    cap_n = cap_T = 0;
  }
  template <typename T>
  int dalloc(T** p, int64_t count) {
    RT_HIP(hipMalloc((void**)p, count * sizeof(T)));
    bufs.push_back(*p);
    return RWKVTTS_OK;
  }
  int palloc(Planes* p, int64_t count) {
    int rc = dalloc(&p->h, 2 * count);
    p->l = p->h + count;
    return rc;
  }
  const float* F(int g, int i, int t) const { return wf + rwkvtts_codec_offset(&d, g, i, t); }
  const bf16_t* B(int g, int i, int t) const { return wb + rwkvtts_codec_offset(&d, g, i, t); }

  int init(int dev, const rwkvtts_codec_dims& dims, const float* host_w, int weight_path) {
    d = dims;
    device = dev;
    RT_CHECK(d.n_up >= 1 && d.n_up <= 4 && d.latent_dim == d.spk_dim && d.prenet_dim <= 512 &&
                 d.fsq_dims <= 16 && d.codebook_dim <= 64 && d.fsq_levels >= 2,
             RWKVTTS_EINVAL, "codec: unsupported dims");
    RT_CHECK(d.latent_dim % 64 == 0 && d.prenet_dim % 64 == 0 && d.prenet_inter % 64 == 0 &&
                 (d.dec_channels >> d.n_up) % 32 == 0 && (d.dec_channels >> d.n_up) <= 112,
             RWKVTTS_EINVAL, "codec: channel counts must be multiples of 64 (last stage: of 32, <= 112)");
    for (int i = 0; i < d.n_up; ++i)
      RT_CHECK(d.up_rates[i] >= 1 && d.up_kernels[i] >= d.up_rates[i] && ((d.up_kernels[i] - d.up_rates[i]) % 2) == 0 &&
                   (d.up_kernels[i] + d.up_rates[i] - 1) / d.up_rates[i] <= 8,
               RWKVTTS_EINVAL, "codec: ConvTranspose needs k >= s, even k - s and <= 8 taps per phase");
    RT_HIP(hipSetDevice(device));
    {  // lowest queue priority: the LM decode chain (engine.hip) goes first when both share the GPU
      int least = 0, greatest = 0;
      RT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
      // (a CU-masked stream confining the vocoder to 32 / 128 CUs measured no gain beside the
      // decode)
      RT_HIP(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, least));
    }
#define RT_CONV_ATTR(TN_, KT_, WLO_, NWV_) \
    RT_HIP(hipFuncSetAttribute((const void*)k_conv<TN_, KT_, WLO_, NWV_>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RT_CONV_KERNELS(RT_CONV_ATTR)
#undef RT_CONV_ATTR
#define RT_CONV_ATTR_F(TN_, KT_, WLO_, NWV_) \
    RT_HIP(hipFuncSetAttribute((const void*)k_conv<TN_, KT_, WLO_, NWV_, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    RT_CONV_FUSED(RT_CONV_ATTR_F)
#undef RT_CONV_ATTR_F
    RT_HIP(hipFuncSetAttribute((const void*)k_conv_out, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    // zero page: out-of-range window rows read zeros at channel offsets up to the largest Ci
    RT_HIP(hipMalloc(&zeros, 16384));
    RT_HIP(hipMemset(zeros, 0, 16384));
    const int64_t n = rwkvtts_codec_offset(&d, -1, 0, 0);
    RT_HIP(hipMalloc(&wf, n * sizeof(float)));
    RT_HIP(hipMalloc(&wb, n * sizeof(bf16_t)));
    // the MFMA convs take the three-product path when any of their weights is not bf16-exact
    // (weight_path RWKVTTS_CODEC_WEIGHTS_BF16 / _HILO forces the choice); the lo plane exists only then
    RT_CHECK(weight_path >= RWKVTTS_CODEC_WEIGHTS_AUTO && weight_path <= RWKVTTS_CODEC_WEIGHTS_HILO, RWKVTTS_EINVAL,
             "codec: unknown weight_path");
    wlo = weight_path == RWKVTTS_CODEC_WEIGHTS_AUTO ? !conv_weights_bf16_exact(host_w)
                                                    : weight_path == RWKVTTS_CODEC_WEIGHTS_HILO;
    if (wlo) RT_HIP(hipMalloc(&wlb, n * sizeof(bf16_t)));
    RT_HIP(hipMemcpy(wf, host_w, n * sizeof(float), hipMemcpyHostToDevice));
    k_f32_split_bf16<<<2048, 256, 0, stream>>>(wf, wb, wlb, n);
    RT_HIP(hipGetLastError());
    RT_HIP(hipStreamSynchronize(stream));
    // largest per-frame activation of the WaveGenerator (conv_in or any up stage)
    big_per_tok = (int64_t)d.dec_channels;
    int64_t mul = 1;
    for (int i = 0; i < d.n_up; ++i) {
      mul *= d.up_rates[i];
      big_per_tok = std::max(big_per_tok, mul * (int64_t)(d.dec_channels >> (i + 1)));
    }
    return RWKVTTS_OK;
  }

  int ensure(int n, int T) {
    if (n <= cap_n && T <= cap_T) return RWKVTTS_OK;
    release();
    const int64_t nt = (int64_t)n * T;
    const int Q = RWKVTTS_CODEC_SPK_LATENT;
    int rc = 0;
    rc |= dalloc(&d_tok, nt);
    rc |= dalloc(&d_glob, (int64_t)n * d.n_global);
    rc |= dalloc(&d_ntok, n);
    rc |= dalloc(&xb, nt * d.prenet_dim);
    rc |= palloc(&zp, nt * d.latent_dim);
    rc |= palloc(&up, nt * d.prenet_dim);
    rc |= palloc(&hp, nt * d.prenet_inter);
    rc |= dalloc(&hs, (int64_t)n * Q * d.n_global);
    rc |= dalloc(&dvec, (int64_t)n * d.spk_dim);
    rc |= dalloc(&cond, (int64_t)n * 2 * (d.prenet_layers + 1) * d.prenet_dim);
    rc |= dalloc(&xf, nt * big_per_tok);
    rc |= palloc(&pp[0], nt * big_per_tok);
    rc |= palloc(&pp[1], nt * big_per_tok);
    rc |= dalloc(&pcm, nt * RWKVTTS_HOP);
    if (rc) return RWKVTTS_EHIP;
    cap_n = n;
    cap_T = T;
    return RWKVTTS_OK;
  }

  // every tensor the MFMA conv kernel reads as weights
  bool conv_weights_bf16_exact(const float* w) const {
    std::vector<std::pair<int64_t, int64_t>> ts;  // (offset, count)
    auto add = [&](int g, int i, int t) {
      ts.push_back({rwkvtts_codec_offset(&d, g, i, t), rwkvtts_codec_numel(&d, g, i, t)});
    };
    for (int t : {CD_PRE_W, CD_EMB_W, CD_LIN_W, CD_CIN_W}) add(0, 0, t);
    for (int l = 0; l < d.prenet_layers; ++l)
      for (int t : {CB_PW1_W, CB_PW2_W}) add(1, l, t);
    for (int ub = 0; ub < d.n_up; ++ub)
      for (int t : {CU_T_W, CU_R0_W7, CU_R0_W1, CU_R1_W7, CU_R1_W1, CU_R2_W7, CU_R2_W1}) add(2, ub, t);
    for (auto& tc : ts)
      for (int64_t i = 0; i < tc.second; ++i) {
        const float x = w[tc.first + i];
        if (bf16_to_f32(f32_to_bf16(x)) != x) return false;
      }
    return true;
  }

  hipEvent_t ev0 = nullptr;
  void pbeg() {
    if (!profiling) return;
    (void)hipEventCreate(&ev0);
    (void)hipEventRecord(ev0, stream);
  }
  void pend(const char* name) {
    if (!profiling) return;
    hipEvent_t e1;
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e1, stream);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ev0, e1);
    (void)hipEventDestroy(ev0);
    (void)hipEventDestroy(e1);
    for (auto& p : prof)
      if (p.first == name) {
        p.second.first++;
        p.second.second += ms;
        return;
      }
    prof.push_back({name, {1, (double)ms}});
  }

  // One implicit-GEMM conv launch. Output: f32 y and/or planes (snake(y_alpha) applied).
  struct ConvOut {
    float* y = nullptr;
    Planes p{};
    const float* alpha = nullptr;
    const float* res = nullptr;
    const float* gamma = nullptr;
    const float* rbias = nullptr;
    int64_t rb_bs = 0;
    int act = 0;
    int64_t y_bs = -1;  // per-utterance stride of y / planes / res (-1: same as the input's)
  };
  std::string stage_name(const char* base, int C) { return profiling ? std::string(base) + "@" + std::to_string(C) : std::string(); }
  int conv(int n, int Tmax, const std::string& name, Planes x, int64_t bs, int Ci, int tin_mul, const bf16_t* w,
           int K, int Co, int mode, int dil, int pad, int s, const float* bias, const ConvOut& o) {
    RT_CHECK(Ci % 32 == 0 && Co % 32 == 0, RWKVTTS_EINVAL, "codec conv: channels must be multiples of 32");
    // column tile: 64, or for the last stage's 96 channels 96 (pointwise) / 48 (taps): 32-wide
    // tiles read two LDS fragments per four MFMAs
    int TN = (Co % 64 == 0) ? 64 : ((Co % 96 == 0 && K == 1) ? 96 : (Co % 48 == 0 ? 48 : 32));
    // pointwise (memory-bound) convs: 96-wide column tiles read the input window fewer times
    // (conv1 @ 192 / 384 / 768: 6.9 / 4.1 / 2.2 -> 5.3 / 3.5 / 2.0 ms per batch with the XCD-aware
    // order below; 192-wide tiles halve the occupancy and are slower)
    if (K == 1 && Co % 96 == 0) TN = 96;
    const int ntaps_max = mode == 1 ? (K + s - 1) / s : K;
    const int span = (ntaps_max - 1) * (mode == 1 ? 1 : dil);
    const int KT = ntaps_max <= 1 ? 1 : (ntaps_max <= 3 ? 3 : 7);
    {  // 7-tap convs: 64-wide column tiles by default. 96-wide ones (where the double-buffered
       // chunk fits: RWKVTTS_CONV7_TN=96) make the vocoder alone faster (residual conv7 33.4 ->
       // 31.1 ms per batch) but their 155 KB of LDS leaves no room on the CU for a decode GEMM
       // workgroup (34 KB): beside the next batch's token generator -- the serving shape, the
       // bench -- every GEMM launch then waits for whole vocoder workgroups to retire. 64-wide
       // tiles (124 KB) let them share the CU: decode step 0.883 -> 0.875 ms in the bench, +0.7 %
       // samples/s (same-box A/B x2, tools/bench_ab.sh) for +1 ms of vocoder time. Tests
       // bit-identical either way: the per-element accumulation order does not depend on TN.
      // Round 4: the decode step's persistent workgroups (k_att_persist / k_ffn_persist) take
      // 36.6 KB of LDS, which fits beside a 64-wide tile at dilation 1 only. 48-wide tiles leave
      // room at every dilation: bench A/Bs (13 alternating pairs over three boxes,
      // profiles/r04_conv7_tile_ab.txt) +0.1 to +1.2 % samples/s, within the boxes' run-to-run
      // spread, for +1.5 ms of vocoder time; 64 stays.
      // ConvTranspose: 96-wide tiles measured faster at 96 and 384 output channels (2.54 -> 2.14,
      // 2.30 -> 2.10 ms per batch), slower at 192 (2.51 -> 2.62), equal at 768
      if (mode == 1 && KT == 3 && (Co == 96 || Co == 384)) TN = 96;
      // (Round 6: capping every conv launch's workgroups per CU, by padding its LDS request, so that a
      // persistent decode workgroup always fits beside them -- with the pointwise convs in 64-wide
      // tiles, the ConvTranspose ones too, the 7-tap ones in 48-wide tiles -- left the decode step
      // beside the vocoder unchanged, 0.806-0.816 ms, and the vocoder alone 3-10 ms slower:
      // profiles/r06e_coresidency_ab.txt, tools/experiments/r06_codec_coresidency.patch)
    }
    int nwv = conv_waves(KT);
    const int wplanes = wlo ? 2 : 1;  // weight planes staged per chunk
    auto chunk_rows = [&](int tn, int nw) { return 2 * ((32 * nw + span + 15) & ~15) + wplanes * ntaps_max * tn; };
    auto shm_of = [&](int tn, int nw) {
      return std::max(2 * (size_t)chunk_rows(tn, nw) * 64, (size_t)nw * 32 * (tn + 4) * sizeof(float));
    };
    auto fits = [&](int tn, int nw) {
      return Co % tn == 0 && shm_of(tn, nw) <= 160 * 1024 && chunk_rows(tn, nw) / 16 <= 16 * nw;
    };
    if (wlo && (!fits(TN, nwv) || TN > 96)) {  // (no weight-lo kernel wider than 96 columns)
      // the weight lo plane doubles the staged weights: the (tile width, waves) that fits and
      // stages the fewest LDS rows per output element
      int bt = 0, bw = 0;
      double best = 0.0;
      for (int nw : {conv_waves(KT), 4})
        for (int tn : {96, 64, 48, 32}) {
          if (!fits(tn, nw) || (nw != conv_waves(KT) && KT != 7)) continue;
          const double sc = (double)(32 * nw * tn) / chunk_rows(tn, nw);
          if (sc > best) { best = sc; bt = tn; bw = nw; }
        }
      RT_CHECK(bt > 0, RWKVTTS_EINVAL, "codec conv: no tile fits the LDS with weight lo planes");
      TN = bt;
      nwv = bw;
    }
    const int TM = 32 * nwv;
    const size_t shm = shm_of(TN, nwv);
    RT_CHECK(fits(TN, nwv) && ntaps_max <= 7 && Ci <= 4096, RWKVTTS_EINVAL, "codec conv: tile window too large");
    ConvArgs a{};
    a.xh = x.h; a.xl = x.l; a.x_bs = bs; a.Ci = Ci; a.tin_mul = tin_mul; a.w = w; a.wl = wlb ? wlb + (w - wb) : nullptr; a.K = K; a.Co = Co;
    a.mode = mode; a.dil = dil; a.pad = pad; a.s = s; a.bias = bias; a.rbias = o.rbias; a.rb_bs = o.rb_bs;
    a.gamma = o.gamma; a.res = o.res; a.act = o.act; a.y = o.y; a.yh = o.p.h; a.yl = o.p.l;
    a.y_alpha = o.alpha; a.y_bs = o.y_bs >= 0 ? o.y_bs : bs; a.ntok = d_ntok; a.zeros = zeros;
    a.x_cs = x.cs; a.y_cs = o.p.cs;
    const int phases = mode == 1 ? s : 1;
    dim3 grid((unsigned)((Tmax * (int64_t)tin_mul + TM - 1) / TM), (unsigned)(phases * (Co / TN)), (unsigned)n);
    // XCD-aware order for the long-time-axis residual convs (conv7 and conv1 at >= 32 time tiles:
    // a time tile's column tiles share one L2); the short prenet / conv_in / convT launches keep
    // the default order (2x slower remapped)
    // (the ConvTranspose launches in this order too: 1-8 % slower, the Infinity Cache serves their
    // re-reads)
    a.xmap = 0;
    if (grid.y > 1 && grid.x >= 32 && mode == 0 && (K == 7 || K == 1)) {
      a.xmap = 1;
      a.gx = (int)grid.x;
      a.gy = (int)grid.y;
      grid = dim3((unsigned)(8 * ((grid.x + 7) / 8) * grid.y), 1, (unsigned)n);
    }
    pbeg();
    const int nthr = 64 * nwv;
    bool launched = false;
#define RT_CONV_LAUNCH(TN_, KT_, WLO_, NWV_)                                          \
    if (!launched && TN == TN_ && KT == KT_ && wlo == WLO_ && nwv == NWV_) {          \
      k_conv<TN_, KT_, WLO_, NWV_><<<grid, nthr, shm, stream>>>(a);                   \
      launched = true;                                                                \
    }
    RT_CONV_KERNELS(RT_CONV_LAUNCH)
#undef RT_CONV_LAUNCH
    RT_CHECK(launched, RWKVTTS_EINVAL, "codec conv: no kernel for this tile shape");
    RT_HIP(hipGetLastError());
    pend(name.c_str());
    return RWKVTTS_OK;
  }

  // One residual unit (conv7 -> Snake -> conv1 -> + residual) as ONE launch when it fits: 96
  // channels (one column tile covers every channel the pointwise conv needs), bf16-exact weights
  // (the weight lo plane would not fit beside the 7-tap chunk). Returns 1 if launched, 0 if the
  // caller must run the two convs.
  int resunit_fused(int n, int Tmax, const std::string& name, Planes x, int64_t bs, int C, int tin_mul,
                    const bf16_t* w7, const float* b7, int dil, const float* mid_alpha, const bf16_t* w1,
                    const float* b1, const ConvOut& o, bool* done) {
    *done = false;
    if ((forms & RWKVTTS_CODEC_FORM_SEPARATE_RESUNIT) || wlo || C != 96) return RWKVTTS_OK;
    const int span = 6 * dil;
    int nwv = 0;
    for (int nw : {8, 4}) {  // (4-wave units where 8 do not fit: 8 measured faster)
      const int wr = (32 * nw + span + 15) & ~15;
      const size_t chunk = 2 * (size_t)(2 * wr + 7 * 96) * 64;
      const size_t fused = (size_t)3 * 2 * 32 * nw * 64 + 3 * 96 * 64;
      const size_t epi = (size_t)nw * 32 * 100 * sizeof(float);
      if (std::max(std::max(chunk, fused), epi) <= 160 * 1024 && (2 * wr + 7 * 96) / 16 <= conv_maxb(nw, true) * nw) {
        nwv = nw;
        break;
      }
    }
    if (!nwv) return RWKVTTS_OK;
    const int TM = 32 * nwv, wr = (TM + span + 15) & ~15;
    const size_t shm = std::max(std::max(2 * (size_t)(2 * wr + 7 * 96) * 64, (size_t)3 * 2 * TM * 64 + 3 * 96 * 64),
                                (size_t)nwv * 32 * 100 * sizeof(float));
    ConvArgs a{};
    a.xh = x.h; a.xl = x.l; a.x_bs = bs; a.Ci = C; a.tin_mul = tin_mul; a.w = w7; a.wl = wlb ? wlb + (w7 - wb) : nullptr; a.K = 7; a.Co = C;
    a.mode = 0; a.dil = dil; a.pad = 3 * dil; a.s = 1; a.bias = b7; a.rbias = nullptr; a.rb_bs = 0;
    a.gamma = nullptr; a.res = o.res; a.act = 0; a.y = o.y; a.yh = o.p.h; a.yl = o.p.l;
    a.y_alpha = o.alpha; a.y_bs = o.y_bs >= 0 ? o.y_bs : bs; a.ntok = d_ntok; a.zeros = zeros;
    a.mid_alpha = mid_alpha; a.w1 = w1; a.bias1 = b1;
    a.x_cs = x.cs; a.y_cs = o.p.cs;
    a.xmap = 0;
    dim3 grid((unsigned)((Tmax * (int64_t)tin_mul + TM - 1) / TM), 1, (unsigned)n);
    pbeg();
    if (nwv == 8) k_conv<96, 7, false, 8, true><<<grid, 512, shm, stream>>>(a);
    else k_conv<96, 7, false, 4, true><<<grid, 256, shm, stream>>>(a);
    RT_HIP(hipGetLastError());
    pend(name.c_str());
    *done = true;
    return RWKVTTS_OK;
  }

  // Decode n utterances; semantic[i] has T[i] codes, global[i] n_global codes; pcm[i] gets T[i]*320.
  int decode(const int64_t* const* semantic, const int* T, const int64_t* const* global, int n,
             float* const* out) {
    RT_CHECK(n > 0, RWKVTTS_EINVAL, "codec decode: n must be > 0");
    int Tmax = 0;
    for (int i = 0; i < n; ++i) {
      RT_CHECK(semantic[i] && global[i] && out[i] && T[i] > 0, RWKVTTS_EINVAL, "codec decode: bad utterance");
      Tmax = std::max(Tmax, T[i]);
    }
    int n_codes = 1;
    for (int i = 0; i < d.fsq_dims; ++i) n_codes *= d.fsq_levels;
    std::vector<int> tok((size_t)n * Tmax, 0), glob((size_t)n * d.n_global), ntok(T, T + n);
    for (int i = 0; i < n; ++i) {
      for (int t = 0; t < T[i]; ++t) {
        RT_CHECK(semantic[i][t] >= 0 && semantic[i][t] < d.codebook_size, RWKVTTS_EINVAL,
                 "codec decode: semantic code out of range");
        tok[(size_t)i * Tmax + t] = (int)semantic[i][t];
      }
      for (int t = 0; t < d.n_global; ++t) {
        RT_CHECK(global[i][t] >= 0 && global[i][t] < n_codes, RWKVTTS_EINVAL,
                 "codec decode: global code out of range");
        glob[(size_t)i * d.n_global + t] = (int)global[i][t];
      }
    }
    RT_HIP(hipSetDevice(device));
    int rc = ensure(n, Tmax);
    if (rc) return rc;
    RT_HIP(hipMemcpyAsync(d_tok, tok.data(), tok.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    RT_HIP(hipMemcpyAsync(d_glob, glob.data(), glob.size() * sizeof(int), hipMemcpyHostToDevice, stream));
    RT_HIP(hipMemcpyAsync(d_ntok, ntok.data(), n * sizeof(int), hipMemcpyHostToDevice, stream));
    rc = forward(n, Tmax);
    if (rc) return rc;
    for (int i = 0; i < n; ++i)
      RT_HIP(hipMemcpyAsync(out[i], pcm + (int64_t)i * Tmax * RWKVTTS_HOP, (size_t)T[i] * RWKVTTS_HOP * sizeof(float),
                            hipMemcpyDeviceToHost, stream));
    RT_HIP(hipStreamSynchronize(stream));
    return RWKVTTS_OK;
  }

  int forward(int n, int Tmax) {
    const int L = d.latent_dim, P = d.prenet_dim, I = d.prenet_inter, S = d.spk_dim, G = d.n_global;
    const int Q = RWKVTTS_CODEC_SPK_LATENT;
    const int64_t tL = (int64_t)Tmax * L, tP = (int64_t)Tmax * P, tI = (int64_t)Tmax * I;
    const int64_t cstr = 2 * (int64_t)(d.prenet_layers + 1) * P;  // cond stride per utterance
    int rc;
    // speaker d-vector and every AdaLN scale/shift (cond[req][2 * (layer + 1) + {0, 1}][P])
    pbeg();
    k_fsq<<<n, 256, 0, stream>>>(d_glob, G, d.fsq_levels, d.fsq_dims, F(0, 0, CD_FSQ_W), F(0, 0, CD_FSQ_B), Q, hs);
    k_gemv<<<dim3((S + 3) / 4, n), 256, 0, stream>>>(F(0, 0, CD_SPK_W), F(0, 0, CD_SPK_B), S, Q * G, hs,
                                                     (int64_t)Q * G, dvec, S);
    {
      GemvJobs jb{};
      int nj = 0;
      auto flush = [&]() {
        if (nj) k_gemv_jobs<<<dim3((P + 3) / 4, n, nj), 256, 0, stream>>>(jb, P, S, dvec, S, cstr);
        nj = 0;
      };
      for (int l = -1; l < d.prenet_layers; ++l) {
        if (nj + 2 > kMaxGemvJobs) flush();
        jb.w[nj] = l < 0 ? F(0, 0, CD_N0_SW) : F(1, l, CB_SW);
        jb.b[nj] = l < 0 ? F(0, 0, CD_N0_SB) : F(1, l, CB_SB);
        jb.out[nj++] = cond + 2 * (l + 1) * P;
        jb.w[nj] = l < 0 ? F(0, 0, CD_N0_HW) : F(1, l, CB_HW);
        jb.b[nj] = l < 0 ? F(0, 0, CD_N0_HB) : F(1, l, CB_HB);
        jb.out[nj++] = cond + (2 * (l + 1) + 1) * P;
      }
      flush();
    }
    k_fvq<<<dim3(Tmax, n), 256, 0, stream>>>(d_tok, Tmax, d_ntok, F(0, 0, CD_CODEBOOK), d.codebook_dim,
                                            F(0, 0, CD_OUTP_W), F(0, 0, CD_OUTP_B), L, zp.h, zp.l);
    RT_HIP(hipGetLastError());
    pend("codec_cond");
    // prenet: linear_pre -> embed conv7 -> AdaLN0 -> ConvNeXt blocks -> LN -> linear (+ d)
    {
      ConvOut o;
      o.p = up;
      o.y_bs = tP;
      if ((rc = conv(n, Tmax, "codec_prenet_gemm", zp, tL, L, 1, B(0, 0, CD_PRE_W), 1, P, 0, 1, 0, 1,
                     F(0, 0, CD_PRE_B), o))) return rc;
      ConvOut e;
      e.y = xb;
      if ((rc = conv(n, Tmax, "codec_prenet_gemm", up, tP, P, 1, B(0, 0, CD_EMB_W), 7, P, 0, 1, 3, 1,
                     F(0, 0, CD_EMB_B), e))) return rc;
    }
    pbeg();
    k_dw_ln<<<dim3(Tmax, n), 128, 0, stream>>>(xb, xb, nullptr, nullptr, Tmax, d_ntok, P, nullptr, nullptr, cond,
                                               cond + P, cstr);
    RT_HIP(hipGetLastError());
    pend("codec_ln");
    for (int l = 0; l < d.prenet_layers; ++l) {
      pbeg();
      k_dw_ln<<<dim3(Tmax, n), 128, 0, stream>>>(xb, nullptr, up.h, up.l, Tmax, d_ntok, P, F(1, l, CB_DW_W),
                                                 F(1, l, CB_DW_B), cond + 2 * (l + 1) * P,
                                                 cond + (2 * (l + 1) + 1) * P, cstr);
      RT_HIP(hipGetLastError());
      pend("codec_ln");
      ConvOut o1;
      o1.p = hp;
      o1.act = 1;
      o1.y_bs = tI;
      if ((rc = conv(n, Tmax, "codec_prenet_gemm", up, tP, P, 1, B(1, l, CB_PW1_W), 1, I, 0, 1, 0, 1,
                     F(1, l, CB_PW1_B), o1))) return rc;
      ConvOut o2;
      o2.y = xb;
      o2.res = xb;
      o2.gamma = F(1, l, CB_GAMMA);
      o2.y_bs = tP;
      if ((rc = conv(n, Tmax, "codec_prenet_gemm", hp, tI, I, 1, B(1, l, CB_PW2_W), 1, P, 0, 1, 0, 1,
                     F(1, l, CB_PW2_B), o2))) return rc;
    }
    pbeg();
    k_dw_ln<<<dim3(Tmax, n), 128, 0, stream>>>(xb, nullptr, up.h, up.l, Tmax, d_ntok, P, nullptr, nullptr,
                                               F(0, 0, CD_FLN_W), F(0, 0, CD_FLN_B), 0);
    RT_HIP(hipGetLastError());
    pend("codec_ln");
    {
      ConvOut o;
      o.p = zp;
      o.rbias = dvec;
      o.rb_bs = S;
      o.y_bs = tL;
      if ((rc = conv(n, Tmax, "codec_prenet_gemm", up, tP, P, 1, B(0, 0, CD_LIN_W), 1, L, 0, 1, 0, 1,
                     F(0, 0, CD_LIN_B), o))) return rc;
    }
    // WaveGenerator: conv_in -> [snake -> convT -> 3 x residual unit] x n_up -> snake -> conv_out
    // Its planes are channel-blocked ([C / 32][Tmax * mul][32] per utterance) unless
    // RWKVTTS_CODEC_FORM_CHANNEL_LAST (the arithmetic is the same either way)
    const int64_t bs = (int64_t)Tmax * big_per_tok;
    const bool blk = !(forms & RWKVTTS_CODEC_FORM_CHANNEL_LAST);
    auto PB = [&](int i, int m) {  // pp[i] holding a tensor of Tmax * m rows
      Planes q = pp[i];
      q.cs = blk ? (int64_t)Tmax * m * 32 : 0;
      return q;
    };
    int C = d.dec_channels, mul = 1, cur = 0;
    {
      ConvOut o;
      o.p = PB(cur, 1);
      o.alpha = F(2, 0, CU_SNAKE);
      // conv_in reads the prenet planes with the prenet's per-utterance stride
      o.y_bs = bs;
      if ((rc = conv(n, Tmax, "codec_conv_in", zp, tL, L, 1, B(0, 0, CD_CIN_W), 7, C, 0, 1, 3, 1,
                     F(0, 0, CD_CIN_B), o))) return rc;
    }
    static const int dils[3] = {1, 3, 9};
    for (int ub = 0; ub < d.n_up; ++ub) {
      const int Co = C / 2, s = d.up_rates[ub], K = d.up_kernels[ub];
      ConvOut ot;
      ot.y = xf;
      ot.p = PB(cur ^ 1, mul * s);
      ot.alpha = F(2, ub, CU_R0_A1);
      if ((rc = conv(n, Tmax, stage_name("codec_convT", Co), PB(cur, mul), bs, C, mul, B(2, ub, CU_T_W), K, Co, 1, 1, 0, s,
                     F(2, ub, CU_T_B), ot))) return rc;
      cur ^= 1;
      mul *= s;
      C = Co;
      for (int r = 0; r < 3; ++r) {
        const int o = r * (CU_R1_A1 - CU_R0_A1);
        {
          ConvOut of;
          of.y = r < 2 ? xf : nullptr;
          of.res = xf;
          of.p = PB(cur ^ 1, mul);
          of.alpha = r < 2 ? F(2, ub, CU_R0_A1 + o + (CU_R1_A1 - CU_R0_A1))
                           : (ub + 1 < d.n_up ? F(2, ub + 1, CU_SNAKE) : F(0, 0, CD_SOUT_A));
          bool done = false;
          if ((rc = resunit_fused(n, Tmax, stage_name("codec_resunit", C), PB(cur, mul), bs, C, mul, B(2, ub, CU_R0_W7 + o),
                                  F(2, ub, CU_R0_B7 + o), dils[r], F(2, ub, CU_R0_A2 + o), B(2, ub, CU_R0_W1 + o),
                                  F(2, ub, CU_R0_B1 + o), of, &done))) return rc;
          if (done) {
            cur ^= 1;
            continue;
          }
        }
        ConvOut o7;
        o7.p = PB(cur ^ 1, mul);
        o7.alpha = F(2, ub, CU_R0_A2 + o);
        if ((rc = conv(n, Tmax, stage_name("codec_res_conv7", C), PB(cur, mul), bs, C, mul, B(2, ub, CU_R0_W7 + o), 7, C, 0, dils[r],
                       3 * dils[r], 1, F(2, ub, CU_R0_B7 + o), o7))) return rc;
        cur ^= 1;
        ConvOut o1;
        // the f32 residual stream after a stage's last unit is never read (the next ConvTranspose
        // or conv_out reads the planes, and the ConvTranspose rewrites xf): planes only
        o1.y = r < 2 ? xf : nullptr;
        o1.res = xf;
        o1.p = PB(cur ^ 1, mul);
        o1.alpha = r < 2 ? F(2, ub, CU_R0_A1 + o + (CU_R1_A1 - CU_R0_A1))
                         : (ub + 1 < d.n_up ? F(2, ub + 1, CU_SNAKE) : F(0, 0, CD_SOUT_A));
        if ((rc = conv(n, Tmax, stage_name("codec_res_conv1", C), PB(cur, mul), bs, C, mul, B(2, ub, CU_R0_W1 + o), 1, C, 0, 1, 0, 1,
                       F(2, ub, CU_R0_B1 + o), o1))) return rc;
        cur ^= 1;
      }
    }
    pbeg();
    const size_t shm = (size_t)(kOutT + 6) * (C + 1) * sizeof(float);
    k_conv_out<<<dim3((unsigned)((Tmax * (int64_t)mul + kOutT - 1) / kOutT), n), kOutT, shm, stream>>>(
        pp[cur].h, pp[cur].l, bs, PB(cur, mul).cs, C, mul, d_ntok, F(0, 0, CD_COUT_W), F(0, 0, CD_COUT_B), pcm,
        (int64_t)Tmax * RWKVTTS_HOP);
    RT_HIP(hipGetLastError());
    pend("codec_conv_out");
    return RWKVTTS_OK;
  }

};

// ---- synthetic weights (counter-based, deterministic) -----------------------------------
static inline uint64_t cmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline double cnormal(uint64_t h) {
  const double s = (double)(h & 0xFFFF) + (double)((h >> 16) & 0xFFFF) + (double)((h >> 32) & 0xFFFF) +
                   (double)((h >> 48) & 0xFFFF);
  return (s / 65536.0 - 2.0) * 1.7320508075688772;
}
static inline double cuniform(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

// (scale kind, std) of each tensor; bf16 = used as an MFMA operand (stored bf16-exact)
static void codec_init_rule(const rwkvtts_codec_dims* d, int g, int idx, int t, int* kind, double* sd, int* bf16) {
  const double L = d->latent_dim, P = d->prenet_dim, I = d->prenet_inter, S = d->spk_dim;
  *kind = 0; *sd = 0.02; *bf16 = 0;  // kind 0: sd * normal, 1: 1 + sd * normal, 2: 0.5 + uniform, 3: const sd
  if (g == 0) {
    switch (t) {
      case CD_CODEBOOK: *sd = 1.0; break;
      case CD_OUTP_W: *sd = 1.0 / sqrt((double)d->codebook_dim); break;
      case CD_FSQ_W: *sd = 1.0 / sqrt((double)d->fsq_dims); break;
      case CD_SPK_W: *sd = 1.0 / sqrt((double)RWKVTTS_CODEC_SPK_LATENT * d->n_global); break;
      case CD_PRE_W: *sd = 1.0 / sqrt(L); *bf16 = 1; break;
      case CD_EMB_W: *sd = 1.0 / sqrt(7.0 * P); *bf16 = 1; break;
      case CD_N0_SW: case CD_N0_HW: *sd = 0.1 / sqrt(S); break;
      case CD_N0_SB: *kind = 1; break;
      case CD_FLN_W: *kind = 1; *sd = 0.05; break;
      case CD_LIN_W: *sd = 1.0 / sqrt(P); *bf16 = 1; break;
      case CD_CIN_W: *sd = 1.0 / sqrt(7.0 * L); *bf16 = 1; break;
      case CD_SOUT_A: *kind = 2; break;
      case CD_COUT_W: *sd = 0.2 / sqrt(7.0 * (d->dec_channels >> d->n_up)); break;
      default: break;
    }
    return;
  }
  if (g == 1) {
    switch (t) {
      case CB_DW_W: *sd = 1.0 / sqrt(7.0); break;
      case CB_SW: case CB_HW: *sd = 0.1 / sqrt(S); break;
      case CB_SB: *kind = 1; break;
      case CB_PW1_W: *sd = 1.0 / sqrt(P); *bf16 = 1; break;
      case CB_PW2_W: *sd = 1.0 / sqrt(I); *bf16 = 1; break;
      case CB_GAMMA: *kind = 3; *sd = 1.0 / d->prenet_layers; break;
      default: break;
    }
    return;
  }
  const double Ci = d->dec_channels >> idx, Co = d->dec_channels >> (idx + 1);
  switch (t) {
    case CU_SNAKE: case CU_R0_A1: case CU_R0_A2: case CU_R1_A1: case CU_R1_A2: case CU_R2_A1: case CU_R2_A2:
      *kind = 2; break;
    case CU_T_W: *sd = 1.0 / sqrt(Ci * d->up_kernels[idx] / d->up_rates[idx]); *bf16 = 1; break;
    case CU_R0_W7: case CU_R1_W7: case CU_R2_W7: *sd = 0.5 / sqrt(7.0 * Co); *bf16 = 1; break;
    case CU_R0_W1: case CU_R1_W1: case CU_R2_W1: *sd = 0.5 / sqrt(Co); *bf16 = 1; break;
    default: break;
  }
}

}  // namespace rwkvtts

using namespace rwkvtts;

struct rwkvtts_codec {
  Codec c;
};

extern "C" {

int64_t rwkvtts_codec_blob_bytes(const rwkvtts_codec_dims* d) {
  if (!d) return -1;
  return rwkvtts_codec_offset(d, -1, 0, 0) * (int64_t)sizeof(float);
}

int rwkvtts_codec_synth_weights(const rwkvtts_codec_dims* d, uint64_t seed, float* out) {
  RT_CHECK(d && out, RWKVTTS_EINVAL, "codec_synth_weights: null argument");
  const int64_t total = rwkvtts_codec_offset(d, -1, 0, 0);
  memset(out, 0, total * sizeof(float));
  memcpy(out, d, sizeof(*d));  // header: dims
  for (int g = 0; g < 3; ++g) {
    const int nidx = g == 0 ? 1 : (g == 1 ? d->prenet_layers : d->n_up);
    const int nt = g == 0 ? CD_GLOBAL_COUNT : (g == 1 ? CB_COUNT : CU_COUNT);
    for (int i = 0; i < nidx; ++i)
      for (int t = 0; t < nt; ++t) {
        int kind, bf;
        double sd;
        codec_init_rule(d, g, i, t, &kind, &sd, &bf);
        const uint64_t key = cmix(seed ^ (0xA0761D6478BD642Full * (uint64_t)((g * 64 + i) * 64 + t + 1)));
        float* p = out + rwkvtts_codec_offset(d, g, i, t);
        const int64_t n = rwkvtts_codec_numel(d, g, i, t);
        for (int64_t e = 0; e < n; ++e) {
          const uint64_t h = cmix(key ^ (uint64_t)e);
          double v = kind == 0 ? sd * cnormal(h) : kind == 1 ? 1.0 + sd * cnormal(h) : kind == 2 ? 0.5 + cuniform(h) : sd;
          float f = (float)v;
          if (bf) f = bf16_to_f32(f32_to_bf16(f));
          p[e] = f;
        }
      }
  }
  return RWKVTTS_OK;
}

int rwkvtts_codec_create(int device, const rwkvtts_codec_dims* d, const float* weights, rwkvtts_codec** out) {
  return rwkvtts_codec_create_ex(device, d, weights, RWKVTTS_CODEC_WEIGHTS_AUTO, out);
}

int rwkvtts_codec_create_ex(int device, const rwkvtts_codec_dims* d, const float* weights, int weight_path,
                            rwkvtts_codec** out) {
  RT_CHECK(d && weights && out, RWKVTTS_EINVAL, "codec_create: null argument");
  *out = nullptr;
  try {
    rwkvtts_codec* c = new rwkvtts_codec();
    const int rc = c->c.init(device, *d, weights, weight_path);
    if (rc != RWKVTTS_OK) {
      delete c;
      return rc;
    }
    *out = c;
    return RWKVTTS_OK;
  } catch (const std::exception& ex) {
    set_error(ex.what());
    return RWKVTTS_ENOMEM;
  }
}

int rwkvtts_codec_destroy(rwkvtts_codec* c) {
  delete c;
  return RWKVTTS_OK;
}

int rwkvtts_codec_decode(rwkvtts_codec* c, const int64_t* semantic, int T, const int64_t* global, float* pcm) {
  RT_CHECK(c && semantic && global && pcm && T > 0, RWKVTTS_EINVAL, "codec_decode: bad arguments");
  return c->c.decode(&semantic, &T, &global, 1, &pcm);
}

int rwkvtts_codec_decode_batch(rwkvtts_codec* c, const int64_t* const* semantic, const int* T,
                               const int64_t* const* global, int n, float* const* pcm) {
  RT_CHECK(c && semantic && T && global && pcm && n > 0, RWKVTTS_EINVAL, "codec_decode_batch: bad arguments");
  try {
    return c->c.decode(semantic, T, global, n, pcm);
  } catch (const std::exception& ex) {
    set_error(ex.what());
    return RWKVTTS_ENOMEM;
  }
}

int rwkvtts_codec_set_forms(rwkvtts_codec* c, uint32_t forms) {
  RT_CHECK(c, RWKVTTS_EINVAL, "codec_set_forms: null codec");
  RT_CHECK((forms & ~(RWKVTTS_CODEC_FORM_SEPARATE_RESUNIT | RWKVTTS_CODEC_FORM_CHANNEL_LAST)) == 0, RWKVTTS_EINVAL,
           "codec_set_forms: unknown forms bits");
  c->c.forms = forms;
  return RWKVTTS_OK;
}

int rwkvtts_codec_set_profiling(rwkvtts_codec* c, int on) {
  RT_CHECK(c, RWKVTTS_EINVAL, "null codec");
  c->c.profiling = on != 0;
  c->c.prof.clear();
  return RWKVTTS_OK;
}

int rwkvtts_codec_profile_entry(rwkvtts_codec* c, int idx, char* name, int name_cap, int64_t* launches,
                                double* total_ms) {
  RT_CHECK(c && idx >= 0 && idx < (int)c->c.prof.size(), RWKVTTS_EINVAL, "profile index out of range");
  const auto& p = c->c.prof[idx];
  if (name && name_cap > 0) {
    strncpy(name, p.first.c_str(), name_cap - 1);
    name[name_cap - 1] = 0;
  }
  if (launches) *launches = p.second.first;
  if (total_ms) *total_ms = p.second.second;
  return RWKVTTS_OK;
}

int rwkvtts_codec_profile_count(rwkvtts_codec* c) { return c ? (int)c->c.prof.size() : -1; }

}  // extern "C"
