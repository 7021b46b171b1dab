// sampler.hip -- exact device restatement of src/rwkv_sampler.rs:55-211
// (sample_logits_with_top_p_k) plus the on-device phase controller of
// src/normal_mode_inference.rs:222-391 and src/zero_shot_inference.rs:128-309.
//
// Bit-exactness with the reference's host sampler (Rust on Linux, glibc libm):
//  * exp: glibc 2.35 expf (ARM optimized-routines algorithm, x86_64 FMA variant) re-run in
//    double with explicit fma -- verified bit-identical against libm on every float in
//    [-104, 0] (tests/test_expf_exact.py), which covers every exp(l - max) the sampler takes;
//  * sums that the reference forms sequentially (softmax denominator, top-p cumulative in sorted
//    order, index-order sums, multinomial cumulative) are formed sequentially in the same order
//    by one lane; everything else (max, top-k threshold, masks, divisions, counts) is
//    order-independent and runs block-parallel;
//  * stable descending sort == sort on the key (p bits, ~index).
//  * rand 0.8 StdRng draw k == ChaCha12(key, block k/16)[k%16]; f32 = (u32 >> 8) * 2^-24.
// Rows up to kSampleMaxN run with the row in LDS; longer rows (the full 77,923-token vocabulary)
// run the same code with the row, sort keys and index list in a global scratch (k_sample_rows_wide),
// so every top-k / top-p combination of the reference is accepted. temperature != 1 uses a
// double-precision powf (not glibc's).
#include "sampler.h"
#include "exact_math.h"

namespace rwkvtts {

__device__ inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d)               \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

// word `index` of the ChaCha12 (djb layout, stream 0) keystream
__device__ uint32_t chacha12_word(const uint32_t* key, uint64_t index) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; ++i) in[4 + i] = key[i];
  const uint64_t ctr = index >> 4;
  in[12] = (uint32_t)ctr;
  in[13] = (uint32_t)(ctr >> 32);
  in[14] = 0;
  in[15] = 0;
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = in[i];
  for (int i = 0; i < 12; i += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  const int w = (int)(index & 15);
  uint32_t out = 0;
  for (int i = 0; i < 16; ++i)
    if (i == w) out = x[i] + in[i];
  return out;
}

// the whole ChaCha12 block `ctr` (words 16 ctr .. 16 ctr + 15 of the keystream)
__device__ void chacha12_block(const uint32_t* key, uint64_t ctr, uint32_t* out) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; ++i) in[4 + i] = key[i];
  in[12] = (uint32_t)ctr;
  in[13] = (uint32_t)(ctr >> 32);
  in[14] = 0;
  in[15] = 0;
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = in[i];
  for (int i = 0; i < 12; i += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

// rng.gen::<f32>() draw `index` through a per-stream block cache in the control block (one
// thread): a hit reads one word, a miss computes the block and stores it
__device__ float draw_cached(const uint32_t* key, uint64_t index, uint32_t* blk, uint64_t* blk_id) {
  const uint64_t b = index >> 4;
  uint32_t w;
  if (*blk_id == b + 1) {
    w = blk[index & 15];
  } else {
    uint32_t o[16];
    chacha12_block(key, b, o);
    for (int i = 0; i < 16; ++i) blk[i] = o[i];
    *blk_id = b + 1;
    w = blk[index & 15];
  }
  return (float)(w >> 8) * (1.0f / 16777216.0f);
}

__device__ inline float draw_f32(const uint32_t* key, uint64_t index) {
  return (float)(chacha12_word(key, index) >> 8) * (1.0f / 16777216.0f);
}

// Optional phase stamps (debug builds of a call only: pointer is null in production), in
// s_memrealtime ticks (100 MHz, one clock for every CU: the unit of the TL=1 launch timeline).
#define STAMP(k)                                                         \
  do {                                                                   \
    if (stamps && threadIdx.x == 0) stamps[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

__device__ inline float readlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ inline int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// wave-uniform sequential f32 sum of p[b..e) (all 64 lanes of the calling wave participate):
// 64 elements are staged into lanes per round and added in order from registers.
__device__ inline float add64(float s, float v) {  // s + v[lane 0] + ... + v[lane 63], in order
#pragma unroll
  for (int i = 0; i < 64; ++i) s += readlane_f(v, i);
  return s;
}
// Sequential adds of non-negative values: padding lanes hold +0.0, and s + 0 == s exactly.
__device__ inline float wave_serial_add(float s, const float* p, int b, int e) {
  const int lane = threadIdx.x & 63;
  for (int q = b; q < e; q += 64) s = add64(s, (q + lane < e) ? p[q + lane] : 0.0f);
  return s;
}
// Quantised increment of adding e (bits b) to an f32 s in binade E (ulp u = 2^(E-23); the
// denormal range counts as E = -126): RN(s + e) = s + u * (a + [frac(e/u) > 1/2]) while the
// result stays in the binade. Flags a tie (frac == 1/2: the result then depends on the parity of
// s) and an increment too large for the binade.
__device__ inline uint32_t qinc(uint32_t b, int E, bool& flag) {
  const uint32_t ef = (b >> 23) & 0xFFu;
  uint32_t M = b & 0x7FFFFFu;
  int ex;
  if (ef == 0) ex = -149;
  else { M |= 0x800000u; ex = (int)ef - 150; }
  if (M == 0) return 0u;
  const int sh = (E - 23) - ex;  // e / u = M * 2^-sh
  if (sh <= 0) {
    if (sh < -7) { flag = true; return 0u; }
    const uint32_t a = M << (-sh);
    if (a >= 0x1000000u) flag = true;
    return a;
  }
  if (sh > 25) return 0u;  // e < u / 4
  const uint32_t a = M >> sh, r = M & ((1u << sh) - 1u), half = 1u << (sh - 1);
  if (r == half) flag = true;
  return a + (r > half ? 1u : 0u);
}
// u * mm for mm < 2^24 in binade E (E = -126: denormal or the lowest normal binade, bits = mm)
__device__ inline float binade_value(uint32_t mm, int E) {
  return __builtin_bit_cast(float, E == -126 ? mm : (((uint32_t)(E + 127) << 23) | (mm & 0x7FFFFFu)));
}
// Exact sequential f32 sum s + p[b] + ... + p[e-1] (p >= 0) by one wave, 128 elements per
// round: every element's increment is quantised for s's binade and prefix-summed across the
// wave; the first element that would leave the binade, tie or overflow the binade is added
// with a real f32 add, and the round restarts after it. Bit-identical to the serial loop.
__device__ float wave_exact_add(float s, const float* p, int b, int e) {
  const int lane = threadIdx.x & 63;
  int pos = b;
  while (pos < e) {
    const uint32_t sb = __builtin_bit_cast(uint32_t, s);
    const int ef = (int)((sb >> 23) & 0xFFu);
    const int E = ef ? ef - 127 : -126;
    const uint32_t m = ef ? ((sb & 0x7FFFFFu) | 0x800000u) : (sb & 0x7FFFFFu);
    const int i0 = pos + 2 * lane, i1 = i0 + 1;
    bool f0 = false, f1 = false;
    const uint32_t q0 = i0 < e ? qinc(__builtin_bit_cast(uint32_t, p[i0]), E, f0) : 0u;
    const uint32_t q1 = i1 < e ? qinc(__builtin_bit_cast(uint32_t, p[i1]), E, f1) : 0u;
    const uint32_t lt = q0 + q1;
    uint32_t incl = lt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o);
      if (lane >= o) incl = min(incl + v, 0x4000000u);
    }
    uint32_t excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0u;
    const bool c0 = f0 || (i0 < e && m + excl + q0 >= 0x1000000u);
    const bool c1 = f1 || (i1 < e && m + excl + q0 + q1 >= 0x1000000u);
    const uint64_t bal = __ballot(c0 || c1);
    if (bal == 0) {
      s = binade_value(m + (uint32_t)readlane_i((int)incl, 63), E);
      pos += 128;
      continue;
    }
    const int fl = __ffsll((long long)bal) - 1;
    const bool c0l = readlane_i(c0 ? 1 : 0, fl) != 0;
    const uint32_t exl = (uint32_t)readlane_i((int)excl, fl);
    const uint32_t pre = c0l ? exl : exl + (uint32_t)readlane_i((int)q0, fl);
    const int f = pos + 2 * fl + (c0l ? 0 : 1);
    s = binade_value(m + pre, E);
    s = s + p[f];
    pos = f + 1;
  }
  return s;
}
// Sequential f32 sum s + p[b] + ... + p[e-1] by ONE lane from its own registers: each 128-
// element piece is pulled in with 32 back-to-back 16-byte LDS reads, then added in order -- one
// dependent v_add per element, no cross-lane traffic. b must be a multiple of 4.
template <int NE>
__device__ inline float addNE(float s, const float* p) {
  float4_ v[NE / 4];
#pragma unroll
  for (int q = 0; q < NE / 4; ++q) v[q] = *(const float4_*)(p + 4 * q);
#pragma unroll
  for (int q = 0; q < NE / 4; ++q) {
    s += v[q][0];
    s += v[q][1];
    s += v[q][2];
    s += v[q][3];
  }
  return s;
}
template <int NE>
__device__ inline float lane_serial_add(float s, const float* p, int b, int e) {
  for (; b + NE <= e; b += NE) s = addNE<NE>(s, p + b);
  for (; b + 4 <= e; b += 4) {
    const float4_ v = *(const float4_*)(p + b);
    s += v[0];
    s += v[1];
    s += v[2];
    s += v[3];
  }
  for (; b < e; ++b) s += p[b];
  return s;
}
// In-order prefix sums of one 64-block: lane i receives s + v[0] + ... + v[i] (sequential).
__device__ inline float prefix64(float s, float v, float* total) {
  // partly unrolled: fully unrolled, the 64 `lane == i` masks are loop invariants that the
  // compiler hoists to the kernel entry (k_advance's preamble) and spills
  float out = 0.0f;
  const int lane = threadIdx.x & 63;
#pragma unroll 8
  for (int i = 0; i < 64; ++i) {
    s += readlane_f(v, i);
    out = lane == i ? s : out;
  }
  *total = s;
  return out;
}

// Shared-memory layout of one sampling workgroup (NT threads, NW = NT / 64 waves).
// fred[0..NW) / ired[8..8+2 NW): block reductions; fred[16..22) / ired[0..8): named results.
struct SampleSmem {
  float* p;           // [n] logits -> e -> probabilities
  uint64_t* keys;     // [cap rounded up to a power of two] sort keys (p bits << 32 | ~index)
  int* list;          // [cap] positive indices in index order
  int* scan;          // [8] block-scan wave totals
  double* dscan;      // [8]
  uint32_t* sub_t;    // [NT][2] sub-chunk parity maps of the exact-sum emulation
  int* sub_e;         // [NT] binade each sub-chunk map was simulated for (kNoBinade: unusable)
  int* chunk_e;       // [64] predicted binade per chunk
  uint32_t* chunk_t;  // [64][2]
  int* chunk_ok;      // [64]
  int* runs;          // [4 * 128] binade runs of the exact-sum emulation: start, end, map
  uint64_t* etab;     // [32] glibc expf's 2^(i/32) table
  float* fred;        // [32]
  int* ired;          // [48]
  int cap;            // keys / list capacity (kSampleMaxSorted in LDS, the row length in scratch)
};

__device__ inline int wave_sum_i(int v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int NT>
__device__ inline float block_max(float v, float* fred) {
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = fred[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) m = fmaxf(m, fred[w]);
  return m;
}

// DPP row shift: lane l of each 16-lane row receives lane l - N of the same row, lanes with no
// source receive 0 (the update's old value)
template <int N>
__device__ inline int dpp_shr(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x110 + N, 0xF, 0xF, false);
}
template <int N>
__device__ inline double dpp_shr(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)dpp_shr<N>((int)(uint32_t)u), hi = (uint32_t)dpp_shr<N>((int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int N>
__device__ inline uint32_t dpp_shr(uint32_t v) {
  return (uint32_t)dpp_shr<N>((int)v);
}
__device__ inline double readlane_d(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// inclusive prefix sum over the wave's 64 lanes (DPP row shifts, then the row totals by readlane)
__device__ inline double wave_incl_scan_d(double x) {
  x += dpp_shr<1>(x);
  x += dpp_shr<2>(x);
  x += dpp_shr<4>(x);
  x += dpp_shr<8>(x);
  const double r0 = readlane_d(x, 15), r1 = readlane_d(x, 31), r2 = readlane_d(x, 47);
  const int row = (threadIdx.x & 63) >> 4;
  return x + (row == 0 ? 0.0 : (row == 1 ? r0 : (row == 2 ? r0 + r1 : (r0 + r1) + r2)));
}

__device__ inline uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
// rank_of(q) = #{j < m : key(j) > q} for every lane's q (wave-wide; lanes without a query pass
// any q). The m keys are read 64 at a time into lanes and broadcast by readlane: no LDS round trip
// per key (a per-key LDS broadcast loop is latency-bound: 13.8K cycles for the certified path's
// ranking at a few hundred candidates). Padding keys are 0, which exceeds no q.
template <typename KeyAt>
__device__ inline int wave_rank_gt(uint64_t q, int m, const KeyAt& key_at) {
  const int lane = threadIdx.x & 63;
  int rank = 0;
  for (int j0 = 0; j0 < m; j0 += 64) {
    const uint64_t kl = j0 + lane < m ? key_at(j0 + lane) : 0ull;
#pragma unroll
    for (int j = 0; j < 64; ++j) rank += readlane_u64(kl, j) > q ? 1 : 0;
  }
  return rank;
}
__device__ inline int readlane_t(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ inline uint32_t readlane_t(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ inline double readlane_t(double v, int l) { return readlane_d(v, l); }

// block-wide exclusive scans (NT threads): per wave an inclusive scan of each 16-lane row on DPP
// row shifts, row offsets from the row totals (readlane), then the NT/64 wave totals
template <int NT, typename T>
__device__ inline T block_excl_scan_t(T v, T* scratch, T* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
  x += dpp_shr<1>(x);
  x += dpp_shr<2>(x);
  x += dpp_shr<4>(x);
  x += dpp_shr<8>(x);
  {
    const T r0 = readlane_t(x, 15), r1 = readlane_t(x, 31), r2 = readlane_t(x, 47);
    const int row = lane >> 4;
    const T off = row == 0 ? (T)0 : (row == 1 ? r0 : (row == 2 ? r0 + r1 : (r0 + r1) + r2));
    x += off;
  }
  __syncthreads();
  if (lane == 63) scratch[w] = x;
  __syncthreads();
  T base = 0;
  for (int k = 0; k < w; ++k) base += scratch[k];
  T t = scratch[0];
#pragma unroll
  for (int k = 1; k < NT / 64; ++k) t += scratch[k];
  *tot = t;
  return base + x - v;
}
template <int NT>
__device__ inline int block_excl_scan(int v, int* scratch, int* tot) { return block_excl_scan_t<NT, int>(v, scratch, tot); }

// compact indices with p > 0 into list (index order); returns count (may exceed capacity:
// then list is incomplete and callers fall back to a scan of p).
// (the arrays are passed one by one: an out-of-line callee taking the SampleSmem by reference
// makes the caller keep the struct in scratch memory)
template <int NT>
__device__ int compact_positive_(const float* p, int* list, int* scan, int cap, int n) {
  const int chunk = (n + NT - 1) / NT;
  const int b = min(n, (int)threadIdx.x * chunk), e = min(n, b + chunk);
  int cnt = 0;
  for (int i = b; i < e; ++i) cnt += p[i] > 0.0f;
  int tot;
  int off = block_excl_scan<NT>(cnt, scan, &tot);
  for (int i = b; i < e; ++i)
    if (p[i] > 0.0f) {
      if (off < cap) list[off] = i;
      ++off;
    }
  __syncthreads();
  return tot;
}
template <int NT>
__device__ inline int compact_positive(const SampleSmem& sm, int n) {
  return compact_positive_<NT>(sm.p, sm.list, sm.scan, sm.cap, n);
}

// index-order sequential f32 sum of p by one wave (only positive entries contribute: +0 adds
// are exact); positive values staged into lanes, added in order from registers.
__device__ float wave_sum_positive_(const float* p, const int* list, int cap, int n, int npos) {
  const int lane = threadIdx.x & 63;
  float s = 0.0f;
  if (npos <= cap) {
    for (int q0 = 0; q0 < npos; q0 += 64) {
      const float v = (q0 + lane < npos) ? p[list[q0 + lane]] : 0.0f;
      const int cnt = min(64, npos - q0);
      for (int i = 0; i < cnt; ++i) s += readlane_f(v, i);
    }
  } else {
    for (int q0 = 0; q0 < n; q0 += 64) {
      const float v = (q0 + lane < n) ? p[q0 + lane] : 0.0f;
      const int cnt = min(64, n - q0);
      for (int i = 0; i < cnt; ++i) s += readlane_f(v, i);
    }
  }
  return s;
}
__device__ inline float wave_sum_positive(const SampleSmem& sm, int n, int npos) {
  return wave_sum_positive_(sm.p, sm.list, sm.cap, n, npos);
}

// ---------------------------------------------------------------------------------------
// Exact parallel emulation of the sequential f32 sum  s = (((0 + e0) + e1) + ...) + e_{n-1}
// for e_i >= 0 (rwkv_sampler.rs:88, `probs.iter().sum()`).
// While s stays inside one binade [2^E, 2^(E+1)), s = m * u with u = 2^(E-23) and
//   RN(s + e) = u * (m + a + c),  a = floor(e/u),  c = 1 if frac(e/u) > 1/2,
//   c = (m + a) & 1 if frac(e/u) == 1/2 (ties to even), else 0,
// so a run of additions only depends on the parity of m: it is a map {0,1} -> (increment,
// parity), and such maps compose. Each of 64 chunks is simulated for the binade predicted from
// the exact (double) prefix sum at its start; one lane then walks the chunks, applying a
// chunk's map when the running s really is in the predicted binade and stays in it (m + T <
// 2^24), and otherwise adding that chunk's elements one by one. The result is bit-identical
// to the sequential loop by construction.
// ---------------------------------------------------------------------------------------
__device__ inline void sum_sim_elem(uint32_t b, int E, uint32_t& T0, uint32_t& T1, int& q0, int& q1, bool& ok) {
  const uint32_t ef = (b >> 23) & 0xFFu;
  uint32_t M = b & 0x7FFFFFu;
  int ex;
  if (ef == 0) ex = -149;
  else { M |= 0x800000u; ex = (int)ef - 150; }
  uint32_t a = 0;
  int cls = 0;  // 0 below half, 1 tie, 2 above
  if (M != 0) {
    const int sh = (E - 23) - ex;
    if (sh <= 0) {
      if (sh < -8) { ok = false; return; }
      a = M << (-sh);
      if (a >= 0x1000000u) { ok = false; return; }
    } else if (sh <= 24) {
      a = M >> sh;
      const uint32_t r = M & ((1u << sh) - 1u), half = 1u << (sh - 1);
      cls = r > half ? 2 : (r == half ? 1 : 0);
    }
  }
  const uint32_t c0 = (cls == 2 || (cls == 1 && ((q0 + a) & 1u))) ? 1u : 0u;
  const uint32_t c1 = (cls == 2 || (cls == 1 && ((q1 + a) & 1u))) ? 1u : 0u;
  T0 += a + c0;
  T1 += a + c1;
  q0 = (int)((q0 + a + c0) & 1u);
  q1 = (int)((q1 + a + c1) & 1u);
  if (T0 >= 0x1000000u || T1 >= 0x1000000u) ok = false;
}

constexpr int kNoBinade = 1 << 20;  // sub_e of a sub-chunk whose simulation failed

struct NoOther {
  __device__ void operator()() const {}
};

// `other` runs on waves 1.. while wave 0 walks the chunk maps (the walk is serial; the other
// waves would idle). It may not use workgroup barriers.
template <int NT, typename Other = NoOther>
__device__ float exact_seq_sum_chunks(const SampleSmem& sm, int n, uint64_t* stamps = nullptr, const Other& other = Other()) {
  constexpr int NS = NT / 64;  // sub-chunks per chunk (64 chunks, one per lane of wave 0)
  constexpr int NE = NT >= 1024 ? 64 : 128;  // serial-add register batch
  const int tid = threadIdx.x;
  // chunks and sub-chunks start 16-byte aligned (the serial adds read float4)
  const int CH = (((n + 63) / 64) + 3) & ~3, SUB = (((CH + NS - 1) / NS) + 3) & ~3;
  const int chunk = tid / NS, sub = tid % NS;
  const int cb = min(n, chunk * CH), ce = min(n, cb + CH);
  const int sb = min(ce, cb + sub * SUB), se = min(ce, sb + SUB);
  double ds = 0.0;
  for (int i = sb; i < se; ++i) ds += (double)sm.p[i];
  double dtot;
  const double pre = block_excl_scan_t<NT, double>(ds, sm.dscan, &dtot);
  STAMP(10);
  // every sub-chunk is simulated for the binade predicted from the prefix at its OWN start, so a
  // chunk that crosses a binade still has usable sub-chunk maps on either side of the crossing
  const float pf = (float)pre;
  const uint32_t pb = __builtin_bit_cast(uint32_t, pf);
  const int E = (int)((pb >> 23) & 0xFFu) - 127;
  bool ok = pf >= 0x1p-100f && pf < 0x1p+100f;
  uint32_t T0 = 0, T1 = 0;
  int q0 = 0, q1 = 1;
  for (int i = sb; i < se && ok; ++i) sum_sim_elem(__builtin_bit_cast(uint32_t, sm.p[i]), E, T0, T1, q0, q1, ok);
  sm.sub_t[2 * tid] = T0;
  sm.sub_t[2 * tid + 1] = T1;
  sm.sub_e[tid] = ok ? E : kNoBinade;
  __syncthreads();
  STAMP(11);
  if (tid < 64) {  // compose the NS sub-chunk maps of chunk `tid` (all predicted in one binade)
    const int clen = min(n, tid * CH + CH) - min(n, tid * CH);
    const int E0 = sm.sub_e[NS * tid];
    bool cok = E0 != kNoBinade;
    for (int s = 1; s < NS; ++s) cok &= s * SUB >= clen || sm.sub_e[NS * tid + s] == E0;
    for (int pin = 0; pin < 2; ++pin) {
      int par = pin;
      uint32_t T = 0;
      for (int s = 0; s < NS; ++s) {
        const uint32_t t = sm.sub_t[2 * (NS * tid + s) + par];
        T += t;
        par = (int)((par + t) & 1u);
      }
      if (T >= 0x1000000u) cok = false;
      sm.chunk_t[2 * tid + pin] = T;
    }
    sm.chunk_ok[tid] = cok;
    sm.chunk_e[tid] = E0;
  }
  __syncthreads();
  STAMP(12);
  int nfast = 0;
  if (tid < 64) {
    // Wave 0. Chunk c's map lives in lane c. Runs of consecutive usable chunks predicted in the
    // same binade are composed by a segmented parallel prefix of their parity maps, so the walk
    // below does one O(1) step per run; unusable chunks (binade crossings) are added serially.
    const int nch = (n + CH - 1) / CH;
    const int lane = tid;
    const int okv = lane < nch ? sm.chunk_ok[lane] : 0, ev = sm.chunk_e[lane];
    uint32_t P0 = sm.chunk_t[2 * lane], P1 = sm.chunk_t[2 * lane + 1];
    const int okp = __shfl_up(okv, 1), evp = __shfl_up(ev, 1);
    const bool head = lane == 0 || !okv || !okp || evp != ev;
    bool F = head;
    // segmented inclusive scan: P = (chunks from the run head to this chunk), composed in order
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t q0 = __shfl_up(P0, o), q1 = __shfl_up(P1, o);
      const bool qf = __shfl_up(F ? 1 : 0, o) != 0;
      if (lane >= o && !F) {
        const uint32_t n0 = min(q0 + ((q0 & 1u) ? P1 : P0), 0x2000000u);        // incoming parity 0
        const uint32_t n1 = min(q1 + (((1u + q1) & 1u) ? P1 : P0), 0x2000000u);  // incoming parity 1
        P0 = n0;
        P1 = n1;
        F = qf;
      }
    }
    const uint64_t heads = __ballot(head) & (nch >= 64 ? ~0ull : ((1ull << nch) - 1ull));
    // chunk `lane`'s sub-chunk maps, for chunks that cannot be applied whole
    uint32_t sT0[NS], sT1[NS];
    int sE[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      sT0[j] = sm.sub_t[2 * (NS * lane + j)];
      sT1[j] = sm.sub_t[2 * (NS * lane + j) + 1];
      sE[j] = sm.sub_e[NS * lane + j];
    }
    uint64_t sadd_cyc = 0;  // diagnostics (stamps): cycles in element-wise fallback adds
    // chunk c in order: each sub-chunk by its map when s is in the binade it was simulated for
    // and stays there, otherwise element by element on one lane
    auto add_chunk = [&](float s, int c) -> float {
      const int cb0 = c * CH, ce0 = min(n, cb0 + CH);
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int b1 = cb0 + j * SUB;
        if (b1 < ce0) {
          s = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, s)));
          const uint32_t sb4 = __builtin_bit_cast(uint32_t, s);
          const int ef4 = (int)((sb4 >> 23) & 0xFFu);
          bool fast = false;
          if (ef4 != 0 && ef4 - 127 == readlane_i(sE[j], c)) {
            const uint32_t m = (sb4 & 0x7FFFFFu) | 0x800000u;
            const uint32_t T = (uint32_t)((m & 1u) ? readlane_i((int)sT1[j], c) : readlane_i((int)sT0[j], c));
            if (m + T < 0x1000000u) {
              s = __builtin_bit_cast(float, (sb4 & 0xFF800000u) | ((m + T) & 0x7FFFFFu));
              fast = true;
            }
          }
          if (!fast) {
            const int e1 = min(ce0, b1 + SUB);
            float t = 0.0f;
            const uint64_t fb = stamps ? __builtin_amdgcn_s_memtime() : 0;
            if (lane == 0) t = lane_serial_add<NE>(s, sm.p, b1, e1);
            s = readlane_f(t, 0);
            if (stamps) sadd_cyc += __builtin_amdgcn_s_memtime() + (uint64_t)(s != s) - fb;
          }
        }
      }
      return s;
    };
    float s = 0.0f;
    int c = 0;
    while (c < nch) {
      // s and c are wave-uniform; say so, so that the walk runs on scalar registers and scalar
      // branches (readlane with an SGPR lane select) instead of divergent-looking VGPR code
      s = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, s)));
      c = __builtin_amdgcn_readfirstlane(c);
      const uint32_t sb2 = __builtin_bit_cast(uint32_t, s);
      const int ef = (int)((sb2 >> 23) & 0xFFu);
      const bool is_head = (heads >> c) & 1ull;
      if (is_head && readlane_i(okv, c) && ef != 0 && ef - 127 == readlane_i(ev, c)) {
        const uint64_t later = heads >> (c + 1);
        const int r = later ? c + __ffsll((long long)later) - 1 : nch - 1;  // last chunk of the run
        const uint32_t m = (sb2 & 0x7FFFFFu) | 0x800000u;
        const uint32_t T = (uint32_t)((m & 1u) ? readlane_i((int)P1, r) : readlane_i((int)P0, r));
        if (m + T < 0x1000000u) {
          s = __builtin_bit_cast(float, (sb2 & 0xFF800000u) | ((m + T) & 0x7FFFFFu));
          nfast += r - c + 1;
          c = r + 1;
          continue;
        }
      }
      // unusable chunk, or a run whose prediction failed: add chunk c sub-chunk by sub-chunk
      s = add_chunk(s, c);
      ++c;
      // the chunks after c (if inside a run) are no longer run heads; step them one at a time
      while (c < nch && !((heads >> c) & 1ull)) {
        s = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, s)));
        c = __builtin_amdgcn_readfirstlane(c);
        const uint32_t sb3 = __builtin_bit_cast(uint32_t, s);
        const int ef3 = (int)((sb3 >> 23) & 0xFFu);
        bool fast = false;
        if (readlane_i(okv, c) && ef3 != 0 && ef3 - 127 == readlane_i(ev, c)) {
          const uint32_t m = (sb3 & 0x7FFFFFu) | 0x800000u;
          const uint32_t T = (uint32_t)((m & 1u) ? sm.chunk_t[2 * c + 1] : sm.chunk_t[2 * c]);
          if (m + T < 0x1000000u) {
            s = __builtin_bit_cast(float, (sb3 & 0xFF800000u) | ((m + T) & 0x7FFFFFu));
            fast = true;
            ++nfast;
          }
        }
        if (!fast) s = add_chunk(s, c);
        ++c;
      }
    }
    if (tid == 0) {
      sm.fred[16] = s;
      if (stamps) {
        stamps[14] = nfast;
        stamps[15] = sadd_cyc;
      }
    }
  } else {
    other();
  }
  __syncthreads();
  STAMP(13);
  return sm.fred[16];
}

// ---------------------------------------------------------------------------------------
// The same sum for rows up to kSampleMaxN, by binade runs instead of chunks. With e >= 0 the
// running f32 sum s_i (before element i) stays within gamma_n <= n 2^-24 (relative) of the exact
// prefix pre_i (Higham, recursive summation), and pre_i only grows. Element i is SAFE in binade E
// when pre_i >= 2^E (1 + d) and pre_{i+1} <= 2^(E+1) (1 - d), d = 2^-k >= 2 (n-1) 2^-24: then s_i and
// s_{i+1} are both in [2^E, 2^(E+1)), so the add is the quantised increment of the parity map
// above. The safe elements of one binade form ONE contiguous run (pre is monotone), so a run is
// keyed by E: its map is composed across the threads it spans by a segmented scan, and the walk
// applies one map per binade (about log2(sum / e_first) of them) and adds only the rest -- the
// ranges of the threads that hold a binade crossing -- one by one. The walk still
// checks each run against the real s and adds the run serially if a check fails (never, by the
// bound; the fallback keeps the result exact regardless).
// ---------------------------------------------------------------------------------------
constexpr int kRunEMin = -100, kRuns = 128;  // run table: binades [-100, 27]

struct PMap {  // parity map: from parity p, add T[p] ulps
  uint32_t t0, t1;
};
__device__ inline PMap pcompose(PMap a, PMap b) {  // a, then b
  const uint32_t n0 = a.t0 + ((a.t0 & 1u) ? b.t1 : b.t0);
  const uint32_t n1 = a.t1 + (((1u + a.t1) & 1u) ? b.t1 : b.t0);
  return PMap{min(n0, 0x2000000u), min(n1, 0x2000000u)};
}
template <int NT, typename Other = NoOther>
__device__ float exact_seq_sum_runs(const SampleSmem& sm, int n, uint64_t* stamps = nullptr, const Other& other = Other()) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int* rstart = sm.runs;
  int* rend = sm.runs + kRuns;
  uint32_t* rt = (uint32_t*)(sm.runs + 2 * kRuns);  // [kRuns][2]
  if (tid < kRuns) rend[tid] = -1;
  // safety band d = 2^-k >= 2 (n - 1) 2^-24 >= 2 gamma_(n-1) (n <= kSampleMaxN = 2^14: k >= 9)
  int lg = 0;
  while ((1 << lg) < n - 1) ++lg;
  const uint64_t dm = 1ull << (52 - (23 - lg));  // d 2^52 (the double fraction field of 1 + d)
  const int SUB = (n + NT - 1) / NT;
  const int b = min(n, tid * SUB), e = min(n, b + SUB);
  double ds = 0.0;
  for (int i = b; i < e; ++i) ds += (double)sm.p[i];
  double dtot;
  double lo = block_excl_scan_t<NT, double>(ds, sm.dscan, &dtot);  // its barriers order rend[] init
  STAMP(10);
  // pass 1: a thread whose whole range lies in one binade's safe band (its first and last
  // prefixes decide it: pre is monotone) composes the map of its range; any other range -- the
  // few that hold a binade crossing -- is left to the walk, element by element. The safety
  // tests read only the high words of the doubles: the band edges d 2^52 and 2^52 - 2 d 2^52 have
  // zero low words (d >= 2^-20), and the upper test is taken strictly (a stricter test only adds
  // elements to the walk).
  const uint32_t DM = (uint32_t)(dm >> 32), DMAX = (1u << 20) - 2 * DM;
  const uint32_t lw = (uint32_t)(__builtin_bit_cast(uint64_t, lo) >> 32);
  const uint32_t hw = (uint32_t)(__builtin_bit_cast(uint64_t, lo + ds) >> 32);
  const int E = (int)(lw >> 20) - 1023;  // lo >= 0: no sign bit
  const bool wsafe = b < e && E >= kRunEMin && E <= kRunEMin + kRuns - 1 && (lw & 0xFFFFFu) >= DM &&
                     (hw >> 20) == (lw >> 20) && (hw & 0xFFFFFu) < DMAX;
  PMap T{0u, 0u};
  if (wsafe) {
    for (int i = b; i < e; ++i) {
      // the element's increment in ulps of binade E (safe: sh >= 1), ties to even by parity
      const uint32_t xb = __builtin_bit_cast(uint32_t, sm.p[i]);
      const uint32_t ef = (xb >> 23) & 0xFFu;
      const uint32_t M = (xb & 0x7FFFFFu) | (ef ? 0x800000u : 0u);
      const int ex = ef ? (int)ef - 150 : -149;
      const int sh = min((E - 23) - ex, 31);
      const uint32_t a = M >> sh, r = M & ((1u << sh) - 1u), half = (1u << sh) >> 1;
      const uint32_t up = r > half ? 1u : 0u, tie = r == half ? 1u : 0u;
      const uint32_t m0 = a + (up | (tie & a & 1u)), m1 = a + (up | (tie & ~a & 1u));
      T.t0 += (T.t0 & 1u) ? m1 : m0;
      T.t1 += ((1u + T.t1) & 1u) ? m1 : m0;
    }
  }
  const int tE = wsafe ? E : kNoBinade;
  sm.sub_e[tid] = tE;
  // parity-free maps (no half-ulp tie anywhere: t0 == t1) compose by plain addition
  const int ties = __syncthreads_or(wsafe && T.t0 != T.t1);
  STAMP(11);
  const int prevE = tid > 0 ? sm.sub_e[tid - 1] : kNoBinade;
  const int nextE = tid + 1 < NT ? sm.sub_e[tid + 1] : kNoBinade;
  const bool contL = wsafe && prevE == tE, contR = wsafe && nextE == tE;
  if (wsafe && !contL) rstart[tE - kRunEMin] = b;
  if (wsafe && !contR) rend[tE - kRunEMin] = e;
  if (!ties) {
    // a run's map = (inclusive prefix at its last thread) - (exclusive prefix at its head), in
    // uint32 arithmetic mod 2^32 (a run adds < 2^24 ulps)
    uint32_t tot;
    const uint32_t P = block_excl_scan_t<NT, uint32_t>(wsafe ? T.t0 : 0u, (uint32_t*)sm.scan, &tot);
    if (wsafe && !contL) rt[2 * (tE - kRunEMin)] = P;
    __syncthreads();
    if (wsafe && !contR) {
      const uint32_t full = P + T.t0 - (contL ? rt[2 * (tE - kRunEMin)] : P);
      rt[2 * (tE - kRunEMin)] = full;
      rt[2 * (tE - kRunEMin) + 1] = full;
    }
  } else {
    // segmented exclusive scan over threads of (run head, parity map): carry = the run's map so far
    bool f = !contL;
    PMap x = T;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y0 = __shfl_up(x.t0, o), y1 = __shfl_up(x.t1, o);
      const bool yf = __shfl_up(f ? 1 : 0, o) != 0;
      if (lane >= o && !f) {
        x = pcompose(PMap{y0, y1}, x);
        f = yf;
      }
    }
    // wave totals -> LDS (the double scan's scratch: 8 x (flag, t0, t1) as ints)
    int* wt = (int*)sm.dscan;
    if (lane == 63) { wt[3 * w] = f ? 1 : 0; wt[3 * w + 1] = (int)x.t0; wt[3 * w + 2] = (int)x.t1; }
    uint32_t e0 = __shfl_up(x.t0, 1), e1 = __shfl_up(x.t1, 1);
    bool ef = __shfl_up(f ? 1 : 0, 1) != 0;
    if (lane == 0) { e0 = 0u; e1 = 0u; ef = false; }
    __syncthreads();
    PMap c{0u, 0u};  // carry into this wave: waves 0 .. w-1 in order
    for (int k = 0; k < w; ++k) {
      const PMap kv{(uint32_t)wt[3 * k + 1], (uint32_t)wt[3 * k + 2]};
      c = wt[3 * k] ? kv : pcompose(c, kv);
    }
    const PMap v = ef ? PMap{e0, e1} : pcompose(c, PMap{e0, e1});
    if (wsafe && !contR) {
      const PMap full = contL ? pcompose(v, T) : T;
      rt[2 * (tE - kRunEMin)] = full.t0;
      rt[2 * (tE - kRunEMin) + 1] = full.t1;
    }
  }
  __syncthreads();
  STAMP(12);
  if (tid < 64) {
    // wave 0 walks the runs in binade order (= element order), adding the unsafe elements
    // between them on lane 0
    const int s0 = rstart[lane], e0 = rend[lane], s1 = rstart[lane + 64], e1 = rend[lane + 64];
    const uint32_t a0 = rt[2 * lane], b0 = rt[2 * lane + 1], a1 = rt[2 * (lane + 64)], b1 = rt[2 * (lane + 64) + 1];
    uint64_t m0 = __ballot(e0 >= 0), m1 = __ballot(e1 >= 0);
    float s = 0.0f;
    int pos = 0;
    uint64_t sadd = 0;
    // unsafe elements in order: 64 at a time pulled into the lanes by one LDS read, then added
    // in order from the registers (no dependent LDS latency per element)
    auto serial = [&](int from, int to) {
      if (from >= to) return;
      const uint64_t t0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
      for (int q = from; q < to; q += 64) {
        const float v = q + lane < to ? sm.p[q + lane] : 0.0f;
        const int cnt = __builtin_amdgcn_readfirstlane(min(64, to - q));
        int i = 0;
        for (; i + 4 <= cnt; i += 4) {
          s += readlane_f(v, i);
          s += readlane_f(v, i + 1);
          s += readlane_f(v, i + 2);
          s += readlane_f(v, i + 3);
        }
        for (; i < cnt; ++i) s += readlane_f(v, i);
      }
      if (stamps) sadd += __builtin_amdgcn_s_memtime() + (uint64_t)(s != s) - t0;
    };
    while (m0 | m1) {
      const bool hiw = m0 == 0;
      const uint64_t m = hiw ? m1 : m0;
      const int l = __builtin_ctzll(m);
      if (hiw) m1 &= m1 - 1; else m0 &= m0 - 1;
      const int k = l + (hiw ? 64 : 0);
      const int rs = readlane_i(hiw ? s1 : s0, l), re = readlane_i(hiw ? e1 : e0, l);
      const uint32_t T0 = (uint32_t)readlane_i((int)(hiw ? a1 : a0), l);
      const uint32_t T1 = (uint32_t)readlane_i((int)(hiw ? b1 : b0), l);
      if (rs < pos) {  // cannot happen (runs are disjoint and ordered); stay exact regardless
        serial(pos, re);
        pos = max(pos, re);
        continue;
      }
      serial(pos, rs);
      s = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, s)));
      const uint32_t sb = __builtin_bit_cast(uint32_t, s);
      const int ef = (int)((sb >> 23) & 0xFFu);
      const uint32_t mm = (sb & 0x7FFFFFu) | 0x800000u;
      const uint32_t T = (mm & 1u) ? T1 : T0;
      if (ef != 0 && ef - 127 == k + kRunEMin && mm + T < 0x1000000u)
        s = __builtin_bit_cast(float, (sb & 0xFF800000u) | ((mm + T) & 0x7FFFFFu));
      else
        serial(rs, re);
      pos = re;
    }
    serial(pos, n);
    if (tid == 0) {
      sm.fred[16] = s;
      if (stamps) {
        stamps[14] = __builtin_amdgcn_s_memtime();
        stamps[15] = sadd;
      }
    }
  } else {
    other();
  }
  __syncthreads();
  STAMP(13);
  return sm.fred[16];
}

template <int NT, typename Other = NoOther>
__device__ float exact_seq_sum(const SampleSmem& sm, int n, uint64_t* stamps = nullptr, const Other& other = Other()) {
  if (n <= kSampleMaxN) return exact_seq_sum_runs<NT>(sm, n, stamps, other);
  return exact_seq_sum_chunks<NT>(sm, n, stamps, other);
}

// bitonic sort (descending) of M (power of two) keys in LDS by the whole workgroup
template <int NT>
__device__ void bitonic_desc(uint64_t* keys, int M) {
  for (int k = 2; k <= M; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < M; q += NT) {
        const int ixj = q ^ j;
        if (ixj > q) {
          const uint64_t A = keys[q], B = keys[ixj];
          const bool desc = (q & k) == 0;
          if (desc ? (A < B) : (A > B)) { keys[q] = B; keys[ixj] = A; }
        }
      }
      __syncthreads();
    }
  }
}

__device__ inline uint64_t pkey(float p, int i) {
  return ((uint64_t)__builtin_bit_cast(uint32_t, p) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
}

constexpr int kFastK = 256;     // largest top-k of the fast path
constexpr int kFastCap = 1024;  // candidate capacity (sm.keys[0, kFastCap)); ranked keys at 2048
static_assert(kSampleMaxSorted >= 2048 + kFastCap, "fast-path key regions");

// The fast path's candidates are exactly a superset of the top-k by (p desc, index asc):
// at least k elements have e >= L, so the k-th largest p is >= P = RN(L / S) (division rounds
// monotonically). An element left out has e < T = RN(L (1 - 2^-19)) < L (1 - 2^-20), so
// e / S < (L / S)(1 - 2^-20) and, with L / S normal (ulp <= 2^-23 of it), RN(e / S) <= P - 8 ulp < P:
// it can be neither in the top k nor tied with its last member.
__device__ inline bool sample_fast_ok(float sum, float L, int nc, int top_k) {
  if (!(sum > 0.0f) || !(L > 0.0f) || nc < top_k || nc > kFastCap) return false;
  const float P = L / sum;
  return P >= 0x1p-126f && P <= 1.0f;
}

__device__ inline float draw_r(const uint32_t* key, uint64_t draw, bool fixed42) {
  if (!fixed42) return draw_f32(key, draw);
  uint32_t k42[8];
  uint64_t st = 42;
  const uint64_t MUL = 6364136223846793005ull, INC = 11634580456473284103ull;
  for (int i = 0; i < 8; ++i) {
    st = st * MUL + INC;
    const uint32_t xs = (uint32_t)(((st >> 18) ^ st) >> 27);
    const uint32_t rot = (uint32_t)(st >> 59);
    k42[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
  }
  return draw_f32(k42, 0);
}

// Steps (2)-(6) of rwkv_sampler.rs:55-211 restricted to the candidates (temperature 1):
// p = e / S for the nc candidates, top-k by rank, top-p over the k sorted survivors (:108-153,
// cutoff, zeroing below it, the equal-to-cutoff adjustment with the index-order survivor sum),
// multinomial over the survivors in index order (:174-207). Every other element has p = 0 after
// top-k and adds exactly nothing to any sequential sum, so results equal the full path's.
template <int NT>
__device__ __attribute__((always_inline)) int sample_fast(const SampleSmem& sm, int nc, float sum, float top_p,
                                                          int top_k, const uint32_t* key, uint64_t draw,
                                                          bool fixed42, float* dbg, uint64_t* stamps) {
  const int tid = threadIdx.x;
  uint64_t* pk = sm.keys + 2048;
  for (int c = tid; c < nc; c += NT) {
    const uint64_t ce = sm.keys[c];
    pk[c] = pkey(__builtin_bit_cast(float, (uint32_t)(ce >> 32)) / sum, (int)(uint32_t)ce);
  }
  __syncthreads();
  STAMP(4);
  // top-k: rank among the candidates (keys unique), the k best land sorted in keys[0, k)
  for (int c = tid; c < nc; c += NT) {
    const uint64_t kc = pk[c];
    int rank = 0;
    for (int j = 0; j < nc; ++j) rank += pk[j] > kc ? 1 : 0;
    if (rank < top_k) sm.keys[rank] = kc;
  }
  __syncthreads();
  STAMP(5);
  STAMP(6);
  // top-p over the sorted survivors (all p >= P > 0): wave 0, sequential cumulative
  if (tid < 64) {
    int m = top_k, found = 0, ceq = 0;
    float cutoff = 0.0f;
    if (top_p < 1.0f) {
      float cum = 0.0f;
      for (int q0 = 0; q0 < top_k && !found; q0 += 64) {
        const bool in = q0 + tid < top_k;
        const float pv = in ? __builtin_bit_cast(float, (uint32_t)(sm.keys[q0 + tid] >> 32)) : 0.0f;
        float tot;
        const float pre = prefix64(cum, pv, &tot);
        const uint64_t hit = __ballot(in && pre >= top_p);
        if (hit) {
          found = 1;
          cutoff = readlane_f(pv, __builtin_ctzll(hit));
        }
        cum = tot;
      }
      if (found) {  // survivors p >= cutoff: a prefix of the sorted order
        m = 0;
        for (int q0 = 0; q0 < top_k; q0 += 64) {
          const bool in = q0 + tid < top_k;
          const float pv = in ? __builtin_bit_cast(float, (uint32_t)(sm.keys[q0 + tid] >> 32)) : 0.0f;
          m += __popcll(__ballot(in && pv >= cutoff));
          ceq += __popcll(__ballot(in && pv == cutoff));
        }
      }
    }
    if (tid == 0) {
      sm.ired[2] = found;
      sm.ired[3] = ceq;
      sm.ired[6] = m;
      sm.fred[17] = cutoff;
    }
  }
  __syncthreads();
  const int m = sm.ired[6];
  // survivors into index order: list[rank by index] = index, p at its index
  for (int t = tid; t < m; t += NT) {
    const uint64_t kt = sm.keys[t];
    const uint32_t lt = (uint32_t)kt;  // ~index: larger means a smaller index
    int r = 0;
    for (int j = 0; j < m; ++j) r += (uint32_t)sm.keys[j] > lt ? 1 : 0;
    const int it = (int)(0xFFFFFFFFu - lt);
    sm.list[r] = it;
    sm.p[it] = __builtin_bit_cast(float, (uint32_t)(kt >> 32));
  }
  __syncthreads();
  STAMP(7);
  STAMP(8);
  if (tid < 64) {
    const int found = sm.ired[2], ceq = sm.ired[3];
    const float cutoff = sm.fred[17];
    bool adj_on = false;
    float adj = 0.0f;
    if (top_p < 1.0f && found && top_p > 0.0f) {
      float s2 = 0.0f;  // index-order sequential sum of the survivors (:129)
      for (int q0 = 0; q0 < m; q0 += 64) {
        const float v = q0 + tid < m ? sm.p[sm.list[q0 + tid]] : 0.0f;
        const int cnt = min(64, m - q0);
        for (int i = 0; i < cnt; ++i) s2 += readlane_f(v, i);
      }
      if (s2 < top_p && ceq > 0) {
        adj = (top_p - s2) / (float)ceq;
        adj_on = true;
      }
    }
    const float r = sm.fred[21];  // the draw, made by the last wave during the exact sum
    int ret = -1;
    if (r <= 0.0f) {
      ret = 0;  // cum at index 0 is >= 0 >= r
    } else {
      float cum = 0.0f;
      for (int q0 = 0; q0 < m && ret < 0; q0 += 64) {
        const bool in = q0 + tid < m;
        const int idx_l = in ? sm.list[q0 + tid] : 0;
        float v = in ? sm.p[idx_l] : 0.0f;
        if (adj_on && in && v == cutoff) v = cutoff + adj;
        float tot;
        const float pre = prefix64(cum, v, &tot);
        const uint64_t hit = __ballot(in && r <= pre);
        if (hit) ret = readlane_i(idx_l, __builtin_ctzll(hit));
        cum = tot;
      }
      if (ret < 0) ret = sm.list[m - 1];  // highest index with p > 0 (:183-189)
    }
    if (tid == 0) {
      sm.ired[5] = ret;
      if (dbg) { dbg[0] = sum; dbg[1] = r; }
    }
  }
  __syncthreads();
  STAMP(9);
  return sm.ired[5];
}

// ---------------------------------------------------------------------------------------
// Certified fast path: the token WITHOUT the exact sequential softmax sum.
//
// The exact emulation of the sequential f32 sum S (exact_seq_sum) is the serial part of the
// sampler. But the sampled index depends on S only through comparisons -- top-k membership,
// the top-p cut, and the draw r against the index-order cumulative -- and S lies within a
// rigorous interval around the real sum E = sum e_i (computed here in f64, to ~n 2^-53):
// recursive f32 summation of n non-negative terms errs by at most (n - 1) 2^-24 E (1 + O(n u)),
// widened here to n 2^-23 E. Every p_i = RN(e_i / S) then lies in [e_i / S_hi (1 - 2^-24),
// e_i / S_lo (1 + 2^-24)] and every sequential f32 cumulative of j + 1 such terms within
// (1 -+ (j + 1) 2^-23) of the exact sums of those bounds. When, over that whole interval,
// (a) the k-th and (k+1)-th largest e (by e desc, index asc) cannot round to equal p (ratio >= 1 +
//     2^-22, p normal), so the top-k set is the one ranked on e,
// (b) the top-p cumulative over the k survivors stays below top_p (no cut: rwkv_sampler.rs:108-153
//     then changes nothing), and
// (c) r is not inside the uncertainty band of the cumulative it is compared with,
// the result equals the exact algorithm's for EVERY S in the interval, hence for the exact S;
// otherwise the caller runs the exact sum. Returns the index, or -1 (not certified).
// sm.keys[0, nc): candidates (e bits << 32 | index); E: f64 sum of e over the row; r: the draw.
// The crude relative bound on the sequential f32 sum S of n non-negative terms around their real
// sum E: recursive summation errs by at most (n - 1) 2^-24 E, widened to n 2^-23, plus the f64
// sum's own error.
__device__ inline double crude_sum_eps(int n) { return (double)n * 0x1p-23 + 0x1p-36; }

template <int NT>
__device__ __attribute__((always_inline)) int sample_cert(const SampleSmem& sm, int n, int nc, double E, float r, float top_p, int top_k,
                           double eps, uint64_t* stamps = nullptr) {
  const int tid = threadIdx.x;
  STAMP(7);
  uint64_t* srt = sm.keys + 2048;  // candidates ranked by (e desc, index asc)
  uint64_t* idx_o = sm.keys + 3072;  // survivors in index order (e bits << 32 | index)
  static_assert(kSampleMaxSorted >= 3072 + kFastK, "certified-path key regions");
  auto qkey = [&](int j) {
    const uint64_t kj = sm.keys[j];
    return (kj & 0xFFFFFFFF00000000ull) | (uint64_t)(0xFFFFFFFFu - (uint32_t)kj);
  };
  for (int c0 = 0; c0 < nc; c0 += NT) {
    if (c0 + (tid & ~63) >= nc) break;  // wave-uniform: no candidate in this wave
    const int c = c0 + tid;
    const uint64_t qc = c < nc ? qkey(c) : ~0ull;
    const int rank = wave_rank_gt(qc, nc, qkey);
    if (c < nc) srt[rank] = qc;
  }
  __syncthreads();
  STAMP(8);
  // survivors (ranks < k) into index order
  for (int t0 = 0; t0 < top_k; t0 += NT) {
    if (t0 + (tid & ~63) >= top_k) break;  // wave-uniform
    const int t = t0 + tid;
    const uint64_t kt = t < top_k ? srt[t] : 0ull;
    const uint32_t it = 0xFFFFFFFFu - (uint32_t)kt;
    // rank by index ascending == rank by ~index descending: #{j : ~idx_j > ~idx_t}
    auto nkey = [&](int j) { return (uint64_t)(uint32_t)srt[j]; };
    const int ri = wave_rank_gt((uint64_t)(uint32_t)kt, top_k, nkey);
    if (t < top_k) idx_o[ri] = (kt & 0xFFFFFFFF00000000ull) | it;
  }
  __syncthreads();
  STAMP(9);
  int ret = -1;
  if (tid < 64) {
    const double s_lo = E * (1.0 - eps), s_hi = E * (1.0 + eps);
    const double u = 0x1p-24, ua = 0x1p-23;
    bool ok = E > 0.0 && s_lo > 0.0 && E < 3.0e38;
    // (a) the top-k boundary
    const float ek = __builtin_bit_cast(float, (uint32_t)(srt[top_k - 1] >> 32));
    if (ok && nc > top_k) {
      const float eb = __builtin_bit_cast(float, (uint32_t)(srt[top_k] >> 32));
      ok = (double)ek >= (double)eb * (1.0 + 0x1p-22);
    }
    // (nc == k: every non-candidate has e < L (1 - 2^-19) <= e_k (1 - 2^-19), see sample_fast_ok)
    ok = ok && (double)ek / s_hi >= 0x1p-120;
    // (b) no top-p cut: the whole survivor mass stays below top_p
    double tot_hi = 0.0;
    for (int q0 = 0; q0 < top_k; q0 += 64) {
      const double e = q0 + tid < top_k ? (double)__builtin_bit_cast(float, (uint32_t)(idx_o[q0 + tid] >> 32)) : 0.0;
      tot_hi += readlane_d(wave_incl_scan_d(e), 63);
    }
    tot_hi = tot_hi / s_lo * (1.0 + u) * (1.0 + (double)top_k * ua);
    if (top_p < 1.0f) ok = ok && tot_hi < (double)top_p;
    STAMP(12);
    // (c) the draw against the index-order cumulative
    if (ok) {
      if (r <= 0.0f) {
        ret = 0;  // cum at index 0 is >= 0 >= r
      } else {
        double plo = 0.0, phi = 0.0, hi_prev = 0.0;
        bool amb = false;
        for (int q0 = 0; q0 < top_k && ret < 0 && !amb; q0 += 64) {
          const bool in = q0 + tid < top_k;
          const uint64_t kv = in ? idx_o[q0 + tid] : 0ull;
          const double e = in ? (double)__builtin_bit_cast(float, (uint32_t)(kv >> 32)) : 0.0;
          // inclusive prefix sums of the p bounds (lane order = index order)
          const double a = wave_incl_scan_d(e / s_hi * (1.0 - u)), b = wave_incl_scan_d(e / s_lo * (1.0 + u));
          const int j = q0 + tid;  // survivors summed so far: j + 1
          const double lo = (plo + a) * (1.0 - (double)(j + 1) * ua);
          const double hi = (phi + b) * (1.0 + (double)(j + 1) * ua);
          const uint64_t le = __ballot(in && (double)r <= lo);
          const uint64_t hm = __ballot(in && (double)r <= hi);  // possibly at or before
          if (le) {
            const int f = __builtin_ctzll(le);
            // no earlier survivor may catch r: the first possible one is f itself
            const int fh = __builtin_ctzll(hm);
            if (fh == f && (f > 0 || hi_prev < (double)r)) ret = __builtin_amdgcn_readlane((int)(uint32_t)kv, f);
            else amb = true;
          } else if (hm) {
            amb = true;
          }
          plo = readlane_d(plo + a, 63);
          phi = readlane_d(phi + b, 63);
          hi_prev = phi * (1.0 + (double)min(q0 + 64, top_k) * ua);
        }
        if (ret < 0 && !amb) ret = (int)(uint32_t)idx_o[top_k - 1];  // past every survivor: highest index
        if (amb) ret = -1;
      }
    }
    if (tid == 0) sm.ired[7] = ret;
  }
  STAMP(13);
  __syncthreads();
  return sm.ired[7];
}

// The sampler. p holds the (masked) logits on entry. Returns the index in every thread.
// status: 0 ok, RWKVTTS_EUNSUPPORTED for the documented limitation.
template <int NT>
__device__ __attribute__((always_inline)) int sample_block(const SampleSmem& sm, int n, float temperature, float top_p,
                            int top_k, const uint32_t* key, uint64_t draw, bool fixed42,
                            float* dbg, int* status, uint64_t* stamps = nullptr, bool cert = true,
                            bool prepped = false) {
  const int tid = threadIdx.x;
  *status = 0;
  if (n == 0) return 0;
  if (!prepped) STAMP(1);
  // (2) softmax: max, exp, sequential sum (exact emulation), divide. prepped (advance_prep): p
  // already holds e = exp(l - max), the candidates, L, the f64 sum and the draw are in place.
  if (!prepped) {
  float mx = -__builtin_inff();
  if (tid < 32) sm.etab[tid] = exp2_tab(tid);  // ordered before the reads by block_max's barriers
  for (int i = tid; i < n; i += NT) mx = fmaxf(mx, sm.p[i]);
  mx = block_max<NT>(mx, sm.fred);
  {
    const uint64_t* et = sm.etab;
    auto tab = [et](int i) { return et[i]; };
    int i = tid;
    for (; i + 3 * NT < n; i += 4 * NT) {  // four independent elements per round
      const float x0 = sm.p[i], x1 = sm.p[i + NT], x2 = sm.p[i + 2 * NT], x3 = sm.p[i + 3 * NT];
      sm.p[i] = glibc_expf_t(x0 - mx, tab);
      sm.p[i + NT] = glibc_expf_t(x1 - mx, tab);
      sm.p[i + 2 * NT] = glibc_expf_t(x2 - mx, tab);
      sm.p[i + 3 * NT] = glibc_expf_t(x3 - mx, tab);
    }
    for (; i < n; i += NT) sm.p[i] = glibc_expf_t(sm.p[i] - mx, tab);
  }
  }
  // Fast path (top-k <= kFastK, no temperature step): while wave 0 walks the exact sum, the
  // other waves collect the top-k candidates on the unnormalised e = exp(l - max), so that after
  // the sum only the candidates are divided, ranked and sampled. See sample_fast_ok below.
  static_assert(NT <= 512, "fred[8 + wave] per candidate wave");
  const bool want_fast = top_k > 0 && top_k < n && top_k <= kFastK && !(temperature != 1.0f && temperature > 0.0f);
  if (tid == 0 && !prepped) {
    sm.ired[30] = 0;  // sub-group arrival counter of the candidate waves
    sm.ired[31] = 0;  // candidate count
    sm.fred[20] = 0.0f;
  }
  __syncthreads();
  STAMP(2);
  auto collect = [&]() {
    if (!want_fast) return;
    constexpr int NC = NT - 64, NWC = NT / 64 - 1;
    const int ct = tid - 64, lane = tid & 63;
    // lower bound L of the k-th largest e: min over the NWC waves of the ceil(k/NWC)-th largest
    // thread-local maximum (each wave holds that many disjoint elements >= L)
    float lm = -1.0f;
    for (int i = ct; i < n; i += NC) lm = fmaxf(lm, sm.p[i]);
    const int kw = (top_k + NWC - 1) / NWC;
    int gt = 0, ge = 0;
#pragma unroll 16
    for (int j = 0; j < 64; ++j) {
      const float o = readlane_f(lm, j);
      gt += o > lm ? 1 : 0;
      ge += o >= lm ? 1 : 0;
    }
    const uint64_t selm = __ballot(gt < kw && kw <= ge);
    const float vw = readlane_f(lm, __builtin_ctzll(selm));
    if (lane == 0) {
      sm.fred[8 + (tid >> 6)] = vw;
      __hip_atomic_fetch_add(&sm.ired[30], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // sub-group barrier of the candidate waves (wave 0 is busy in the walk; all waves of the
    // workgroup are resident, so the spin terminates)
    while (__hip_atomic_load(&sm.ired[30], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NWC)
      __builtin_amdgcn_s_sleep(1);
    float L = sm.fred[9];
#pragma unroll
    for (int w = 2; w < NT / 64; ++w) L = fminf(L, sm.fred[8 + w]);
    if (!(L > 0.0f)) return;  // no usable bound: the general path runs
    if (tid == 64) sm.fred[20] = L;
    // candidates: e >= T = L (1 - 2^-19) (see sample_fast_ok), appended as (e bits, index)
    const float T = L * (1.0f - 0x1p-19f);
    for (int i0 = 0; i0 < n; i0 += NC) {
      const int i = i0 + ct;
      const float v = i < n ? sm.p[i] : 0.0f;
      const bool c = i < n && v >= T;
      const uint64_t bm = __ballot(c);
      if (bm) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&sm.ired[31], __popcll(bm));
        base = __builtin_amdgcn_readfirstlane(base);
        const int off = base + __popcll(bm & ((1ull << lane) - 1ull));
        if (c && off < kFastCap) sm.keys[off] = ((uint64_t)__builtin_bit_cast(uint32_t, v) << 32) | (uint32_t)i;
      }
    }
  };
  // waves 1..: the candidates, then (last wave) the uniform draw of step (6) -- a ChaCha12
  // block, thousands of cycles on one wave -- both while wave 0 walks the exact sum
  auto other = [&]() {
    collect();
    if (tid == NT - 64) sm.fred[21] = draw_r(key, draw, fixed42);
  };
  // certified path (sample_cert): wave 0 takes the real sum in f64 while the others collect the
  // candidates and draw; the exact sequential sum runs only when the decision is not certified
  // (one instance of exact_seq_sum either way: its `other` work is skipped once done)
  bool other_done = prepped;
  if (prepped) {
    const int nc = sm.ired[31];
    const float L = sm.fred[20];
    if (want_fast && !dbg && cert && n <= kSampleMaxN && L > 0.0f && nc >= top_k && nc <= kFastCap) {
      const int ret = sample_cert<NT>(sm, n, nc, sm.dscan[12], sm.fred[21], top_p, top_k, sm.dscan[13], stamps);
      STAMP(11);
      if (ret >= 0) return ret;
    }
  } else if (want_fast && !dbg && cert && n <= kSampleMaxN) {
    if (tid < 64) {
      double e = 0.0;
      for (int i = tid; i < n; i += 64) e += (double)sm.p[i];
      for (int o = 32; o >= 1; o >>= 1) e += __shfl_xor(e, o);
      if (tid == 0) sm.dscan[12] = e;
    } else {
      other();
    }
    __syncthreads();
    STAMP(10);
    other_done = true;
    const int nc = sm.ired[31];
    const float L = sm.fred[20];
    if (L > 0.0f && nc >= top_k && nc <= kFastCap) {
      const int ret = sample_cert<NT>(sm, n, nc, sm.dscan[12], sm.fred[21], top_p, top_k, crude_sum_eps(n));
      STAMP(11);
      if (ret >= 0) return ret;
    }
  }
  auto other_once = [&]() {
    if (!other_done) other();
  };
  const float sum = exact_seq_sum<NT>(sm, n, stamps, other_once);
  STAMP(3);
  if (want_fast) {
    const int nc = sm.ired[31];
    const float L = sm.fred[20];
    if (sample_fast_ok(sum, L, nc, top_k)) return sample_fast<NT>(sm, nc, sum, top_p, top_k, key, draw, fixed42, dbg, stamps);
  }
  if (sum > 0.0f)
    for (int i = tid; i < n; i += NT) sm.p[i] = sm.p[i] / sum;
  __syncthreads();
  STAMP(4);
  // sorted (p desc, index asc) candidate keys; valid for the first n_sorted entries
  int n_sorted = -1;
  // (3) top-k (:95-105): candidates above a lower bound of the k-th largest, sorted
  if (top_k > 0 && top_k < n) {
    bool done = false;
    if (top_k <= 64 * (NT / 64)) {
      // lower bound L: min over waves of the ceil(k/NW)-th largest thread-local maximum (each of
      // the NW waves holds that many disjoint elements >= L, so at least k elements are >= L)
      const int chunk = (n + NT - 1) / NT;
      const int b = min(n, tid * chunk), e = min(n, b + chunk);
      float lm = -1.0f;  // every p >= 0
      for (int i = b; i < e; ++i) lm = fmaxf(lm, sm.p[i]);
      // the kw-th largest of the wave's 64 local maxima: the value v with #{> v} < kw <= #{>= v}
      // (every lane counts against all 64 values read back through readlane; ties give the same v)
      const int lane = tid & 63;
      const int kw = (top_k + NT / 64 - 1) / (NT / 64);
      int gt = 0, ge = 0;
#pragma unroll 16
      for (int j = 0; j < 64; ++j) {
        const float o = readlane_f(lm, j);
        gt += o > lm ? 1 : 0;
        ge += o >= lm ? 1 : 0;
      }
      const uint64_t selm = __ballot(gt < kw && kw <= ge);
      const float vw = readlane_f(lm, __builtin_ctzll(selm));
      if (lane == 0) sm.fred[tid >> 6] = vw;
      __syncthreads();
      float Lm = sm.fred[0];
#pragma unroll
      for (int w = 1; w < NT / 64; ++w) Lm = fminf(Lm, sm.fred[w]);
      const float L = fmaxf(Lm, 0.0f);
      int cnt = 0;
      for (int i = b; i < e; ++i) cnt += sm.p[i] >= L;
      int tot;
      int off = block_excl_scan<NT>(cnt, sm.scan, &tot);
      if (tot <= sm.cap) {
        for (int i = b; i < e; ++i)
          if (sm.p[i] >= L) sm.keys[off++] = pkey(sm.p[i], i);
        if (tot <= NT) {
          // rank sort (keys are unique): candidate tid's place = number of larger keys; every
          // thread reads the same key per iteration (LDS broadcast) and one barrier replaces the
          // bitonic network's log2(M)(log2(M)+1)/2 barrier stages
          __syncthreads();
          const uint64_t kq = tid < tot ? sm.keys[tid] : 0ull;
          int rank = 0;
          if (tid < tot)
            for (int j = 0; j < tot; ++j) rank += sm.keys[j] > kq ? 1 : 0;
          __syncthreads();
          if (tid < tot) sm.keys[rank] = kq;
          __syncthreads();
        } else {
          int M = 1;
          while (M < tot) M <<= 1;
          for (int q = tot + tid; q < M; q += NT) sm.keys[q] = 0ull;
          __syncthreads();
          bitonic_desc<NT>(sm.keys, M);
        }
        // zero everything, then restore the k survivors
        for (int i = tid; i < n; i += NT) sm.p[i] = 0.0f;
        __syncthreads();
        for (int q = tid; q < top_k; q += NT) {
          const uint64_t kk = sm.keys[q];
          sm.p[0xFFFFFFFFu - (uint32_t)kk] = __builtin_bit_cast(float, (uint32_t)(kk >> 32));
        }
        __syncthreads();
        n_sorted = top_k;
        done = true;
      }
    }
    if (!done) {  // general path: bisection on the bits of the k-th largest probability
      uint32_t lo = 0, hi = 0x7F800000u;
      int cnt_hi = 0, it = 0;
      while (hi - lo > 1) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        int c = 0;
        for (int i = tid; i < n; i += NT) c += __builtin_bit_cast(uint32_t, sm.p[i]) >= mid;
        c = wave_sum_i(c);
        if ((tid & 63) == 0) sm.ired[8 + (it & 1) * (NT / 64) + (tid >> 6)] = c;
        __syncthreads();
        const int* r4 = sm.ired + 8 + (it & 1) * (NT / 64);
        int t4 = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) t4 += r4[w];
        if (t4 >= top_k) lo = mid;
        else { hi = mid; cnt_hi = t4; }
        ++it;
      }
      const float t = __builtin_bit_cast(float, lo);
      const int need_eq = top_k - cnt_hi;
      const int chunk = (n + NT - 1) / NT;
      const int b = min(n, tid * chunk), e = min(n, b + chunk);
      int cnt = 0;
      for (int i = b; i < e; ++i) cnt += (sm.p[i] == t);
      int tot;
      int rank = block_excl_scan<NT>(cnt, sm.scan, &tot);
      for (int i = b; i < e; ++i) {
        const float v = sm.p[i];
        if (v < t) sm.p[i] = 0.0f;
        else if (v == t) {
          if (rank >= need_eq) sm.p[i] = 0.0f;
          ++rank;
        }
      }
      __syncthreads();
    }
  }
  STAMP(5);
  int npos = compact_positive<NT>(sm, n);
  STAMP(6);
  // (4) top-p (:108-153)
  if (top_p < 1.0f) {
    if (n_sorted < 0 || n_sorted > npos) {
      // survivors not yet sorted (or fewer positives than k): sort the positive ones
      if (npos > sm.cap) {
        *status = RWKVTTS_EUNSUPPORTED;
        return 0;
      }
      int M = 1;
      while (M < npos) M <<= 1;
      for (int q = tid; q < M; q += NT) sm.keys[q] = q < npos ? pkey(sm.p[sm.list[q]], sm.list[q]) : 0ull;
      __syncthreads();
      bitonic_desc<NT>(sm.keys, M);
    }
    if (tid < 64) {  // sequential cumulative in sorted order (wave-uniform, keys staged in lanes)
      float cum = 0.0f, cutoff = 0.0f;
      int found = 0;
      for (int q0 = 0; q0 < npos && !found; q0 += 64) {
        const bool in = q0 + tid < npos;
        const float pv_l = in ? __builtin_bit_cast(float, (uint32_t)(sm.keys[q0 + tid] >> 32)) : 0.0f;
        float tot;
        const float pre = prefix64(cum, pv_l, &tot);
        const uint64_t hit = __ballot(in && pre >= top_p);
        if (hit) {
          const int i = __builtin_ctzll(hit);
          found = 1;
          cutoff = readlane_f(pv_l, i);
        }
        cum = tot;
      }
      if (!found && 0.0f >= top_p && npos < n) { found = 1; cutoff = 0.0f; }  // top_p <= 0 with zeros
      if (tid == 0) {
        sm.fred[17] = cutoff;
        sm.ired[2] = found;
      }
    }
    __syncthreads();
    if (sm.ired[2]) {
      const float cutoff = sm.fred[17];
      for (int i = tid; i < n; i += NT)
        if (sm.p[i] < cutoff) sm.p[i] = 0.0f;
      __syncthreads();
      if (top_p > 0.0f) {
        npos = compact_positive<NT>(sm, n);
        if (tid == 0) sm.ired[3] = 0;
        __syncthreads();
        int c = 0;
        for (int i = tid; i < n; i += NT) c += (sm.p[i] == cutoff);
        c = wave_sum_i(c);
        if ((tid & 63) == 0) atomicAdd(&sm.ired[3], c);
        __syncthreads();
        if (tid < 64) {
          const float cur = wave_sum_positive(sm, n, npos);
          if (tid == 0) {
            sm.ired[4] = 0;
            if (cur < top_p && sm.ired[3] > 0) {
              sm.fred[18] = (top_p - cur) / (float)sm.ired[3];
              sm.ired[4] = 1;
            }
          }
        }
        __syncthreads();
        if (sm.ired[4]) {
          const float adj = sm.fred[18];
          for (int i = tid; i < n; i += NT)
            if (sm.p[i] == cutoff) sm.p[i] = cutoff + adj;
          __syncthreads();
        }
      }
    }
    npos = compact_positive<NT>(sm, n);
  }
  STAMP(7);
  // (5) temperature (:156-171)
  if (temperature != 1.0f && temperature > 0.0f) {
    const float tinv = 1.0f / temperature;
    for (int i = tid; i < n; i += NT) {
      const float v = sm.p[i];
      if (v > 0.0f) sm.p[i] = (float)exp2(log2((double)v) * (double)tinv);
    }
    __syncthreads();
    npos = compact_positive<NT>(sm, n);
    if (tid < 64) {
      const float s2 = wave_sum_positive(sm, n, npos);
      if (tid == 0) sm.fred[19] = s2;
    }
    __syncthreads();
    const float s2 = sm.fred[19];
    if (s2 > 0.0f)
      for (int i = tid; i < n; i += NT) sm.p[i] = sm.p[i] / s2;
    __syncthreads();
  }
  STAMP(8);
  // (6) multinomial (:174-207): wave 0, cumulative in index order from lanes
  if (tid < 64) {
    const float r = sm.fred[21];  // the draw, made by the last wave during the exact sum
    int ret = -1;
    if (r <= sm.p[0]) {
      ret = 0;
    } else {
      const bool listed = npos <= sm.cap;
      const int cnt_all = listed ? npos : n;
      float cum = 0.0f;
      int last_pos = -1;
      for (int q0 = 0; q0 < cnt_all && ret < 0; q0 += 64) {
        const bool in = q0 + tid < cnt_all;
        const int idx_l = in ? (listed ? sm.list[q0 + tid] : q0 + tid) : 0;
        const float v = in ? sm.p[idx_l] : 0.0f;
        float tot;
        const float pre = prefix64(cum, v, &tot);
        const uint64_t hit = __ballot(in && r <= pre);
        const uint64_t posm = __ballot(in && v > 0.0f);
        if (posm) last_pos = readlane_i(idx_l, 63 - __builtin_clzll(posm));
        if (hit) ret = readlane_i(idx_l, __builtin_ctzll(hit));
        cum = tot;
      }
      if (ret < 0) ret = last_pos;  // highest index with p > 0 (:183-189)
    }
    if (ret < 0) ret = 0;
    if (tid == 0) {
      sm.ired[5] = ret;
      if (dbg) { dbg[0] = sum; dbg[1] = r; }
    }
  }
  __syncthreads();
  STAMP(9);
  return sm.ired[5];
}

template <int NT>
__device__ SampleSmem carve(char* base, int n, bool sorted_in_lds = true) {
  SampleSmem sm;
  const int npad = (n + 3) & ~3;
  const int ns = sorted_in_lds ? kSampleMaxSorted : 0;
  char* q = base;
  sm.p = (float*)q; q += (size_t)npad * 4;
  sm.keys = (uint64_t*)q; q += (size_t)ns * 8;
  sm.dscan = (double*)q; q += 16 * 8;
  sm.list = (int*)q; q += (size_t)ns * 4;
  sm.scan = (int*)q; q += 16 * 4;
  sm.sub_t = (uint32_t*)q; q += 2 * NT * 4;
  sm.sub_e = (int*)q; q += NT * 4;
  sm.chunk_e = (int*)q; q += 64 * 4;
  sm.chunk_t = (uint32_t*)q; q += 128 * 4;
  sm.chunk_ok = (int*)q; q += 64 * 4;
  sm.runs = (int*)q; q += 4 * kRuns * 4;
  sm.etab = (uint64_t*)q; q += 32 * 8;
  sm.fred = (float*)q; q += 32 * 4;
  sm.ired = (int*)q;
  sm.cap = kSampleMaxSorted;
  return sm;
}
template <int NT>
inline size_t smem_bytes(int n) {
  const int npad = (n + 3) & ~3;
  return (size_t)npad * 4 + kSampleMaxSorted * 8 + 16 * 8 + kSampleMaxSorted * 4 + 16 * 4 + 2 * NT * 4 + NT * 4 +
         256 + 512 + 256 + 4 * kRuns * 4 + 32 * 8 + 32 * 4 + 48 * 4;
}
constexpr int kSampleThreads = 512;  // one workgroup per sampled row

__global__ __launch_bounds__(kSampleThreads) void k_sample_rows(SampleRowArgs a) {
  constexpr int NT = kSampleThreads;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SampleSmem sm = carve<NT>(smem, a.n);
  const int row = blockIdx.x;
  uint64_t* stamps = a.stamps ? a.stamps + row * 16 : nullptr;
  STAMP(0);
  const float* lg = a.logits + (int64_t)row * a.ld;
  for (int i = threadIdx.x; i < a.n; i += NT) sm.p[i] = lg[i];
  __syncthreads();
  if (threadIdx.x == 0 && a.forbid >= 0 && a.forbid < a.n) sm.p[a.forbid] = -__builtin_inff();
  __syncthreads();
  int status;
  const int id = sample_block<NT>(sm, a.n, a.temperature, a.top_p, a.top_k,
                              a.keys ? a.keys + row * 8 : nullptr, a.draws ? a.draws[row] : 0,
                              a.keys == nullptr, a.dbg ? a.dbg + row * 2 : nullptr, &status, stamps);
  if (threadIdx.x == 0) a.out[row] = status ? status : id;
}

// Rows longer than kSampleMaxN: the row (p), its sort keys and index list live in a per-row
// global scratch region (wide_scratch_bytes), the small scan / reduction arrays in LDS. All of
// the row's accesses stay inside its own workgroup, whose barriers order them.
__host__ __device__ inline int wide_keys_len(int n) {
  int m = 1;
  while (m < n) m <<= 1;
  return m;
}
size_t wide_scratch_bytes(int n) {
  const size_t npad = (size_t)((n + 3) & ~3);
  return (npad * 4 + (size_t)wide_keys_len(n) * 8 + (size_t)n * 4 + 255) & ~(size_t)255;
}

__global__ __launch_bounds__(kSampleThreads) void k_sample_rows_wide(SampleRowArgs a) {
  constexpr int NT = kSampleThreads;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int row = blockIdx.x;
  char* g = a.scratch + (size_t)row * a.scratch_stride;
  // small arrays in LDS (carve with n = 0 and no keys / list), the row's arrays in scratch
  SampleSmem sm = carve<NT>(smem, 0, false);
  sm.p = (float*)g;
  sm.keys = (uint64_t*)(g + (size_t)((a.n + 3) & ~3) * 4);
  sm.list = (int*)((char*)sm.keys + (size_t)wide_keys_len(a.n) * 8);
  sm.cap = a.n;
  uint64_t* stamps = a.stamps ? a.stamps + row * 16 : nullptr;
  STAMP(0);
  const float* lg = a.logits + (int64_t)row * a.ld;
  for (int i = threadIdx.x; i < a.n; i += NT) sm.p[i] = lg[i];
  __syncthreads();
  if (threadIdx.x == 0 && a.forbid >= 0 && a.forbid < a.n) sm.p[a.forbid] = -__builtin_inff();
  __syncthreads();
  int status;
  const int id = sample_block<NT>(sm, a.n, a.temperature, a.top_p, a.top_k,
                              a.keys ? a.keys + row * 8 : nullptr, a.draws ? a.draws[row] : 0,
                              a.keys == nullptr, a.dbg ? a.dbg + row * 2 : nullptr, &status, stamps);
  if (threadIdx.x == 0) a.out[row] = status ? status : id;
}

void launch_sample_rows(const SampleRowArgs& a, int rows, hipStream_t st) {
  if (a.n > kSampleMaxN) {
    // the LDS carve of k_sample_rows_wide holds no row, keys or list
    const size_t lds = smem_bytes<kSampleThreads>(0) - kSampleMaxSorted * 12;
    RT_LAUNCH(k_sample_rows_wide, dim3(rows), dim3(kSampleThreads), lds, st, a);
    return;
  }
  RT_LAUNCH(k_sample_rows, dim3(rows), dim3(kSampleThreads), smem_bytes<kSampleThreads>(a.n), st, a);
}

// ---------------------------------------------------------------------------------------
// Phase controller: one workgroup per step row that carries logits.
// ---------------------------------------------------------------------------------------
__device__ inline float load_logit(const AdvanceArgs& a, const float* lg, int i) {
  float v = lg[i];
  for (int p = 1; p < a.n_part; ++p) v += lg[p * a.part_stride + i];
  return v;
}

// The row's logits into LDS: four elements per round with all their partial-slab loads issued
// before any add (each element still sums its slabs in order p = 0, 1, ...: same values)
template <int NT>
__device__ inline void load_logits_row(const AdvanceArgs& a, const float* lg, float* p, int n) {
  int i = threadIdx.x;
  for (; i + 3 * NT < n; i += 4 * NT) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = lg[i + u * NT];
    for (int q = 1; q < a.n_part; ++q) {
      float w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = lg[q * a.part_stride + i + u * NT];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += w[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) p[i + u * NT] = v[u];
  }
  for (; i < n; i += NT) p[i] = load_logit(a, lg, i);
}

// k_advance's preparation of a row for sample_block(prepped = true), with the row in registers
// instead of LDS round trips: element i = tid + k NT of thread tid (k < PT); every partial-slab
// load of the row is issued before the first add (each element sums its slabs in order p = 0, 1,
// ..., as load_logit does) and the last wave makes the draw (a ChaCha12 block) while they are in
// flight; block max; e = glibc expf(l - max) into p (the exact paths read it there); the real sum
// E of the row in f64 from per-thread partial sums (any order: its error, <= n 2^-53 E, is inside
// sample_cert's 2^-36 term); and, for top-k <= kFastK, the bound L and the candidates
// e >= L (1 - 2^-19) appended straight from the registers (the collect() of sample_block with all
// NW waves: each wave holds >= ceil(k / NW) elements >= its ceil(k / NW)-th largest thread-local
// maximum, so >= k elements are >= L). Leaves: p = e, fred[20] = L (0: no bound), ired[31] = the
// candidate count with the keys in keys[0, min(count, kFastCap)), fred[21] = r, dscan[12] = E.
// The row length N is a template parameter: every i < N test but the last element's folds away
// (with a runtime n the compiler hoisted seventeen lane masks per test into the kernel's preamble
// and spilled them, +5 us per launch). mask_eos: the last element (EOS, semantic rows) is -inf.
// The row's logits into registers, every partial-slab load issued before the first add (element i
// = tid + k NT sums its slabs in order p = 0, 1, ..., as load_logit does). Issued by k_advance
// before it reads the slot's control block. Indices past the row are clamped (never used).
template <int NT, int PT>
__device__ __attribute__((always_inline)) void advance_load_row(const AdvanceArgs& a, const float* lg, float* v) {
  const int last = a.ld - 1, tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < PT; ++k) v[k] = lg[min(tid + k * NT, last)];
  if (a.n_part == 2) {
    float w[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) w[k] = lg[a.part_stride + min(tid + k * NT, last)];
#pragma unroll
    for (int k = 0; k < PT; ++k) v[k] += w[k];
  } else if (a.n_part == 4) {
    float w[3][PT];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int k = 0; k < PT; ++k) w[q][k] = lg[(q + 1) * a.part_stride + min(tid + k * NT, last)];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int k = 0; k < PT; ++k) v[k] += w[q][k];
  } else {
    for (int q = 1; q < a.n_part; ++q)
#pragma unroll
      for (int k = 0; k < PT; ++k) v[k] += lg[q * a.part_stride + min(tid + k * NT, last)];
  }
}

template <int NT, int N, int PT>
__device__ __attribute__((always_inline)) void advance_prep(const float* raw, const SampleSmem& sm, bool mask_eos,
                                                            int top_k, const uint32_t* key, uint64_t draw,
                                                            uint32_t* blk, uint64_t* blk_id, uint64_t* stamps) {
  constexpr int NW = NT / 64, n = N;
  static_assert(PT * NT >= N, "row registers");
  const int masked = mask_eos ? N - 1 : -1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float v[PT];
#pragma unroll
  for (int k = 0; k < PT; ++k) v[k] = raw[k];
  if (tid == NT - 64) sm.fred[21] = draw_cached(key, draw, blk, blk_id);
  if (tid < 32) sm.etab[tid] = exp2_tab(tid);
  if (tid == 0) sm.ired[31] = 0;
  float mx = -__builtin_inff();
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int i = tid + k * NT;
    if (i == masked) v[k] = -__builtin_inff();
    if (i < n) mx = fmaxf(mx, v[k]);
  }
  STAMP(1);
  mx = block_max<NT>(mx, sm.fred);  // its barriers also order etab / ired[31] / fred[21]
  STAMP(3);
  const uint64_t* et = sm.etab;
  auto tab = [et](int j) { return et[j]; };
  double es = 0.0;
  float lm = -1.0f;  // every e >= 0
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int i = tid + k * NT;
    if (i < n) {
      const float e = glibc_expf_t(v[k] - mx, tab);
      v[k] = e;
      sm.p[i] = e;
      es += (double)e;
      lm = fmaxf(lm, e);
    }
  }
  STAMP(4);
  es = readlane_d(wave_incl_scan_d(es), 63);
  const bool want = top_k > 0 && top_k < n && top_k <= kFastK;
  if (want) {
    const int kw = (top_k + NW - 1) / NW;
    int gt = 0, ge = 0;
#pragma unroll 16
    for (int j = 0; j < 64; ++j) {
      const float o = readlane_f(lm, j);
      gt += o > lm ? 1 : 0;
      ge += o >= lm ? 1 : 0;
    }
    const uint64_t selm = __ballot(gt < kw && kw <= ge);
    const float vw = readlane_f(lm, __builtin_ctzll(selm));
    if (lane == 0) sm.fred[8 + wave] = vw;
  }
  if (lane == 0) sm.dscan[wave] = es;
  STAMP(5);
  __syncthreads();
  STAMP(6);
  float L = 0.0f;
  if (want) {
    L = sm.fred[8];
#pragma unroll
    for (int w = 1; w < NW; ++w) L = fminf(L, sm.fred[8 + w]);
  }
  if (L > 0.0f) {
    // the wave's candidates counted first (ballots only), ONE LDS atomic per wave reserves their
    // slots, then they are written in the same k-major order (the list's order across waves was
    // the atomics' order before as well; its consumers do not depend on it)
    const float T = L * (1.0f - 0x1p-19f);
    uint64_t bms[PT];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int i = tid + k * NT;
      bms[k] = __ballot(i < n && v[k] >= T);
      tot += __popcll(bms[k]);
    }
    if (tot) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&sm.ired[31], tot);
      base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const int i = tid + k * NT;
        const int off = base + __popcll(bms[k] & ((1ull << lane) - 1ull));
        if (((bms[k] >> lane) & 1ull) && off < kFastCap)
          sm.keys[off] = ((uint64_t)__builtin_bit_cast(uint32_t, v[k]) << 32) | (uint32_t)i;
        base += __popcll(bms[k]);
      }
    }
  }
  // A tight rigorous bound on S (the crude one put 1.4 % of the bench's rows' draws inside a
  // cumulative's uncertainty band -- and a row that falls back to the exact sum holds the whole
  // launch, ~1 step in 3): S = sum e_i in index order, addition i (i >= 1) rounds by at most half
  // an ulp of its result s_i, and s_i <= P_i (1 + eps0) with P_i the real prefix sum and eps0 the
  // crude bound, so |S - E| <= B = sum_i 2^(floor(log2(P_i (1 + eps0))) - 24) (the f32 half-ulp at
  // that binade, >= 2^-150); B is typically ~5x below n 2^-23 E. Threads take contiguous chunks of
  // p; the index list region (unused on this path) holds the f64 partials.
  STAMP(14);
  double E = sm.dscan[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) E += sm.dscan[w];
  {
    double* dbuf = (double*)sm.list;  // 2 NT doubles
    constexpr int C = (N + NT - 1) / NT, G = NT / 64;
    const int b = min(n, tid * C), e = min(n, b + C);
    double ts = 0.0;
    for (int i = b; i < e; ++i) ts += (double)sm.p[i];
    dbuf[tid] = ts;
    __syncthreads();
    if (tid < 64) {  // exclusive prefix of the chunk sums
      double g[G], acc = 0.0;
#pragma unroll
      for (int q = 0; q < G; ++q) {
        g[q] = dbuf[lane * G + q];
        acc += g[q];
      }
      double run = wave_incl_scan_d(acc) - acc;
#pragma unroll
      for (int q = 0; q < G; ++q) {
        dbuf[NT + lane * G + q] = run;
        run += g[q];
      }
    }
    __syncthreads();
    const double up = 1.0 + crude_sum_eps(n) + 0x1p-30;
    double P = dbuf[NT + tid], bp = 0.0;
    for (int i = b; i < e; ++i) {
      P += (double)sm.p[i];
      if (i > 0) {
        const int k = max((int)((__builtin_bit_cast(uint64_t, P * up) >> 52) & 0x7FF) - 1023, -126);
        bp += __builtin_bit_cast(double, (uint64_t)(k - 24 + 1023) << 52);
      }
    }
    dbuf[tid] = bp;
    __syncthreads();
    if (tid < 64) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < G; ++q) acc += dbuf[lane * G + q];
      const double B = readlane_d(wave_incl_scan_d(acc), 63);
      if (tid == 0) sm.dscan[13] = B / E * (1.0 + 0x1p-30) + 0x1p-36;
    }
  }
  if (tid == 0) {
    sm.dscan[12] = E;
    sm.fred[20] = L;
  }
  __syncthreads();
  STAMP(10);
}

__device__ __attribute__((always_inline)) void advance_body(const AdvanceArgs& a, char* smem) {
  constexpr int NT = kSampleThreads;
  const int row = blockIdx.x;
  uint64_t* stamps = a.stamps ? a.stamps + row * 16 : nullptr;
  STAMP(0);
  // the row's logits are requested first: they do not depend on the control block
  constexpr int NS = RWKVTTS_EOS_TOKEN + 1, PT = (NS + NT - 1) / NT;
  const float* lg = a.logits + (int64_t)row * a.ld;
  float raw[PT];
  advance_load_row<NT, PT>(a, lg, raw);
  const int slot = a.row_slot[row];
  SlotCtrl* c = a.ctrl + slot;
  const int phase = c->phase;  // uniform (read by all threads before any write)
  __syncthreads();
  if (phase == kPhDone) return;
  if (phase == kPhGFeed) {  // this step fed g31+8196: its logits are unused (RnnOption::Last)
    if (threadIdx.x == 0) {
      c->next_token = RWKVTTS_TAG_1;
      // semantic_limit = min(max_tokens, 2048) may be 0 (normal_mode_inference.rs:316): the
      // TAG_1 forward that follows has no observable output then, so the request ends here
      c->phase = c->sem_limit > 0 ? kPhSemantic : kPhDone;
    }
    return;
  }
  // one prepared sampling call site for both phases (one inlined sample_block instance):
  // global rows [0, 4096), semantic rows [0, 8192] (j > 8192 and the tags are -inf in the reference)
  const bool glob = phase == kPhGlobal;
  const SampleSmem sm = carve<NT>(smem, NS);
  const bool eos_masked = !glob && (c->fixed || (c->mode == 1 && c->n_sem < c->hard_min));
  const int n = glob ? 4096 : NS, top_k = glob ? c->top_k_g : c->top_k_s;
  const uint32_t* key = glob ? c->gkey : c->skey;
  const uint64_t draw = glob ? c->gdraw : c->sdraw;
  // attempt 1 (zero-shot only): EOS drawn while the window rule does not stop the request ->
  // re-draw with EOS masked from the same logits and the next draw (zero_shot_inference.rs:287-297)
  int id = 0, status;
  uint64_t used = 1;
  bool stop = false, masked = eos_masked;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (glob) advance_prep<NT, 4096, PT>(raw, sm, false, top_k, key, draw + attempt, c->gblk, &c->gblk_id, stamps);
    else advance_prep<NT, NS, PT>(raw, sm, masked, top_k, key, draw + attempt, c->sblk, &c->sblk_id, stamps);
    id = sample_block<NT>(sm, n, 1.0f, 0.95f, top_k, key, draw + attempt, false, nullptr, &status, stamps,
                          a.cert != 0, true);
    used = attempt + 1;
    if (glob || id != RWKVTTS_EOS_TOKEN) break;
    if (c->mode == 0) {
      stop = true;
      break;
    }
    const int wl = c->win_len;
    const int non_eos = __builtin_popcount((uint32_t)c->win_bits & ((1u << wl) - 1u));
    const float ratio = wl > 0 ? (float)non_eos / (float)wl : 0.0f;
    if (wl >= 12 && ratio >= 0.7f) {
      stop = true;
      break;
    }
    masked = true;
    __syncthreads();  // every thread has read the row state before the re-draw rewrites it
  }
  STAMP(15);
  if (glob) {
    if (threadIdx.x == 0) {
      c->gdraw += 1;
      c->global_out[c->n_global++] = id;
      c->next_token = id + RWKVTTS_GLOBAL_TOKEN_OFFSET;
      if (c->n_global == RWKVTTS_N_GLOBAL) c->phase = kPhGFeed;
    }
    return;
  }
  if (threadIdx.x == 0) {
    c->sdraw += used;
    if (stop) {
      c->phase = kPhDone;
    } else {
      if (c->mode == 1) {
        c->win_bits = ((c->win_bits << 1) | (id != RWKVTTS_EOS_TOKEN ? 1 : 0)) & 0xFFF;
        if (c->win_len < 12) c->win_len++;
      }
      a.sem_out[(int64_t)slot * RWKVTTS_SEMANTIC_LIMIT + c->n_sem] = id;
      c->n_sem++;
      c->next_token = id;
      if (c->n_sem >= c->sem_limit) c->phase = kPhDone;
    }
  }
}

__global__ __launch_bounds__(kSampleThreads, 2) void k_advance(AdvanceArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tl_begin(a.tl);
  advance_body(a, smem);
  tl_end(a.tl);
}

int launch_advance(const AdvanceArgs& a0, hipStream_t st, int cert) {
  AdvanceArgs a = a0;
  a.cert = cert;  // 0: always walk the exact sequential sum (RWKVTTS_FORM_EXACT_SAMPLER)
  RT_LAUNCH(k_advance, dim3(a.n_rows), dim3(kSampleThreads), smem_bytes<kSampleThreads>(RWKVTTS_EOS_TOKEN + 1),
                     st, a);
  return a.n_rows;
}

}  // namespace rwkvtts
