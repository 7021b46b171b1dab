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
// Limitation (generic API only): top-p over more than 4096 positive probabilities (top_k == 0
// or > 4096) is rejected; temperature != 1 uses a double-precision powf (not glibc's).
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

__device__ inline float draw_f32(const uint32_t* key, uint64_t index) {
  return (float)(chacha12_word(key, index) >> 8) * (1.0f / 16777216.0f);
}

// Shared-memory layout of one sampling workgroup (256 threads).
struct SampleSmem {
  float* p;         // [n]
  uint64_t* keys;   // [kSampleMaxSorted]
  int* list;        // [kSampleMaxSorted] positive indices in index order
  int* hist;        // [256]
  int* scan;        // [257]
  float* fred;      // [8]
  int* ired;        // [8]
};

__device__ inline float block_max(float v, float* fred) {
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(fred[0], fred[1]), fmaxf(fred[2], fred[3]));
}

// exclusive scan of one int per thread (256 threads); returns this thread's offset, total in *tot
__device__ inline int block_excl_scan(int v, int* scan, int* tot) {
  __syncthreads();
  scan[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < 256; ++i) {
      const int c = scan[i];
      scan[i] = acc;
      acc += c;
    }
    scan[256] = acc;
  }
  __syncthreads();
  *tot = scan[256];
  return scan[threadIdx.x];
}

// compact indices with p > 0 into list (index order); returns count (may exceed capacity:
// then list is incomplete and callers fall back to a scan of p).
__device__ int compact_positive(const SampleSmem& sm, int n) {
  const int chunk = (n + 255) / 256;
  const int b = threadIdx.x * chunk, e = min(n, b + chunk);
  int cnt = 0;
  for (int i = b; i < e; ++i) cnt += sm.p[i] > 0.0f;
  int tot;
  int off = block_excl_scan(cnt, sm.scan, &tot);
  for (int i = b; i < e; ++i)
    if (sm.p[i] > 0.0f) {
      if (off < kSampleMaxSorted) sm.list[off] = i;
      ++off;
    }
  __syncthreads();
  return tot;
}

// index-order sequential f32 sum of p (only positive entries contribute: +0 adds are exact)
__device__ float serial_sum_positive(const SampleSmem& sm, int n, int npos) {
  float s = 0.0f;
  if (npos <= kSampleMaxSorted) {
    for (int q = 0; q < npos; ++q) s += sm.p[sm.list[q]];
  } else {
    for (int i = 0; i < n; ++i) s += sm.p[i];
  }
  return s;
}

// The sampler. p holds the (masked) logits on entry. Returns the index in every thread.
// status: 0 ok, RWKVTTS_EUNSUPPORTED for the documented limitation.
__device__ int sample_block(const SampleSmem& sm, int n, float temperature, float top_p,
                            int top_k, const uint32_t* key, uint64_t draw, bool fixed42,
                            float* dbg, int* status) {
  const int tid = threadIdx.x;
  *status = 0;
  if (n == 0) return 0;
  // (2) softmax: max, exp, sequential sum, divide
  float mx = -__builtin_inff();
  for (int i = tid; i < n; i += 256) mx = fmaxf(mx, sm.p[i]);
  mx = block_max(mx, sm.fred);
  for (int i = tid; i < n; i += 256) sm.p[i] = glibc_expf(sm.p[i] - mx);
  __syncthreads();
  if (tid == 0) {
    float s = 0.0f;
    int i = 0;
    for (; i + 4 <= n; i += 4) {
      const float4_ q = *(const float4_*)(sm.p + i);
      s += q[0];
      s += q[1];
      s += q[2];
      s += q[3];
    }
    for (; i < n; ++i) s += sm.p[i];
    sm.fred[4] = s;
  }
  __syncthreads();
  const float sum = sm.fred[4];
  if (sum > 0.0f)
    for (int i = tid; i < n; i += 256) sm.p[i] = sm.p[i] / sum;
  __syncthreads();
  // (3) top-k: radix-select the k-th largest (p desc, index asc)
  if (top_k > 0 && top_k < n) {
    uint32_t prefix = 0, mask = 0;
    int remaining = top_k;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      sm.hist[tid] = 0;
      __syncthreads();
      for (int i = tid; i < n; i += 256) {
        const uint32_t u = __builtin_bit_cast(uint32_t, sm.p[i]);
        if ((u & mask) == prefix) atomicAdd(&sm.hist[(u >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int acc = 0, D = 0;
        for (int d = 255; d >= 0; --d) {
          if (acc + sm.hist[d] >= remaining) { D = d; break; }
          acc += sm.hist[d];
        }
        sm.ired[0] = D;
        sm.ired[1] = remaining - acc;
      }
      __syncthreads();
      prefix |= (uint32_t)sm.ired[0] << shift;
      mask |= 0xFFu << shift;
      remaining = sm.ired[1];
      __syncthreads();
    }
    const float t = __builtin_bit_cast(float, prefix);
    const int need_eq = remaining;
    const int chunk = (n + 255) / 256;
    const int b = tid * chunk, e = min(n, b + chunk);
    int cnt = 0;
    for (int i = b; i < e; ++i) cnt += (sm.p[i] == t);
    int tot;
    int rank = block_excl_scan(cnt, sm.scan, &tot);
    for (int i = b; i < e; ++i) {
      const float v = sm.p[i];
      if (v < t) {
        sm.p[i] = 0.0f;
      } else if (v == t) {
        if (rank >= need_eq) sm.p[i] = 0.0f;
        ++rank;
      }
    }
    __syncthreads();
  }
  int npos = compact_positive(sm, n);
  // (4) top-p
  if (top_p < 1.0f) {
    if (npos > kSampleMaxSorted) {
      *status = RWKVTTS_EUNSUPPORTED;
      return 0;
    }
    int M = 1;
    while (M < npos) M <<= 1;
    for (int q = tid; q < M; q += 256)
      sm.keys[q] = q < npos ? (((uint64_t)__builtin_bit_cast(uint32_t, sm.p[sm.list[q]]) << 32) |
                               (uint64_t)(0xFFFFFFFFu - (uint32_t)sm.list[q]))
                            : 0ull;
    __syncthreads();
    for (int k = 2; k <= M; k <<= 1) {  // bitonic sort, descending
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int q = tid; q < M; q += 256) {
          const int ixj = q ^ j;
          if (ixj > q) {
            const uint64_t A = sm.keys[q], B = sm.keys[ixj];
            const bool desc = (q & k) == 0;
            if (desc ? (A < B) : (A > B)) { sm.keys[q] = B; sm.keys[ixj] = A; }
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0) {
      float cum = 0.0f, cutoff = 0.0f;
      int found = 0;
      for (int q = 0; q < npos; ++q) {
        const float pv = __builtin_bit_cast(float, (uint32_t)(sm.keys[q] >> 32));
        cum += pv;
        if (cum >= top_p) { found = 1; cutoff = pv; break; }
      }
      if (!found && npos < n && cum >= top_p) { found = 1; cutoff = 0.0f; }  // (unreachable for top_p > 0)
      if (!found && npos == 0 && 0.0f >= top_p) { found = 1; cutoff = 0.0f; }
      sm.fred[5] = cutoff;
      sm.ired[2] = found;
    }
    __syncthreads();
    if (sm.ired[2]) {
      const float cutoff = sm.fred[5];
      for (int i = tid; i < n; i += 256)
        if (sm.p[i] < cutoff) sm.p[i] = 0.0f;
      __syncthreads();
      if (top_p > 0.0f) {
        npos = compact_positive(sm, n);
        sm.ired[3] = 0;
        __syncthreads();
        int c = 0;
        for (int i = tid; i < n; i += 256) c += (sm.p[i] == cutoff);
        if (c) atomicAdd(&sm.ired[3], c);
        __syncthreads();
        if (tid == 0) {
          const float cur = serial_sum_positive(sm, n, npos);
          sm.ired[4] = 0;
          if (cur < top_p && sm.ired[3] > 0) {
            sm.fred[6] = (top_p - cur) / (float)sm.ired[3];
            sm.ired[4] = 1;
          }
        }
        __syncthreads();
        if (sm.ired[4]) {
          const float adj = sm.fred[6];
          for (int i = tid; i < n; i += 256)
            if (sm.p[i] == cutoff) sm.p[i] = cutoff + adj;
          __syncthreads();
        }
      }
    }
  }
  npos = compact_positive(sm, n);
  // (5) temperature
  if (temperature != 1.0f && temperature > 0.0f) {
    const float tinv = 1.0f / temperature;
    for (int i = tid; i < n; i += 256) {
      const float v = sm.p[i];
      if (v > 0.0f) sm.p[i] = (float)exp2(log2((double)v) * (double)tinv);
    }
    __syncthreads();
    npos = compact_positive(sm, n);
    if (tid == 0) sm.fred[7] = serial_sum_positive(sm, n, npos);
    __syncthreads();
    const float s2 = sm.fred[7];
    if (s2 > 0.0f)
      for (int i = tid; i < n; i += 256) sm.p[i] = sm.p[i] / s2;
    __syncthreads();
  }
  // (6) multinomial
  if (tid == 0) {
    uint32_t k42[8];
    if (fixed42) {
      uint64_t st = 42;
      const uint64_t MUL = 6364136223846793005ull, INC = 11634580456473284103ull;
      for (int i = 0; i < 8; ++i) {
        st = st * MUL + INC;
        const uint32_t xs = (uint32_t)(((st >> 18) ^ st) >> 27);
        const uint32_t rot = (uint32_t)(st >> 59);
        k42[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
      }
    }
    const float r = fixed42 ? draw_f32(k42, 0) : draw_f32(key, draw);
    int ret = -1;
    if (r <= sm.p[0]) {
      ret = 0;
    } else if (npos <= kSampleMaxSorted) {
      float cum = 0.0f;
      for (int q = 0; q < npos; ++q) {
        cum += sm.p[sm.list[q]];
        if (r <= cum) { ret = sm.list[q]; break; }
      }
      if (ret < 0 && npos > 0) ret = sm.list[npos - 1];
    } else {
      float cum = 0.0f;
      for (int i = 0; i < n; ++i) {
        cum += sm.p[i];
        if (r <= cum) { ret = i; break; }
      }
      if (ret < 0)
        for (int i = n - 1; i >= 0; --i)
          if (sm.p[i] > 0.0f) { ret = i; break; }
    }
    if (ret < 0) ret = 0;
    sm.ired[5] = ret;
    if (dbg) { dbg[0] = sum; dbg[1] = r; }
  }
  __syncthreads();
  return sm.ired[5];
}

__device__ SampleSmem carve(char* base, int n) {
  SampleSmem sm;
  const int npad = (n + 3) & ~3;
  sm.p = (float*)base;
  sm.keys = (uint64_t*)(base + (int64_t)npad * 4);
  sm.list = (int*)(sm.keys + kSampleMaxSorted);
  sm.hist = sm.list + kSampleMaxSorted;
  sm.scan = sm.hist + 256;
  sm.fred = (float*)(sm.scan + 260);
  sm.ired = (int*)(sm.fred + 8);
  return sm;
}
inline size_t smem_bytes(int n) {
  const int npad = (n + 3) & ~3;
  return (size_t)npad * 4 + kSampleMaxSorted * 8 + kSampleMaxSorted * 4 + 256 * 4 + 260 * 4 + 8 * 4 + 8 * 4;
}

__global__ __launch_bounds__(256) void k_sample_rows(SampleRowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SampleSmem sm = carve(smem, a.n);
  const int row = blockIdx.x;
  const float* lg = a.logits + (int64_t)row * a.ld;
  for (int i = threadIdx.x; i < a.n; i += 256) sm.p[i] = lg[i];
  __syncthreads();
  if (threadIdx.x == 0 && a.forbid >= 0 && a.forbid < a.n) sm.p[a.forbid] = -__builtin_inff();
  __syncthreads();
  int status;
  const int id = sample_block(sm, a.n, a.temperature, a.top_p, a.top_k,
                              a.keys ? a.keys + row * 8 : nullptr, a.draws ? a.draws[row] : 0,
                              a.keys == nullptr, a.dbg ? a.dbg + row * 2 : nullptr, &status);
  if (threadIdx.x == 0) a.out[row] = status ? status : id;
}

void launch_sample_rows(const SampleRowArgs& a, int rows, hipStream_t st) {
  hipLaunchKernelGGL(k_sample_rows, dim3(rows), dim3(256), smem_bytes(a.n), st, a);
}

// ---------------------------------------------------------------------------------------
// Phase controller: one workgroup per step row that carries logits.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_advance(AdvanceArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int row = blockIdx.x;
  const int slot = a.row_slot[row];
  SlotCtrl* c = a.ctrl + slot;
  const int phase = c->phase;  // uniform (read by all threads before any write)
  __syncthreads();
  if (phase == kPhDone) return;
  if (phase == kPhGFeed) {  // this step fed g31+8196: its logits are unused (RnnOption::Last)
    if (threadIdx.x == 0) {
      c->next_token = RWKVTTS_TAG_1;
      c->phase = kPhSemantic;
    }
    return;
  }
  const float* lg = a.logits + (int64_t)row * a.ld;
  if (phase == kPhGlobal) {
    const SampleSmem sm = carve(smem, 4096);
    for (int i = threadIdx.x; i < 4096; i += 256) sm.p[i] = lg[i];
    __syncthreads();
    int status;
    const int id = sample_block(sm, 4096, 1.0f, 0.95f, c->top_k_g, c->gkey, c->gdraw, false,
                                nullptr, &status);
    if (threadIdx.x == 0) {
      c->gdraw += 1;
      c->global_out[c->n_global++] = id;
      c->next_token = id + RWKVTTS_GLOBAL_TOKEN_OFFSET;
      if (c->n_global == RWKVTTS_N_GLOBAL) c->phase = kPhGFeed;
    }
    return;
  }
  // semantic: rows [0, 8192] (j > 8192 and the tags are -inf in the reference)
  constexpr int NS = RWKVTTS_EOS_TOKEN + 1;
  const SampleSmem sm = carve(smem, NS);
  const bool eos_masked = c->fixed || (c->mode == 1 && c->n_sem < c->hard_min);
  for (int i = threadIdx.x; i < NS; i += 256) sm.p[i] = lg[i];
  __syncthreads();
  if (threadIdx.x == 0 && eos_masked) sm.p[RWKVTTS_EOS_TOKEN] = -__builtin_inff();
  __syncthreads();
  int status;
  int id = sample_block(sm, NS, 1.0f, 0.95f, c->top_k_s, c->skey, c->sdraw, false, nullptr, &status);
  uint64_t used = 1;
  bool stop = false;
  if (id == RWKVTTS_EOS_TOKEN) {
    if (c->mode == 0) {
      stop = true;
    } else {
      const int wl = c->win_len;
      const int non_eos = __builtin_popcount((uint32_t)c->win_bits & ((1u << wl) - 1u));
      const float ratio = wl > 0 ? (float)non_eos / (float)wl : 0.0f;
      if (wl >= 12 && ratio >= 0.7f) {
        stop = true;
      } else {  // re-draw with EOS masked from the same logits (zero_shot_inference.rs:287-297)
        for (int i = threadIdx.x; i < NS; i += 256) sm.p[i] = lg[i];
        __syncthreads();
        if (threadIdx.x == 0) sm.p[RWKVTTS_EOS_TOKEN] = -__builtin_inff();
        __syncthreads();
        id = sample_block(sm, NS, 1.0f, 0.95f, c->top_k_s, c->skey, c->sdraw + 1, false, nullptr,
                          &status);
        used = 2;
      }
    }
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

void launch_advance(const AdvanceArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_advance, dim3(a.n_rows), dim3(256), smem_bytes(RWKVTTS_EOS_TOKEN + 1), st, a);
}

}  // namespace rwkvtts
