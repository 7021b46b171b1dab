// synth.cpp -- deterministic synthetic RWKV-7 weights and the rand 0.8 StdRng
// seed derivation used by the C ABI. Counter-based (splitmix64 of seed/tensor/index) so the
// Python packer (rwkvtts/weights.py) regenerates the identical blob.
#include <math.h>
#include <string.h>

#include <thread>
#include <vector>

#include "common.h"

namespace rwkvtts {

static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// approximately N(0,1): Irwin-Hall of four 16-bit uniforms, exact in double.
static inline double synth_normal(uint64_t h) {
  double s = (double)(h & 0xFFFF) + (double)((h >> 16) & 0xFFFF) + (double)((h >> 32) & 0xFFFF) +
             (double)((h >> 48) & 0xFFFF);
  return (s / 65536.0 - 2.0) * 1.7320508075688772;
}
static inline double synth_uniform(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

// value of element `i` of tensor `t` (layer -1 = global)
static inline double synth_value(const rwkvtts_dims* d, int layer, int t, uint64_t i, uint64_t key) {
  const uint64_t h = splitmix64(key ^ i);
  (void)d;
  if (layer < 0) {
    switch (t) {
      case RWKVTTS_T_EMB: return synth_normal(h) * 0.5;
      case RWKVTTS_T_HEAD: return synth_normal(h) * 0.05;
      case RWKVTTS_T_LN0_W: case RWKVTTS_T_LNOUT_W: return 1.0 + 0.1 * synth_normal(h);
      default: return 0.02 * synth_normal(h);  // biases
    }
  }
  switch (t) {
    case RWKVTTS_L_LN1_W: case RWKVTTS_L_LN2_W: return 1.0 + 0.1 * synth_normal(h);
    case RWKVTTS_L_LN1_B: case RWKVTTS_L_LN2_B: case RWKVTTS_L_LNX_B: return 0.02 * synth_normal(h);
    case RWKVTTS_L_XR: case RWKVTTS_L_XW: case RWKVTTS_L_XK: case RWKVTTS_L_XV:
    case RWKVTTS_L_XA: case RWKVTTS_L_XG: case RWKVTTS_L_FFN_XK: return synth_uniform(h);
    case RWKVTTS_L_W0: return -4.0 + 6.0 * synth_uniform(h);  // decay in (0.55, 0.99)
    case RWKVTTS_L_A0: case RWKVTTS_L_V0: return -1.0 + 2.0 * synth_uniform(h);
    case RWKVTTS_L_KK: case RWKVTTS_L_KA: return 0.5 + 0.5 * synth_uniform(h);
    case RWKVTTS_L_RK: return 0.1 * synth_normal(h);
    case RWKVTTS_L_LNX_W: return 0.5 + 0.5 * synth_uniform(h);
    default: return 0.02 * synth_normal(h);  // every matrix
  }
}

static void fill_tensor(const rwkvtts_dims* d, int dtype, uint64_t seed, int layer, int t,
                        uint8_t* base) {
  int64_t rows, cols;
  const int is_mat = rwkvtts_tensor_shape(d, layer, t, &rows, &cols);
  const uint64_t key = splitmix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)((layer + 1) * 64 + t + 1)));
  const int64_t n = rows * cols;
  const int zero_v = (layer == 0) && (t == RWKVTTS_L_V0 || t == RWKVTTS_L_V1T || t == RWKVTTS_L_V2T);
  if (is_mat) {
    uint16_t* p = (uint16_t*)base;
    for (int64_t i = 0; i < n; ++i) {
      float f = zero_v ? 0.0f : (float)synth_value(d, layer, t, (uint64_t)i, key);
      if (dtype == RWKVTTS_DTYPE_BF16) {
        p[i] = f32_to_bf16(f);
      } else {  // f16, round-to-nearest-even (values are small; no overflow)
        uint32_t u = as_u32(f);
        uint32_t s = (u >> 16) & 0x8000u;
        int e = (int)((u >> 23) & 0xFF) - 127 + 15;
        uint32_t m = u & 0x7FFFFFu;
        uint16_t h;
        if (e <= 0) {
          if (e < -10) {
            h = (uint16_t)s;
          } else {
            m |= 0x800000u;
            int shift = 14 - e;
            uint32_t hm = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
            if (rem > half || (rem == half && (hm & 1))) hm++;
            h = (uint16_t)(s | hm);
          }
        } else {
          uint32_t hm = m >> 13, rem = m & 0x1FFF;
          uint32_t hv = ((uint32_t)e << 10) | hm;
          if (rem > 0x1000 || (rem == 0x1000 && (hm & 1))) hv++;
          h = (uint16_t)(s | hv);
        }
        p[i] = h;
      }
    }
  } else {
    float* p = (float*)base;
    for (int64_t i = 0; i < n; ++i) p[i] = zero_v ? 0.0f : (float)synth_value(d, layer, t, (uint64_t)i, key);
  }
}

}  // namespace rwkvtts

using namespace rwkvtts;

extern "C" int rwkvtts_synth_weights(const rwkvtts_dims* d, int dtype, uint64_t seed, void* out) {
  RT_CHECK(d && out, RWKVTTS_EINVAL, "synth_weights: null argument");
  RT_CHECK(dtype == RWKVTTS_DTYPE_BF16 || dtype == RWKVTTS_DTYPE_F16, RWKVTTS_EINVAL, "bad dtype");
  uint8_t* blob = (uint8_t*)out;
  memset(blob, 0, 256);
  rwkvtts_blob_header* h = (rwkvtts_blob_header*)blob;
  h->magic = RWKVTTS_BLOB_MAGIC;
  h->version = 1;
  h->dtype = dtype;
  h->dims = *d;
  struct Job { int layer, t; };
  std::vector<Job> jobs;
  for (int t = 0; t < RWKVTTS_T_GLOBAL_COUNT; ++t) jobs.push_back({-1, t});
  for (int l = 0; l < d->n_layer; ++l)
    for (int t = 0; t < RWKVTTS_L_COUNT; ++t) jobs.push_back({l, t});
  unsigned nt = std::thread::hardware_concurrency();
  if (nt == 0) nt = 4;
  if (nt > 16) nt = 16;
  std::vector<std::thread> th;
  for (unsigned w = 0; w < nt; ++w) {
    th.emplace_back([&, w]() {
      for (size_t j = w; j < jobs.size(); j += nt)
        fill_tensor(d, dtype, seed, jobs[j].layer, jobs[j].t,
                    blob + rwkvtts_tensor_offset(d, jobs[j].layer, jobs[j].t));
    });
  }
  for (auto& t : th) t.join();
  return RWKVTTS_OK;
}

extern "C" void rwkvtts_rng_seed_from_u64(uint64_t state, rwkvtts_rng* r) {
  // rand_core 0.6.4 SeedableRng::seed_from_u64: PCG32 fill of the 32-byte ChaCha12 key.
  const uint64_t MUL = 6364136223846793005ull, INC = 11634580456473284103ull;
  for (int i = 0; i < 8; ++i) {
    state = state * MUL + INC;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    r->key[i] = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
  }
  r->draw_index = 0;
}

#include "exact_math.h"
// Host self-test hook: the exact expf the GPU sampler runs (tests/test_expf_exact.py).
extern "C" float rwkvtts_debug_expf(float x) { return rwkvtts::glibc_expf(x); }
