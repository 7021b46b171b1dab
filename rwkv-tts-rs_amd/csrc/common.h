// common.h -- shared host/device helpers for the MI355X (gfx950) RWKV-TTS hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string>

#include "../../include/rwkvtts.h"

namespace rwkvtts {

// ---- error handling across the C ABI -------------------------------------------------
void set_error(const std::string& msg);
#define RT_HIP(expr)                                                                  \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      ::rwkvtts::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" + \
                           __FILE__ + ":" + std::to_string(__LINE__));               \
      return RWKVTTS_EHIP;                                                           \
    }                                                                                \
  } while (0)
#define RT_CHECK(cond, code, msg)     \
  do {                                \
    if (!(cond)) {                    \
      ::rwkvtts::set_error(msg);      \
      return code;                    \
    }                                 \
  } while (0)

// ---- numeric helpers -------------------------------------------------------------------
typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef float float4_ __attribute__((ext_vector_type(4)));

__host__ __device__ inline float as_f32(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ inline uint32_t as_u32(float f) { return __builtin_bit_cast(uint32_t, f); }
__host__ __device__ inline float bf16_to_f32(uint16_t h) { return as_f32((uint32_t)h << 16); }
// round-to-nearest-even f32 -> bf16 (finite inputs)
__host__ __device__ inline uint16_t f32_to_bf16(float f) {
  uint32_t u = as_u32(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__host__ __device__ inline float f16_to_f32(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023, u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {
      int sh = 0;
      while (!(m & 1024)) { m <<= 1; ++sh; }
      m &= 1023;
      u = s | ((uint32_t)(127 - 15 - sh + 1) << 23) | (m << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 112) << 23) | (m << 13);
  }
  return as_f32(u);
}

// 16-bit weight / activation-plane formats: bf16 (default) or IEEE f16 (fp16 checkpoints, the
// reference's web-rwkv numerics). Device conversions, f32 -> 16 bit round-to-nearest-even.
__device__ inline float h16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ inline uint16_t f32_to_h16(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
__device__ inline float w16_to_f32(uint16_t v, bool f16) { return f16 ? h16_to_f32(v) : bf16_to_f32(v); }
// device f32 -> bf16 by the hardware converter (v_cvt_pk_bf16_f32, round-to-nearest-even: the
// same bits as f32_to_bf16 for every finite input)
__device__ inline uint16_t f32_to_bf16_hw(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ inline uint16_t f32_to_w16(float x, bool f16) { return f16 ? f32_to_h16(x) : f32_to_bf16_hw(x); }

// x = hi + lo split of two floats into packed 16-bit pairs (hi = RNE(x), lo = RNE(x - hi)):
// one packed convert per plane.
typedef float float2_ __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_ __attribute__((ext_vector_type(2)));
template <bool F16>
__device__ inline void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  if constexpr (F16) {
    const f16x2_ h = __builtin_convertvector((float2_){a, b}, f16x2_);
    const float2_ hf = __builtin_convertvector(h, float2_);
    hi = __builtin_bit_cast(uint32_t, h);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_){a, b} - hf, f16x2_));
  } else {
    const bf16x2_ h = __builtin_convertvector((float2_){a, b}, bf16x2_);
    const uint32_t hb = __builtin_bit_cast(uint32_t, h);
    const float2_ hf = {__builtin_bit_cast(float, hb << 16), __builtin_bit_cast(float, hb & 0xFFFF0000u)};
    hi = hb;
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_){a, b} - hf, bf16x2_));
  }
}

inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// Write-through (sc1) vector stores: the line leaves the XCD's L2 at once instead of staying
// dirty until the end-of-kernel write-back, which the NEXT launch waits for (MI355X_MICROARCH.md
// price list, row boundary: + B / 6 TB/s for B dirty bytes). Buffer stores with cpol sc1.
__device__ inline __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ inline void store_wt(__amdgpu_buffer_rsrc_t r, int off_bytes, float4_ v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_, v), r, off_bytes, 0, 16);
}
__device__ inline void store_wt(__amdgpu_buffer_rsrc_t r, int off_bytes, uint2 v) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64((u32x2_){v.x, v.y}, r, off_bytes, 0, 16);
}
__device__ inline void store_wt(__amdgpu_buffer_rsrc_t r, int off_bytes, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off_bytes, 0, 16);
}

// Launch timeline: start of the launch's first workgroup and end of its last one in
// s_memrealtime ticks (100 MHz, one clock for every CU); ends are max-reduced over 64 slots to keep
// the atomics off one address. Slot layout per launch: [0] start, [2..65] ends. The slot pointer
// is null unless the engine records launch times: the debug timeline (RWKVTTS_TIMELINE, make TL=1)
// or the in-graph kernel timing the bench samples (rwkvtts_set_profiling(e, 2)); with a null slot
// a hook is one uniform branch.
constexpr int kTlStride = 66;
__device__ inline int tl_block() { return (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; }
__device__ inline void tl_begin(unsigned long long* tl) {
  if (tl && threadIdx.x == 0 && tl_block() == 0) tl[0] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
}
__device__ inline void tl_end(unsigned long long* tl) {
  if (tl && threadIdx.x == 0) atomicMax(&tl[2 + (tl_block() & 63)], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// Kernel launches of the LM / sampler path go through RT_LAUNCH. While the engine has a
// profiling window open (Engine::prof_begin .. prof_end) the launch carries the window's HIP
// events (hipExtLaunchKernelGGL): they are stamped by the kernel's own dispatch packet, so the
// elapsed time is the kernel's execution interval (what rocprofv3 --kernel-trace reports), not
// the queue gap an event marker before it would add. The first launch of a window stamps the
// start, every launch the stop. Outside a window this is a plain hipLaunchKernelGGL.
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
  int launches = 0;
};
inline LaunchTiming& launch_timing() {
  static thread_local LaunchTiming t;
  return t;
}
#define RT_LAUNCH(K, G, B, SH, ST, ...)                                                              \
  do {                                                                                               \
    ::rwkvtts::LaunchTiming& lt_ = ::rwkvtts::launch_timing();                                       \
    if (lt_.stop) {                                                                                  \
      hipExtLaunchKernelGGL(K, G, B, SH, ST, lt_.launches == 0 ? lt_.start : nullptr, lt_.stop, 0u, \
                            __VA_ARGS__);                                                            \
      ++lt_.launches;                                                                                \
    } else {                                                                                         \
      hipLaunchKernelGGL(K, G, B, SH, ST, __VA_ARGS__);                                              \
    }                                                                                                \
  } while (0)

}  // namespace rwkvtts
