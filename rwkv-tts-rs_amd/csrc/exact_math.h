// exact_math.h -- glibc 2.35 expf restated for host and device (shared by the GPU sampler and
// the host self-test entry point rwkvtts_debug_expf).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace rwkvtts {

__host__ __device__ inline uint64_t exp2_tab(int i) {
  constexpr uint64_t kExp2Tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
  return kExp2Tab[i];
}

// glibc expf for x <= 0 (and NaN / -inf). sysdeps/ieee754/flt-32/e_expf.c algorithm. `tab`:
// the 32-entry 2^(i/32) table (exp2_tab) -- on the device a copy in LDS, so that the per-element
// gather is a conflict-free LDS read instead of a dependent global load.
template <typename Tab>
__host__ __device__ inline float glibc_expf_t(float x, const Tab& tab) {
  if (x == -__builtin_inff()) return 0.0f;
  if (x != x) return x + x;
  if (x < -0x1.9fe368p6f) return 0.0f;  // underflow to +0
  const double xd = (double)x;
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double z = InvLn2N * xd;
  double kd = z + SHIFT;
  const uint64_t ki = __builtin_bit_cast(uint64_t, kd);
  kd -= SHIFT;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  uint64_t t = tab((int)(ki % 32));
  t += ki << (52 - 5);
  const double s = __builtin_bit_cast(double, t);
  const double zz = __builtin_fma(C0, r, C1);
  double y = __builtin_fma(C2, r, 1.0);
  y = __builtin_fma(zz, r * r, y);
  y = y * s;
  return (float)y;
}
__host__ __device__ inline float glibc_expf(float x) {
  return glibc_expf_t(x, [](int i) { return exp2_tab(i); });
}


}  // namespace rwkvtts
