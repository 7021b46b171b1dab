# debug: the first value workgroups print their staged X row 0 (hi / lo bits of columns 0..3 and
# 64..67) and lane 0's xr sums
s = open("lm_kernels.hip").read()
a = """  __syncthreads();
  const int rg_next = rg + (int)gridDim.z;"""
b = """  __syncthreads();
  if constexpr (ROLE == 2 || ROLE == 7) {
    if (bx < 1 && threadIdx.x == 0 && a.M == 1) {
      const int n = __hip_atomic_fetch_add((gint_t*)(sy.err + 3), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n < 4)
        printf("GRANDBG6 n %d role %d xh %04x %04x %04x %04x xl %04x %04x x64 %04x %04x r1 %04x xr %08x %08x %08x %08x\\n", n, ROLE,
               (int)xh[0], (int)xh[1], (int)xh[2], (int)xh[3], (int)xl[0], (int)xl[1], (int)xh[64], (int)xh[65],
               (int)xh[LD + 0], __builtin_bit_cast(uint32_t, xr[0][0][0]), __builtin_bit_cast(uint32_t, xr[1][0][0]),
               __builtin_bit_cast(uint32_t, xr[2][0][0]), __builtin_bit_cast(uint32_t, xr[3][0][0]));
    }
  }
  const int rg_next = rg + (int)gridDim.z;"""
assert a in s; s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
