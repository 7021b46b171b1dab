# debug: the first value workgroups (slab and granule forms) of one-row passes print their first
# output and weight bits (lane 0 of workgroups 0 and 1, the first 8 launches of a run)
s = open("lm_kernels.hip").read()
a = """  if (ROLE == 6 && sy.gran) {"""
b = """  if constexpr (ROLE == 2 || ROLE == 7) {
    if (bx < 2 && threadIdx.x == 0 && a.M == 1) {
      const int n = __hip_atomic_fetch_add((gint_t*)(sy.err + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n < 16)
        printf("GRANDBG4 n %d role %d bx %d out %08x acc %08x %08x b0 %04x b7 %04x\\n", n, ROLE, bx,
               __builtin_bit_cast(uint32_t, result(0, 0)), __builtin_bit_cast(uint32_t, acc_h[0][0]),
               __builtin_bit_cast(uint32_t, acc_l[0][0]), (int)(uint16_t)b[0][0], (int)(uint16_t)b[7][3]);
    }
  }
  if (ROLE == 6 && sy.gran) {"""
assert a in s; s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
