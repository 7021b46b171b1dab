# debug: the key workgroups of column tile 0 print their row-0 output (lane 0, first launches)
s = open("lm_kernels.hip").read()
a = """  if (ROLE == 6 && sy.gran) {"""
b = """  if constexpr (ROLE == 6) {
    if (tile == 0 && threadIdx.x == 0) {
      const int n = __hip_atomic_fetch_add((gint_t*)(sy.err + 2), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n < 12)
        printf("GRANDBG5 n %d gran %d split %d out %08x x0 %04x %04x\\n", n, sy.gran ? 1 : 0, split,
               __builtin_bit_cast(uint32_t, result(0, 0)), (int)xh[0], (int)xh[1]);
    }
  }
  if (ROLE == 6 && sy.gran) {"""
assert a in s; s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
