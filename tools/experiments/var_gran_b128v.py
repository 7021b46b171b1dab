# variant: the one-row granule polls as volatile 16-byte sc1 loads (two granules per load) instead of
# one 64-bit atomic load per granule
p = "lm_kernels.hip"
s = open(p).read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a[:60]
    s = s.replace(a, b)
rep('''__device__ inline uint64_t ld_gran(const uint64_t* p) {''', '''__device__ inline u64x2_ ld_gran2(const uint64_t* p) {  // volatile (aux bit 31) sc1 16-byte load
  return __builtin_bit_cast(u64x2_, __builtin_amdgcn_raw_buffer_load_b128(wt_rsrc(p), 0, 0, (int)0x80000010u));
}
__device__ inline uint64_t ld_gran(const uint64_t* p) {''')
rep('''        q0 = ld_gran(zp);
        q1 = ld_gran(zp + 1);''', '''        const u64x2_ qq = ld_gran2(zp);
        q0 = qq.x;
        q1 = qq.y;''')
rep('''          for (int e = 0; e < 4; ++e) q[e] = ld_gran(gp + e);''', '''          for (int e = 0; e < 2; ++e) {
            const u64x2_ qq = ld_gran2(gp + 2 * e);
            q[2 * e] = qq.x;
            q[2 * e + 1] = qq.y;
          }''')
open(p, "w").write(s)
