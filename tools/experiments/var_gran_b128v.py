# variant: the one-row granule polls as volatile (aux bit 31) 16-byte sc1 buffer loads through a
# wave-uniform buffer resource (two granules per load) instead of one 64-bit atomic load per granule
p = "lm_kernels.hip"
s = open(p).read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a[:60]
    s = s.replace(a, b)
rep('''__device__ inline uint64_t ld_gran(const uint64_t* p) {''', '''__device__ inline u64x2_ ld_gran2(__amdgpu_buffer_rsrc_t r, int off_bytes) {  // volatile sc1 16-byte load
  return __builtin_bit_cast(u64x2_, __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, (int)0x80000010u));
}
__device__ inline uint64_t ld_gran(const uint64_t* p) {''')
rep('''      const uint64_t* zp = sy.zgran + kbeg + 2 * lane;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t q0, q1;
      for (;;) {
        q0 = ld_gran(zp);
        q1 = ld_gran(zp + 1);''', '''      const auto zr = wt_rsrc(sy.zgran);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t q0, q1;
      for (;;) {
        const u64x2_ qq = ld_gran2(zr, (kbeg + 2 * lane) * 8);
        q0 = qq.x;
        q1 = qq.y;''')
rep('''      const uint32_t tag = gran_tag(sy);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool ok = true;''', '''      const uint32_t tag = gran_tag(sy);
      const auto gr = wt_rsrc(sy.gran);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool ok = true;''')
rep('''          const uint64_t* gp = sy.gran + (int64_t)p * sy.gran_ld + kbeg + 4 * lane;
          uint64_t q[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) q[e] = ld_gran(gp + e);''', '''          uint64_t q[4];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const u64x2_ qq = ld_gran2(gr, (p * sy.gran_ld + kbeg + 4 * lane + 2 * e) * 8);
            q[2 * e] = qq.x;
            q[2 * e + 1] = qq.y;
          }''')
open(p, "w").write(s)
