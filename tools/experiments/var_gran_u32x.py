# variant (diagnostic): the value role's granules taken apart as 32-bit vector elements (q.x data,
# q.y tag, q.z data, q.w tag) of the volatile 16-byte loads -- the form that came out miscompiled in
# round 5 with non-volatile loads (data elements 0 and 2 equal): does it hold with volatile loads?
p = "lm_kernels.hip"
s = open(p).read()
a = """          uint64_t q[4];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const u64x2_ qq = ld_gran2(gr, (p * sy.gran_ld + kbeg + 4 * lane + 2 * e) * 8);
            q[2 * e] = qq.x;
            q[2 * e + 1] = qq.y;
          }
          xr[p][0] = (float4_){__builtin_bit_cast(float, (uint32_t)q[0]), __builtin_bit_cast(float, (uint32_t)q[1]),
                               __builtin_bit_cast(float, (uint32_t)q[2]), __builtin_bit_cast(float, (uint32_t)q[3])};
#pragma unroll
          for (int e = 0; e < 4; ++e) ok = ok && (uint32_t)(q[e] >> 32) == tag;"""
b = """          const u32x4_ w0 = __builtin_bit_cast(u32x4_, ld_gran2(gr, (p * sy.gran_ld + kbeg + 4 * lane) * 8));
          const u32x4_ w1 = __builtin_bit_cast(u32x4_, ld_gran2(gr, (p * sy.gran_ld + kbeg + 4 * lane + 2) * 8));
          xr[p][0] = (float4_){__builtin_bit_cast(float, w0.x), __builtin_bit_cast(float, w0.z),
                               __builtin_bit_cast(float, w1.x), __builtin_bit_cast(float, w1.z)};
          ok = ok && w0.y == tag && w0.w == tag && w1.y == tag && w1.w == tag;"""
assert s.count(a) == 1
s = s.replace(a, b)
open(p, "w").write(s)
