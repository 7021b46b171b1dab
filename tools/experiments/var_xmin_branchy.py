# variant: the round-4 X-load form (rows past M clamped to row M-1) in place of af22040's branchy one
import re
s = open("lm_kernels.hip").read()
a = """        const int o = ((xrow0 + r) * ldx + kbeg + k8) * 2;
        vh[u] = vl[u] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
        if (xrow0 + r < a.M) {
          vh[u] = __builtin_bit_cast(short8, ld_sc1_b128(rh, o));
          vl[u] = __builtin_bit_cast(short8, ld_sc1_b128(rl, o));
        }"""
b = """        const int o = (min(xrow0 + r, a.M - 1) * ldx + kbeg + k8) * 2;
        vh[u] = __builtin_bit_cast(short8, ld_sc1_b128(rh, o));
        vl[u] = __builtin_bit_cast(short8, ld_sc1_b128(rl, o));"""
assert a in s; s = s.replace(a, b)
a = """      const int64_t o = (int64_t)(xrow0 + r) * ldx + kbeg + k8;
      vh[u] = vl[u] = (short8){0, 0, 0, 0, 0, 0, 0, 0};
      if (xrow0 + r < a.M) {
        vh[u] = *(const short8*)(Xhi + o);
        vl[u] = *(const short8*)(Xlo + o);
      }"""
b = """      const int64_t o = (int64_t)min(xrow0 + r, a.M - 1) * ldx + kbeg + k8;
      vh[u] = *(const short8*)(Xhi + o);
      vl[u] = *(const short8*)(Xlo + o);"""
assert a in s; s = s.replace(a, b)
a = """          xr[p][u] = (float4_){0.f, 0.f, 0.f, 0.f};
          if (xrow0 + r < a.M)
            xr[p][u] = __builtin_bit_cast(float4_, ld_sc1_b128(rp, ((xrow0 + r) * a.x_ld + kbeg + k4) * 4));"""
b = """          xr[p][u] = __builtin_bit_cast(float4_, ld_sc1_b128(rp, (min(xrow0 + r, a.M - 1) * a.x_ld + kbeg + k4) * 4));"""
assert a in s; s = s.replace(a, b)
a = """        xr[p][u] = (float4_){0.f, 0.f, 0.f, 0.f};
        if (xrow0 + r < a.M)
          xr[p][u] = *(const float4_*)(a.x_part + p * a.x_part_stride + (int64_t)(xrow0 + r) * a.x_ld + kbeg + k4);"""
b = """        xr[p][u] = *(const float4_*)(a.x_part + p * a.x_part_stride + (int64_t)min(xrow0 + r, a.M - 1) * a.x_ld + kbeg + k4);"""
assert a in s; s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
