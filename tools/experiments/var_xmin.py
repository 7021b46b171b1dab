# variant: persistent-role X loads clamp rows past M to row M-1 (round-4 form) instead of the
# out-of-range offset
s = open("lm_kernels.hip").read()
a = "const int o = xrow0 + r < a.M ? ((xrow0 + r) * ldx + kbeg + k8) * 2 : (int)0x80000000u;"
b = "const int o = (min(xrow0 + r, a.M - 1) * ldx + kbeg + k8) * 2;"
c = "const int o = xrow0 + r < a.M ? ((xrow0 + r) * a.x_ld + kbeg + k4) * 4 : (int)0x80000000u;"
d = "const int o = (min(xrow0 + r, a.M - 1) * a.x_ld + kbeg + k4) * 4;"
assert a in s and c in s
s = s.replace(a, b).replace(c, d)
open("lm_kernels.hip", "w").write(s)
