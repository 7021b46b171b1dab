# variant: the granule value role with the 32-row tile and every row staged (its first version)
s = open("lm_kernels.hip").read()
a = "gemm2_body<1, 8, kXRelu2, F16, 4, 0, false, 7>(va, b, 0, sy);"
assert a in s
s = s.replace(a, "gemm2_body<2, 8, kXRelu2, F16, 4, 0, false, 7>(va, b, 0, sy);")
n = s.count("if (ROLE == 7 && xrow0 + ")
assert n == 3, n
s = s.replace("if (ROLE == 7 && xrow0 + ", "if (false && xrow0 + ")
open("lm_kernels.hip", "w").write(s)
