# variant: an unused kernel emitted ahead of the others (shifts every kernel's code address: does
# code placement alone move the decode step?)
s = open("lm_kernels.hip").read()
a = "namespace rwkvtts {"
assert a in s
i = s.index(a) + len(a)
s = s[:i] + """
__global__ void k_codepad(float* p, int n) {
#pragma unroll
  for (int i = 0; i < 700; ++i) p[(i * 7 + threadIdx.x) % n] += (float)i;
}
""" + s[i:]
open("lm_kernels.hip", "w").write(s)
