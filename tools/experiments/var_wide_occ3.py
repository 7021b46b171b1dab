# variant: k_gemm_wide at three workgroups per CU (<= 168 VGPRs)
s = open('lm_kernels.hip').read()
old = '__global__ __launch_bounds__(256) void k_gemm_wide(GemmArgs a) {'
assert old in s
s = s.replace(old, '__global__ __launch_bounds__(256, 3) void k_gemm_wide(GemmArgs a) {')
open('lm_kernels.hip', 'w').write(s)
