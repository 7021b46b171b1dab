# variant: k_gemm_wide stores its partial slabs with plain 16-byte stores (no write-through)
s = open('lm_kernels.hip').read()
a = s.index('void k_gemm_wide(GemmArgs a)'); b = s.index('tl_end(a.tl);', a)
seg = s[a:b]
old = '''      if (a.wt) {'''
assert seg.count(old) == 1
seg = seg.replace(old, '''      if (col + 4 <= Nn && (((uintptr_t)dst) & 15) == 0) {
        *(float4_*)dst = v;
      } else if (a.wt) {''')
s = s[:a] + seg + s[b:]
open('lm_kernels.hip', 'w').write(s)
